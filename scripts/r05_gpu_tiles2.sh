#!/usr/bin/env bash
# Round 5: the tile kernel's LDS client addresses (LADDR) -- parity tests, then
# resnet56 x 100 device rounds A/B (LADDR on/off) and the rows kernel on the
# same bytes, rocprofv3 kernel stats only.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g12}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_round.py tests/test_gpu_device_clients.py tests/test_gpu_window.py tests/test_gpu_fpf.py -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
log "pytest ok: $(tail -1 "$OUT/pytest.log")"
for LA in 1 0; do
  for CFG in resnet56 femnist_cnn; do
    FEDAVG_SEG_LADDR=$LA timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t_${CFG}_la$LA" -o run \
        -- python scripts/segwin_layout_probe.py --layout separate --config $CFG --calls 30 > "$OUT/t_${CFG}_la$LA.log" 2>&1
    find "$OUT/t_${CFG}_la$LA" -name "*kernel_trace.csv" -delete
    log "$CFG laddr=$LA: $(grep -h '"layout"' "$OUT/t_${CFG}_la$LA.log" | cut -c1-250)"
  done
done
log done
