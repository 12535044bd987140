#!/usr/bin/env bash
# Round 5, GPU session 5: the zero-copy window kernel's descriptor table
# (DESC) -- parity tests, then A/B against the pointer form under rocprofv3
# on the 100 x 25M device round (separate allocations and one arena).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g5}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_round.py tests/test_gpu_window.py tests/test_gpu_device_clients.py -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
log "pytest ok: $(tail -1 "$OUT/pytest.log")"
for L in ${LAYOUTS:-separate arena}; do
  for D in 1 0; do
    FEDAVG_SEGWIN_DESC=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sw_${L}_desc$D" -o run \
        -- python scripts/segwin_layout_probe.py --layout $L --config target_flat --calls 20 > "$OUT/sw_${L}_desc$D.log" 2>&1
    log "segwin $L desc=$D: $(grep -h '"layout"' "$OUT/sw_${L}_desc$D.log" | cut -c1-250)"
  done
done
log done
