#!/usr/bin/env bash
# Round 5: tile kernel cost per key -- resnet56 (350 keys) against the same
# fp32 bytes as one key, tiles forced (and windows for the flat one).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g13}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
for CFG in resnet56 resnet56_flat; do
  for L in separate packed; do
    FEDAVG_SEGWIN_MIN_PER_WAVE=1000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t_${CFG}_$L" -o run \
        -- python scripts/segwin_layout_probe.py --layout $L --config $CFG --calls 30 > "$OUT/t_${CFG}_$L.log" 2>&1
    find "$OUT/t_${CFG}_$L" -name "*kernel_trace.csv" -delete
    log "$CFG $L: $(grep -h '"layout"' "$OUT/t_${CFG}_$L.log" | cut -c1-250)"
  done
done
log done
