#!/usr/bin/env bash
# Round 5: resnet56 x 100 device round -- the fused tile kernel against the
# rows kernel on the same bytes (packed layout), rocprofv3 kernel stats only.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g11}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
for L in ${LAYOUTS:-separate packed}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t_$L" -o run \
      -- python scripts/segwin_layout_probe.py --layout $L --config resnet56 --calls 30 > "$OUT/t_$L.log" 2>&1
  find "$OUT/t_$L" -name "*kernel_trace.csv" -delete
  log "resnet56 $L: $(grep -h '"layout"' "$OUT/t_$L.log" | cut -c1-300)"
done
log done
