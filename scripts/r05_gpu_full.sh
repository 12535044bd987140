#!/usr/bin/env bash
# Round 5: the full GPU gate (pytest -m gpu, smoke, bench) plus the resnet56
# device round's kernel forms (tiles vs windows at min-per-wave 1).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g7}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
if [[ "${SKIP_TESTS:-0}" != 1 ]]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  log "pytest -m gpu ok: $(tail -1 "$OUT/pytest_gpu.log")"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  log "smoke ok: $(tail -1 "$OUT/smoke.log")"
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  log "bench ok: $(cut -c1-200 "$OUT/bench.json")"
fi
for MPW in 16 1; do
  for L in separate packed; do
    FEDAVG_SEGWIN_MIN_PER_WAVE=$MPW timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/r56_${L}_mpw$MPW" -o run -- python scripts/segwin_layout_probe.py --layout $L --config resnet56 --calls 30 \
        > "$OUT/r56_${L}_mpw$MPW.log" 2>&1
    find "$OUT/r56_${L}_mpw$MPW" -name "*kernel_trace.csv" -delete  # 35,000 copies per run: over the 64 MiB merge cap
    log "resnet56 $L mpw=$MPW: $(grep -h '"layout"' "$OUT/r56_${L}_mpw$MPW.log" | cut -c1-300)"
  done
done
log done
