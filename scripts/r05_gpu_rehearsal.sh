#!/usr/bin/env bash
# Round 5: the N > 1 bench path (deferred all-gathers, span timing, chunk
# sweep, parity, CPU baseline) rehearsed with 8 gloo ranks on cuda:0.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g8}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 900 python bench.py --gpus 8 --steps 10 --warmup 3 \
    > "$OUT/rehearsal_gloo8.json" 2> "$OUT/rehearsal_gloo8.err"
log "gloo8 rehearsal: $(cut -c1-400 "$OUT/rehearsal_gloo8.json")"
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
    > "$OUT/rehearsal_gloo2.json" 2> "$OUT/rehearsal_gloo2.err"
log "gloo2 rehearsal: $(cut -c1-400 "$OUT/rehearsal_gloo2.json")"
log done
