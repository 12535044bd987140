#!/usr/bin/env bash
# Round 5: where a resnet56-like streamed round's :217 goes (verify_rows' native
# phases, the finish's host phases), at 16 and 8 intra-op threads.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g9}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
timeout -k 10 300 python -u scripts/stream_install_probe.py --K 100 --P 600372 --keys 350 --rounds 10 --no-plain > "$OUT/stream_resnet56like_t16.jsonl" 2> "$OUT/s16.err"
log "t16: $(tail -1 "$OUT/stream_resnet56like_t16.jsonl" | cut -c1-300)"
OMP_NUM_THREADS=8 timeout -k 10 300 python -u scripts/stream_install_probe.py --K 100 --P 600372 --keys 350 --rounds 10 --no-plain > "$OUT/stream_resnet56like_t8.jsonl" 2> "$OUT/s8.err"
log "t8: $(tail -1 "$OUT/stream_resnet56like_t8.jsonl" | cut -c1-300)"
log done
