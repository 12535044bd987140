#!/usr/bin/env bash
# Round 5, GPU session 2: the sharded finish's host phases (default and more
# hardware queues), resnet56-like streaming :217 with the version-counter
# check, short-launch timing methods against rocprofv3's kernel trace.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g2}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
timeout -k 10 300 python -u scripts/sharded_session_probe.py --shards 1,2,4,8 --rounds 3 > "$OUT/session_default.jsonl" 2> "$OUT/session_default.err"
log "session probe (default queues) ok"
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u scripts/sharded_session_probe.py --shards 8 --rounds 3 > "$OUT/session_hwq16.jsonl" 2> "$OUT/session_hwq16.err"
log "session probe (16 queues) ok"
timeout -k 10 300 python -u scripts/stream_install_probe.py --K 100 --P 600372 --keys 350 --rounds 8 --no-plain > "$OUT/stream_resnet56like.jsonl" 2> "$OUT/stream_resnet56like.err"
log "resnet56-like streaming ok: $(tail -1 "$OUT/stream_resnet56like.jsonl" | cut -c1-300)"
for SC in "8 4" "8 2" "4 8" "2 8" "8 1"; do
  set -- $SC
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lt_s$1_c$2" -o run \
      -- python scripts/launch_timing_probe.py --shard-of $1 --chunks $2 --calls 200 > "$OUT/lt_s$1_c$2.log" 2>&1
  log "launch timing shard-of $1 chunks $2 ok"
done
log done
