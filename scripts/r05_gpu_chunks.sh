#!/usr/bin/env bash
# Round 5: the streaming finish at the target vs the D2H chunking (count, min width)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g43}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
for cfg in 8:2097152 16:1048576 12:1048576 32:524288; do
  n=${cfg%%:*}; m=${cfg##*:}
  FEDAVG_D2H_MAX_CHUNKS=$n FEDAVG_D2H_CHUNK_MIN_COLS=$m timeout -k 10 240 python -u scripts/stream_probe.py --rounds 6 \
      > "$OUT/chunks_$n.jsonl" 2> "$OUT/chunks_$n.err"
  log "chunks=$n: $(python -c "
import json,sys
f=[json.loads(l)['finish_ms'] for l in open(sys.argv[1]) if l.startswith('{')]
print(sorted(f[2:]), 'median', sorted(f[2:])[len(f[2:])//2])" "$OUT/chunks_$n.jsonl")"
done
log done
