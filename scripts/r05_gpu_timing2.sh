#!/usr/bin/env bash
# Round 5, GPU session 4: attached-event spans in bench.py against rocprofv3
# (N = 1 and the N = 8 per-rank chunk shapes), resnet56-like streaming :217.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g4}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
summ() { python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric')][0]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['frac'],r['avg_launch_ms'],d.get('clock_mhz'))" "$1"; }
log start
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_n1_$i.json" 2> "$OUT/bench_n1_$i.err"
  log "bench n1 #$i: $(summ "$OUT/bench_n1_$i.json")"
done
for SC in "8 4" "8 2" "4 4" "2 8" "8 8"; do
  set -- $SC
  timeout -k 10 180 python bench.py --shard-of $1 --chunks $2 --no-cpu-baseline > "$OUT/bench_s$1_c$2.json" 2> "$OUT/bench_s$1_c$2.err"
  log "bench shard-of $1 chunks $2: $(summ "$OUT/bench_s$1_c$2.json")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
    -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_n1.log" 2>&1
log "rocprof n1: $(summ "$OUT/prof_n1.log")"
for SC in "8 4" "8 2"; do
  set -- $SC
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_s$1_c$2" -o run \
      -- python bench.py --shard-of $1 --chunks $2 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_s$1_c$2.log" 2>&1
  log "rocprof s$1 c$2: $(summ "$OUT/prof_s$1_c$2.log")"
done
timeout -k 10 300 python -u scripts/stream_install_probe.py --K 100 --P 600372 --keys 350 --rounds 8 --no-plain > "$OUT/stream_resnet56like.jsonl" 2> "$OUT/stream_resnet56like.err"
log "resnet56-like streaming ok: $(tail -1 "$OUT/stream_resnet56like.jsonl" | cut -c1-300)"
log done
