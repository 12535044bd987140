#!/usr/bin/env bash
# Round 5, GPU session 3: the span timing in bench.py against rocprofv3 at
# N = 1 and the per-rank chunk shapes; the deferred-gather step (world-size-1
# RCCL); resnet56-like streaming :217 with fed-key identity.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g3}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
log "pytest ok: $(tail -1 "$OUT/pytest.log")"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err"
log "bench n1: $(python -c "import json;d=json.load(open('$OUT/bench_n1.json'));r=d['roofline'];print(d['value'],r['frac'],r['avg_launch_ms'],d.get('clock_mhz'))")"
for SC in "8 4" "8 2" "4 4" "2 8"; do
  set -- $SC
  timeout -k 10 180 python bench.py --shard-of $1 --chunks $2 --no-cpu-baseline > "$OUT/bench_s$1_c$2.json" 2> "$OUT/bench_s$1_c$2.err"
  log "bench shard-of $1 chunks $2: $(python -c "import json;d=json.load(open('$OUT/bench_s$1_c$2.json'));r=d['roofline'];print(d['value'],r['frac'],r['avg_launch_ms'],d.get('clock_mhz'))")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
    -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_n1.log" 2>&1
log "rocprof n1 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_s8_c4" -o run \
    -- python bench.py --shard-of 8 --chunks 4 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_s8_c4.log" 2>&1
log "rocprof s8c4 ok"
timeout -k 10 300 python bench.py --force-gather --chunks 4 --no-cpu-baseline > "$OUT/bench_gather_ws1_c4.json" 2> "$OUT/bench_gather_ws1_c4.err"
log "bench force-gather ws1 c4: $(cut -c1-200 "$OUT/bench_gather_ws1_c4.json")"
timeout -k 10 300 python -u scripts/stream_install_probe.py --K 100 --P 600372 --keys 350 --rounds 8 --no-plain > "$OUT/stream_resnet56like.jsonl" 2> "$OUT/stream_resnet56like.err"
log "resnet56-like streaming ok: $(tail -1 "$OUT/stream_resnet56like.jsonl" | cut -c1-300)"
log done
