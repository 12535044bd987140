#!/usr/bin/env bash
# Round 5, GPU session 1: sharded streaming parity + probes, bench with the
# shader clock, PMC traffic at every per-rank chunk geometry the N>1 sweep can
# pick.  Each GPU step has its own limit; the chain stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g1}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
if [[ "${SKIP_TESTS:-0}" != 1 ]]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_autostream.py -x -v \
      --timeout 300 --timeout-method thread > "$OUT/pytest_multi_stream.log" 2>&1
  log "pytest multi+autostream ok: $(tail -1 "$OUT/pytest_multi_stream.log")"
fi
if [[ "${SKIP_PROBES:-0}" != 1 ]]; then
  timeout -k 10 300 python -u scripts/multi_device_probe.py --pack-threads 8,16,32,64,128 --skip-dropin --reps 3 \
      > "$OUT/pack_threads.jsonl" 2> "$OUT/pack_threads.err"
  log "pack threads ok"
  timeout -k 10 600 python -u scripts/stream_install_probe.py --shards 1,2,8 --rounds 4 --delay-ms 20 \
      > "$OUT/stream_shards.jsonl" 2> "$OUT/stream_shards.err"
  log "stream shards ok: $(tail -1 "$OUT/stream_shards.jsonl")"
fi
if [[ "${SKIP_BENCH:-0}" != 1 ]]; then
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  log "bench ok: $(cut -c1-300 "$OUT/bench.json")"
fi
if [[ "${SKIP_PMC:-0}" != 1 ]]; then
  for N in ${PMC_N:-2 4 8}; do
    for C in ${PMC_C:-1 2 4 8}; do
      for CTR in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-include-regex reduce_ --output-format csv \
            -d "$OUT/pmc_s${N}_c${C}_${CTR}" -o run -- python bench.py --shard-of $N --chunks $C --steps 4 \
            --warmup 1 --no-cpu-baseline > "$OUT/pmc_s${N}_c${C}_${CTR}.log" 2>&1
      done
      log "pmc shard-of $N chunks $C ok"
    done
  done
fi
log done
