#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats and
# HBM counters.  Every GPU step has its own time limit; the chain stops at the
# first failure (set -e).  Outputs land in gpurun_out/ (merged back by gpurun).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01}
mkdir -p "$OUT"
echo "[gpu_check] $(date -u +%FT%TZ) start" | tee "$OUT/progress.log"
rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}" >> "$OUT/nproc.txt"

if [[ "${SKIP_TESTS:-0}" != 1 ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  echo "[gpu_check] pytest -m gpu ok" | tee -a "$OUT/progress.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  echo "[gpu_check] smoke ok" | tee -a "$OUT/progress.log"
fi

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "[gpu_check] bench ok: $(cat "$OUT/bench.json")" | tee -a "$OUT/progress.log"

if [[ "${E2E:-0}" == 1 ]]; then
  timeout -k 10 600 python bench.py --e2e --reps 5 > "$OUT/e2e.jsonl" 2> "$OUT/e2e.err"
  echo "[gpu_check] e2e ok" | tee -a "$OUT/progress.log"
fi

if [[ "${SKIP_PROF:-0}" != 1 ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o run \
      -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_stats.log" 2>&1
  echo "[gpu_check] rocprof stats ok" | tee -a "$OUT/progress.log"
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex reduce_ --output-format csv -d "$OUT/prof_fetch" -o run \
      -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_fetch.log" 2>&1
  echo "[gpu_check] rocprof FETCH_SIZE ok" | tee -a "$OUT/progress.log"
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex reduce_ --output-format csv -d "$OUT/prof_write" -o run \
      -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_write.log" 2>&1
  echo "[gpu_check] rocprof WRITE_SIZE ok" | tee -a "$OUT/progress.log"
fi
echo "[gpu_check] $(date -u +%FT%TZ) done" | tee -a "$OUT/progress.log"
