set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01w}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 300 python scripts/small_e2e_probe.py > $OUT/small.jsonl 2> $OUT/small.err
cat $OUT/small.jsonl
timeout -k 10 600 python bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err
cat $OUT/e2e.jsonl
