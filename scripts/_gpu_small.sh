set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01o}; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 300 python scripts/small_shapes.py > $OUT/small_shapes.jsonl 2> $OUT/small_shapes.err
cat $OUT/small_shapes.jsonl
