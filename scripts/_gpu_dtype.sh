set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01q}; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 300 python scripts/dtype_probe.py 100 25000000 > $OUT/dtype_probe.jsonl 2> $OUT/dtype_probe.err
cat $OUT/dtype_probe.jsonl
timeout -k 10 300 python scripts/dtype_probe.py 500 11227812 > $OUT/dtype_probe_k500.jsonl 2>> $OUT/dtype_probe.err
cat $OUT/dtype_probe_k500.jsonl
