set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01sw}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_clients.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_dev.log 2>&1 || { tail -40 $OUT/pytest_dev.log; exit 1; }
echo "device tests: $(tail -1 $OUT/pytest_dev.log)"
timeout -k 10 300 python -u scripts/segments_probe.py --sweep --rounds 4 --reps 6 > $OUT/segsweep.jsonl 2> $OUT/segsweep.err || { tail -30 $OUT/segsweep.err; exit 1; }
cut -c1-160 $OUT/segsweep.jsonl
