set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01dev}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_clients.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_dev.log 2>&1 || { tail -40 $OUT/pytest_dev.log; exit 1; }
echo "device-client tests: $(tail -1 $OUT/pytest_dev.log)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
