set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g46
mkdir -p $O
# the gpu config tests including cfg5 at full size (200 GB resident, two passes), then the whole suite
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $O/pytest_configs.log 2>&1
echo configs ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo gpu tests ok
tail -2 $O/pytest_gpu.log
