set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_autostream.py -x -v --timeout 120 --timeout-method thread > $O/autostream.log 2>&1
echo autostream ok
timeout -k 10 200 python -u scripts/stream_install_probe.py --K 10 --P 7850 --keys 2 --rounds 30 --delay-ms 1 > $O/stream_mnist.jsonl 2> $O/stream_mnist.err
echo mnist ok
tail -1 $O/stream_mnist.jsonl
