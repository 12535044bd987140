set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_autostream.py tests/test_gpu_model_shapes.py tests/test_gpu_parity.py -k "autostream or side_stream or session or model" -x -q --timeout 150 --timeout-method thread > $O/pytest_new.log 2>&1
echo tests ok
timeout -k 10 400 python -u scripts/stream_install_probe.py --rounds 4 > $O/stream_install.jsonl 2> $O/stream_install.err
echo stream ok
timeout -k 10 400 python -u scripts/stream_install_probe.py --rounds 3 --keys 350 --P 600372 > $O/stream_install_resnet56like.jsonl 2> $O/stream_install_r56.err
echo stream2 ok
