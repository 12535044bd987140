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
timeout -k 10 500 python -u scripts/fused_probe.py --shapes 500x11227812 1000x12500000 320x5000000 256x8000000 150x10000000 --variants 200032,0 1800032,0 3400032,0 1800064,0 --rounds 2 --reps 4 > $O/many_clients.jsonl 2> $O/many_clients.err
echo many ok
