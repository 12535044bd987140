set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g34
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_device_clients.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo tests ok
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/fused_segments_probe.py --configs flat flatk90 flatk80 resnet18_gn_k100 resnet56 femnist_cnn --reps 8 > $O/segwin_on.jsonl 2> $O/segwin_on.err
echo on ok
FEDAVG_SEGWIN=0 timeout -k 10 300 python -u scripts/fused_segments_probe.py --configs flat flatk90 flatk80 resnet18_gn_k100 resnet56 femnist_cnn --reps 8 > $O/segwin_off.jsonl 2> $O/segwin_off.err
echo off ok
