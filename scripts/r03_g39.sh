set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g39
mkdir -p $O
C="flat70x600000 flat70x3000000 flat90x1000000 flat90x3000000 flat80x400000 flat100x3000000 flat40x3000000 flat120x3000000"
FEDAVG_SEGWIN=0 timeout -k 10 300 python -u scripts/fused_segments_probe.py --configs $C --reps 8 > $O/seg_tiles.jsonl 2> $O/seg_tiles.err
echo tiles ok
FEDAVG_SEGWIN=2 timeout -k 10 300 python -u scripts/fused_segments_probe.py --configs $C --reps 8 > $O/seg_win.jsonl 2> $O/seg_win.err
echo win ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 70x600000 90x400000 96x1500000 80x3000000 --variants 64,0 --rounds 3 --reps 8 > $O/plan.jsonl 2> $O/plan.err
echo plan ok
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_fused.py tests/test_gpu_device_clients.py tests/test_gpu_model_shapes.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
