set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo tests ok
timeout -k 10 400 python -u scripts/fused_probe.py --shapes 100x25000000 --variants 64,0 200064,0 200128,0 200256,0 210128,0 210256,0 300064,0 310128,0 310256,0 400064,0 410128,0 410256,0 100064,0 --rounds 3 --reps 6 > $O/fused_rs.jsonl 2> $O/fused_rs.err
echo probe1 ok
timeout -k 10 400 python -u scripts/fused_probe.py --shapes 20x25000000 64x10000000 200x10000000 300x5000000 10x1206590 100x600372 --variants 200032,0 200064,0 200128,0 200256,0 --rounds 3 --reps 6 > $O/fused_rs_shapes.jsonl 2> $O/fused_rs_shapes.err
echo probe2 ok
