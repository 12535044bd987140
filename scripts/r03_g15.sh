set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g15
mkdir -p $O
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 97x25000000 100x1000003 100x600372 --variants 64,0 60000042,0 60000012,0 61000042,0 61000044,0 --rounds 3 --reps 6 > $O/win_probe.jsonl 2> $O/win_probe.err
echo probe ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo gpu tests ok
tail -3 $O/pytest_gpu.log
