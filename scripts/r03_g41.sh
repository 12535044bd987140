set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g41
mkdir -p $O
# split-row windows (two waves per window, <= 63 rows each) vs the production window kernel and its loads alone
timeout -k 10 300 python -u -m pytest tests/test_gpu_window.py -k split_row -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo tests ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 90x25000000 --variants 80005002,0 80006002,0 61000042,0 --rounds 3 --reps 8 > $O/win2_k100.jsonl 2> $O/win2_k100.err
echo k100 ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 80x25000000 64x10000000 100x6250000 --variants 80004002,0 80005002,0 80003202,0 --rounds 3 --reps 8 > $O/win2_other.jsonl 2> $O/win2_other.err
echo other ok
