set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g17
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_fused.py -x -v --timeout 200 --timeout-method thread > $O/pytest_win.log 2>&1
echo win tests ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 90x25000000 128x8000000 48x20833333 --variants 64,0 --rounds 3 --reps 6 > $O/prod_probe.jsonl 2> $O/prod_probe.err
echo probe ok
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fused -o run -- python scripts/fused_probe.py --shapes 100x25000000 --variants --rounds 2 --reps 6 > $O/prof_fused.log 2>&1
echo prof ok
