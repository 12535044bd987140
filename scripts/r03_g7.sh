set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo gpu tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_stats.log 2>&1
echo stats ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex reduce_ --output-format csv -d $O/prof_fetch -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_fetch.log 2>&1
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex reduce_ --output-format csv -d $O/prof_write -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_write.log 2>&1
echo write ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg4_stats -o run -- python scripts/fused_probe.py --shapes 500x11227812 --variants --rounds 2 --reps 4 > $O/cfg4_stats.log 2>&1
echo cfg4 stats ok
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex reduce_sqdist --output-format csv -d $O/cfg4_fetch -o run -- python scripts/fused_probe.py --shapes 500x11227812 --variants --rounds 1 --reps 2 > $O/cfg4_fetch.log 2>&1
echo cfg4 fetch ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 --variants 300064,0 5300064,0 5310128,0 5310256,0 310128,0 --rounds 3 --reps 6 > $O/wide_loads.jsonl 2> $O/wide_loads.err
echo wide ok
