set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/prof_fused
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python scripts/fused_probe.py --shapes 100x25000000 --variants --rounds 2 --reps 5 > $O/stats.log 2>&1
echo stats ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python scripts/fused_probe.py --shapes 100x25000000 --variants --rounds 1 --reps 2 > $O/fetch.log 2>&1
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python scripts/fused_probe.py --shapes 100x25000000 --variants --rounds 1 --reps 2 > $O/write.log 2>&1
echo write ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seg_stats -o run -- python scripts/fused_segments_probe.py --configs flat --reps 5 > $O/seg_stats.log 2>&1
echo seg stats ok
