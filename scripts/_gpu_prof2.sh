set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01p}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/small_stats -o run -- python scripts/small_e2e_probe.py --reps 200 > $OUT/small_stats.log 2>&1
echo small ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dtype_stats -o run -- python scripts/dtype_probe.py > $OUT/dtype_stats.log 2>&1
echo dtype ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex reduce_vec --output-format csv -d $OUT/dtype_fetch -o run -- python scripts/dtype_probe.py > $OUT/dtype_fetch.log 2>&1
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex reduce_vec --output-format csv -d $OUT/dtype_write -o run -- python scripts/dtype_probe.py > $OUT/dtype_write.log 2>&1
echo write ok
