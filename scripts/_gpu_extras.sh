# FPF kernel profile, dtype throughput probes and the host-consumer bench (after gpu_check.sh).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01t}; mkdir -p $OUT
timeout -k 10 300 python bench.py --fpf > $OUT/fpf.jsonl 2> $OUT/fpf.err
cat $OUT/fpf.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fpf -o fpf -- python bench.py --fpf --legs hip > $OUT/fpf_prof.log 2>&1
find $OUT/prof_fpf -name '*kernel_stats.csv' -exec cp {} $OUT/fpf_kernel_stats.csv \;
cut -d, -f1-8 $OUT/fpf_kernel_stats.csv
timeout -k 10 300 python bench.py --host-out --no-cpu-baseline > $OUT/bench_host_out.json 2> $OUT/bench_host_out.err
cat $OUT/bench_host_out.json
timeout -k 10 300 python scripts/dtype_probe.py 100 25000000 > $OUT/dtype_probe.jsonl 2> $OUT/dtype_probe.err
cat $OUT/dtype_probe.jsonl
timeout -k 10 300 python scripts/dtype_probe.py 500 11227812 > $OUT/dtype_probe_k500.jsonl 2>> $OUT/dtype_probe.err
cat $OUT/dtype_probe_k500.jsonl
