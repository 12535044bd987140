#!/bin/bash
# Round 6: the production split windows (hand-off kernel) at cfg5's per-GPU
# slice and cfg4, event-timed and under rocprofv3 --stats; then the
# zero-copy cfg4 device round once more.
set -o pipefail
O=gpurun_out/r06/winf_final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rows -o run -- \
  python scripts/fused_probe.py --shapes 1000x12500000 500x11227812 600x10000000 --variants --rounds 4 --reps 5 \
  > $O/rows.jsonl 2> $O/rows.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/zc -o run -- \
  python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --calls 20 > $O/zc.log 2>&1 || exit $?
find $O -name '*kernel_trace.csv' -delete
cat $O/rows.jsonl
grep -h '^{' $O/zc.log
grep -h "winf\|reduce_f32x4\|sqdist_buf\|finalize" $O/rows/run_kernel_stats.csv $O/zc/run_kernel_stats.csv | cut -c1-60,200-
