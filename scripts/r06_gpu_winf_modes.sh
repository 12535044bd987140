#!/bin/bash
# Round 6: hand-off split windows, probe modes: tight polls (1), no priorities
# (2), no turn priority (4), prefetch 24/32; timeline of the tight-poll form.
set -o pipefail
O=gpurun_out/r06/winf_modes
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python scripts/fused_probe.py --shapes 1000x12500000 600x10000000 \
  --variants 91001616,0 91011616,0 91021616,0 91041616,0 91002416,0 91003216,0 --rounds 4 --reps 3 > $O/probe16.jsonl 2> $O/probe16.err || exit $?
timeout -k 10 400 python scripts/fused_probe.py --shapes 500x11227812 400x10000000 \
  --variants 91000808,0 91010808,0 91020808,0 91011608,0 91001608,0 --rounds 4 --reps 3 > $O/probe8.jsonl 2> $O/probe8.err || exit $?
timeout -k 10 300 python scripts/winn_timeline.py --shapes 1000x12500000 --codes 91081616 91091616 > $O/timeline.jsonl 2> $O/timeline.err || exit $?
grep -v two-pass $O/probe16.jsonl $O/probe8.jsonl | cut -c1-200
cat $O/timeline.jsonl
