#!/bin/bash
# Round 6: split-row windows with the chain's weights by DPP broadcast and a
# hand-pipelined mul/add chain (MODE 16), against production; timeline stamps
# (MODE 8 / 24).
set -o pipefail
O=gpurun_out/r06/bcast
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/winn_timeline.py --shapes 1000x12500000 500x11227812 \
  --codes 88800008 90400008 > $O/timeline.jsonl 2> $O/timeline.err || exit $?
timeout -k 10 600 python scripts/fused_probe.py --shapes 1000x12500000 500x11227812 600x10000000 400x10000000 \
  --variants 87000816,0 89600008,0 89600016,0 --rounds 3 --reps 3 > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/timeline.jsonl $O/probe.jsonl
