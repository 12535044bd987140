#!/bin/bash
# Round 6: per-wave s_memtime timeline of the split-row window kernel.
set -o pipefail
O=gpurun_out/r06/timeline
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/winn_timeline.py --shapes 1000x12500000 500x11227812 \
  --codes 88800008 88800016 88800000 --out $O/stamps.npz > $O/timeline.jsonl 2> $O/timeline.err || exit $?
cat $O/timeline.jsonl
