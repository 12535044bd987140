#!/bin/bash
# Round 6: timelines of the zero-copy and the rows hand-off kernels at the same
# client counts (resnet18_gn-sized rows).
set -o pipefail
O=gpurun_out/r06/zc_timeline
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/zc_timeline.py --clients 129 257 500 > $O/zc.jsonl 2> $O/zc.err || { tail -5 $O/zc.err; exit 1; }
timeout -k 10 300 python scripts/winn_timeline.py --nsmax 8 --shapes 129x11227812 257x11227812 500x11227812 \
  --codes 91080808 > $O/rows.jsonl 2> $O/rows.err || { tail -5 $O/rows.err; exit 1; }
cat $O/zc.jsonl $O/rows.jsonl
