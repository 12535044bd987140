#!/bin/bash
# Round 6: the split-row windows with 128 rows per wave (8 waves, 2 per SIMD,
# deep prefetch) against the production 64-row form, at the shapes the
# drop-in sends to them (513-1024 clients) and at cfg4's 500.
set -o pipefail
O=gpurun_out/r06/winn128
mkdir -p $O
export TMPDIR=/tmp
V="87000816,0 89000008,0 89001608,0 89003208,0 89004808,0 89006408,0 89008008,0"
timeout -k 10 600 python scripts/fused_probe.py --shapes 1000x12500000 600x10000000 513x10000000 \
  --variants $V --rounds 3 --reps 3 > $O/probe.jsonl 2> $O/probe.err || exit $?
timeout -k 10 600 python scripts/fused_probe.py --shapes 500x11227812 400x10000000 \
  --variants 87000808,0 89000008,0 89003208,0 89006408,0 --rounds 3 --reps 3 > $O/probe_k500.jsonl 2> $O/probe_k500.err || exit $?
echo done
