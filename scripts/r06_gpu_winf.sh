#!/bin/bash
# Round 6: split-row windows with point-to-point hand-offs (winf) against the
# barrier form with broadcast weights (winn MODE 16) and production.
set -o pipefail
O=gpurun_out/r06/winf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/winn_timeline.py --shapes 1000x12500000 500x11227812 \
  --codes 90400008 91080816 > $O/timeline.jsonl 2> $O/timeline.err || exit $?
cat $O/timeline.jsonl
timeout -k 10 600 python scripts/fused_probe.py --shapes 1000x12500000 500x11227812 999x10000003 600x10000000 513x3000001 400x10000000 370x5000000 \
  --variants 87000816,0 89600016,0 91000816,0 91001616,0 91000808,0 91001608,0 --rounds 3 --reps 3 > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/probe.jsonl
