#!/bin/bash
# Split-row windows with prefetch: where they take over from the register-
# staged tiles (rows), and the zero-copy A/B at 640 and 1000 clients.
set -o pipefail
O=gpurun_out/r05/g49
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python scripts/fused_probe.py --shapes 140x5000000 170x5000000 192x5000000 224x5000000 240x5000000 270x5000000 290x5000000 310x5000000 368x5000000 200x1206590 300x1500000 256x12000000 \
  --variants 87000808,0 87000808,2 87000808,3 87000808,4 87000808,5 \
  --rounds 5 --reps 4 > $O/cross.jsonl 2> $O/cross.err || exit $?
