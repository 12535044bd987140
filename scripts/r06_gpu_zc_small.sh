#!/bin/bash
# Round 6: zero-copy device rounds at 8-64 clients: the production forms
# (tiles <= 16, one-wave windows 17-128) against the split windows
# (FEDAVG_SEG_SPLIT_MIN_K=2), resnet18_gn-shaped clients.
set -o pipefail
O=gpurun_out/r06/zc_small
mkdir -p $O
export TMPDIR=/tmp
for K in 8 10 16 32 64; do
  timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 12 > $O/prod_k$K.log 2>&1 || exit $?
  FEDAVG_SEG_SPLIT_MIN_K=2 timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 12 > $O/split_k$K.log 2>&1 || exit $?
done
for K in 8 10 16 32 64; do echo "K=$K prod $(grep -h '^{' $O/prod_k$K.log | cut -c90-150) | split $(grep -h '^{' $O/split_k$K.log | cut -c90-150)"; done
