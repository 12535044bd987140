#!/bin/bash
# Round 6: zero-copy split windows below 160 clients (FEDAVG_SEG_SPLIT_MIN_K)
# against the tiles / one-wave windows, resnet18_gn-shaped clients.
set -o pipefail
O=gpurun_out/r06/seg129
mkdir -p $O
export TMPDIR=/tmp
for K in 100 120 129 140 150; do
  timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 12 > $O/zc_tiles_k$K.log 2>&1 || exit $?
  FEDAVG_SEG_SPLIT_MIN_K=2 timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 12 > $O/zc_split_k$K.log 2>&1 || exit $?
done
for K in 100 120 129 140 150; do echo "K=$K tiles/windows: $(grep -h '^{' $O/zc_tiles_k$K.log | cut -c80-160)  split: $(grep -h '^{' $O/zc_split_k$K.log | cut -c80-160)"; done
