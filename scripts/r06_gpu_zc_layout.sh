#!/bin/bash
# Round 6: is the zero-copy split windows' gap to the rows kernel at 129-257
# clients the layout (many allocations) or the kernel's addressing?
set -o pipefail
O=gpurun_out/r06/zc_layout
mkdir -p $O
export TMPDIR=/tmp
for K in 129 257 500; do
  for L in separate arena shuffled; do
    timeout -k 10 240 python scripts/segwin_layout_probe.py --layout $L --config resnet18_gn --clients $K --calls 10 > $O/${L}_k$K.log 2>&1 || exit $?
  done
done
grep -h '^{' $O/*.log | cut -c1-150
