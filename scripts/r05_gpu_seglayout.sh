#!/bin/bash
# cfg4 (resnet18_gn x 500) device round: the zero-copy split windows on three
# client layouts against the packed rows' fused pass (rocprofv3 kernel stats).
set -o pipefail
O=gpurun_out/r05/g55
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in separate arena packed; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$L -o run -- \
    python scripts/segwin_layout_probe.py --layout $L --config resnet18_gn --calls 12 > $O/$L.log 2>&1 || exit $?
  find $O/$L -name "*kernel_trace.csv" -delete
done
