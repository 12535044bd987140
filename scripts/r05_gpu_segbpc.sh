#!/bin/bash
# Zero-copy split windows at 257-320 clients (5 waves per workgroup): resident
# workgroups per CU capped by FEDAVG_SEGWINN_PER_CU (probe).
set -o pipefail
O=gpurun_out/r05/g59
mkdir -p $O
export TMPDIR=/tmp
for b in 0 3; do
  export FEDAVG_SEGWINN_PER_CU=$b
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b$b -o run -- \
    python scripts/host_cost_probe.py --configs flat_260x8m flat_300x5m flat_320x3m resnet18_gn --rounds 8 > $O/b$b.jsonl 2> $O/b$b.err || exit $?
  find $O/b$b -name "*kernel_trace.csv" -delete
done
