#!/bin/bash
# HBM traffic and rocprofv3 time of the prefetching split windows (1000 x
# 12.5M and 352 x 5M): FETCH_SIZE and WRITE_SIZE in passes of their own.
set -o pipefail
O=gpurun_out/r05/g52
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sh in 1000x12500000 352x5000000; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex winn --output-format csv -d $O/fetch_$sh -o run -- \
    python scripts/fused_probe.py --shapes $sh --variants --rounds 1 --reps 2 > $O/fetch_$sh.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex winn --output-format csv -d $O/write_$sh -o run -- \
    python scripts/fused_probe.py --shapes $sh --variants --rounds 1 --reps 2 > $O/write_$sh.log 2>&1 || exit $?
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$sh -o run -- \
    python scripts/fused_probe.py --shapes $sh --variants --rounds 2 --reps 4 > $O/stats_$sh.log 2>&1 || exit $?
  find $O/stats_$sh -name "*kernel_trace.csv" -delete
done
