#!/bin/bash
# Split-row windows with the next window's first rows prefetched: parity
# tests, the depth sweep (rows) and the zero-copy A/B (FEDAVG_SPLIT_PREFETCH).
set -o pipefail
O=gpurun_out/r05/g47
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_window.py tests/test_gpu_fused.py tests/test_gpu_device_round.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python scripts/fused_probe.py --shapes 1000x12500000 640x3000000 500x11227812 384x5000000 352x5000000 300x5000000 \
  --variants 85160641,0 87000216,0 87000416,0 87000616,0 87000816,0 87001016,0 87001216,0 85080641,0 87000408,0 87000808,0 87001208,0 \
  --rounds 5 --reps 4 > $O/pf.jsonl 2> $O/pf.err || exit $?
for pf in 0 1; do
  if [ $pf = 0 ]; then export FEDAVG_SPLIT_PREFETCH=0; else unset FEDAVG_SPLIT_PREFETCH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seg_pf$pf -o run -- \
    python scripts/host_cost_probe.py --configs resnet18_gn --rounds 12 > $O/seg_pf$pf.jsonl 2> $O/seg_pf$pf.err || exit $?
  find $O/seg_pf$pf -name "*kernel_trace.csv" -delete
done
