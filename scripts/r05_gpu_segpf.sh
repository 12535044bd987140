#!/bin/bash
# Zero-copy split windows with the same-key prefetch: device-round parity,
# then rocprofv3 kernel stats with the prefetch off and on.  (The measured
# form was not adopted -- DESIGN §5 -- so in the current tree the switch only
# reaches the packed-row kernel and this A/B compares two equal runs.)
set -o pipefail
O=gpurun_out/r05/g51
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_device_round.py tests/test_gpu_window.py > $O/pytest.log 2>&1 || exit $?
for pf in 0 1; do
  if [ $pf = 0 ]; then export FEDAVG_SPLIT_PREFETCH=0; else unset FEDAVG_SPLIT_PREFETCH; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seg_pf$pf -o run -- \
    python scripts/host_cost_probe.py --configs resnet18_gn flat_640x3m flat_1000x5m flat_300x5m --rounds 8 > $O/seg_pf$pf.jsonl 2> $O/seg_pf$pf.err || exit $?
  find $O/seg_pf$pf -name "*kernel_trace.csv" -delete
done
