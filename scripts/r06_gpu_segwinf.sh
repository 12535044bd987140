#!/bin/bash
# Round 6: hand-off split windows in production (rows and zero-copy): the
# window/fused/device-round tests, then cfg4 zero-copy under rocprofv3 with
# the hand-off form and with the barrier form (FEDAVG_SEGWINN_BARRIER=1).
set -o pipefail
O=gpurun_out/r06/segwinf
mkdir -p $O
export TMPDIR=/tmp
if [ "$1" != "--skip-tests" ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_window.py \
  tests/test_gpu_fused.py tests/test_gpu_device_round.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/zc_winf -o run -- \
  python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --calls 12 > $O/zc_winf.log 2>&1 || exit $?
FEDAVG_SEGWINN_BARRIER=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/zc_barrier -o run -- \
  python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --calls 12 > $O/zc_barrier.log 2>&1 || exit $?
timeout -k 10 240 python scripts/segwin_layout_probe.py --layout packed --config resnet18_gn --calls 12 > $O/zc_packed.log 2>&1 || exit $?
# keep the stats, drop the per-dispatch traces (the merge back is capped at 64 MiB)
find $O -name '*kernel_trace.csv' -delete
for f in $O/zc_winf.log $O/zc_barrier.log $O/zc_packed.log; do tail -n 1 $f; done
grep -h segwin $O/zc_*/run_kernel_stats.csv
