#!/bin/bash
# Round 6: zero-copy split windows with power-of-two workgroups per CU:
# device-round tests, then the client-count sweep against the rows kernel.
set -o pipefail
O=gpurun_out/r06/zc_check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_device_round.py \
  tests/test_gpu_device_clients.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for K in 129 160 200 257 300 384 500; do
  timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 10 > $O/sep_k$K.log 2>&1 || exit $?
done
grep -h '^{' $O/sep_k*.log | cut -c1-160
