#!/bin/bash
# Round 6: zero-copy split windows with uniform row loads (ragged windows
# through the same instructions) and the prologue wait; A/B against the
# two-path form; device-round tests first.
set -o pipefail
O=gpurun_out/r06/zc_uni
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_device_round.py \
  tests/test_gpu_device_clients.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for K in 129 200 257 384 500 1000; do
  timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 10 > $O/uni_k$K.log 2>&1 || exit $?
  FEDAVG_SEGWINF_TWO_PATHS=1 timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 10 > $O/two_k$K.log 2>&1 || exit $?
done
for K in 129 200 257 384 500 1000; do echo "K=$K uni $(grep -h '^{' $O/uni_k$K.log | cut -c90-170) | two-path $(grep -h '^{' $O/two_k$K.log | cut -c90-170)"; done
