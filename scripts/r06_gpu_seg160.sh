#!/bin/bash
# Round 6: zero-copy split windows from 160 clients: device-round tests, then
# a 200-client resnet18_gn-shaped round against the tiles (FEDAVG_SEGWINN_BARRIER=1
# keeps the tiles below 257).
set -o pipefail
O=gpurun_out/r06/seg160
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_device_round.py \
  tests/test_gpu_device_clients.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for K in 160 200 256; do
  timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 12 > $O/zc_k$K.log 2>&1 || exit $?
  FEDAVG_SEGWINN_BARRIER=1 timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 12 > $O/zc_tiles_k$K.log 2>&1 || exit $?
done
grep -h '^{' $O/zc_*.log
