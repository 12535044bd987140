#!/bin/bash
# The production plan with the prefetching split windows: parity tests, then
# the production pass against the two passes at the swept shapes.
set -o pipefail
O=gpurun_out/r05/g50
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_window.py tests/test_gpu_fused.py tests/test_gpu_device_round.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python scripts/fused_probe.py --shapes 140x5000000 170x5000000 192x5000000 240x5000000 256x12000000 270x5000000 290x5000000 310x5000000 352x5000000 368x5000000 500x11227812 640x3000000 1000x12500000 200x1206590 300x1500000 \
  --variants --rounds 5 --reps 4 > $O/prod.jsonl 2> $O/prod.err || exit $?
