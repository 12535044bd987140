#!/bin/bash
# Round 6: the split-row windows after removing the turn loop's vmcnt(0)
# (an explicit wait for the window's own rows before the prefetch), the
# prefetch depth again, the timing modes (no chain / no squares) and the
# LDS-DMA rows; production plan first.
set -o pipefail
O=gpurun_out/r06/winn_waits
mkdir -p $O
export TMPDIR=/tmp
V="87000816,0 87001616,0 87002416,0 88100008,0 88200008,0 88000808,0 88002208,0 88002200,0 88002216,0"
timeout -k 10 600 python scripts/fused_probe.py --shapes 1000x12500000 600x10000000 \
  --variants $V --rounds 3 --reps 3 > $O/probe.jsonl 2> $O/probe.err || exit $?
timeout -k 10 600 python scripts/fused_probe.py --shapes 500x11227812 400x10000000 \
  --variants 87000808,0 87001608,0 --rounds 3 --reps 3 > $O/probe_k500.jsonl 2> $O/probe_k500.err || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_window.py tests/test_gpu_fused.py > $O/pytest.log 2>&1 || exit $?
tail -2 $O/pytest.log
