#!/bin/bash
# Round 6: :291 -> delta against the reference's own delta (tests/test_gpu_delta.py),
# plus the suites whose harnesses changed (fpf_replay, loop_replay, install gating).
set -o pipefail
O=gpurun_out/r06/delta
mkdir -p $O
export TMPDIR=/tmp MFL_REPORT_DIR=$O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_delta.py tests/test_gpu_fpf.py tests/test_gpu_autostream.py tests/test_gpu_multi.py > $O/pytest.log 2>&1 || exit $?
tail -3 $O/pytest.log
