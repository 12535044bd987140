#!/bin/bash
# Round 6: the delta parity suite (with the 25M scenario), then the bench line,
# rocprofv3 kernel stats and the two PMC passes of the headline (gpu_check.sh).
set -o pipefail
O=gpurun_out/r06/delta2
mkdir -p $O
export TMPDIR=/tmp MFL_REPORT_DIR=$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_delta.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
unset MFL_REPORT_DIR
RUN_TAG=r06/bench SKIP_TESTS=1 ./scripts/gpu_check.sh
