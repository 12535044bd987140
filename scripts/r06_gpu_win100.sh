#!/bin/bash
# Round 6: the K = 100 window with broadcast weights (MODE 256 / 320) against
# production (MODE 64), then the full GPU suite and smoke.
set -o pipefail
O=gpurun_out/r06/win100
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/fused_probe.py --shapes 100x25000000 90x25000000 100x12500000 \
  --variants 364000042,0 316000042,0 380000042,0 --rounds 4 --reps 5 > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/probe.jsonl
if [ "$1" = "--full" ]; then
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 2 $O/smoke.log
fi
