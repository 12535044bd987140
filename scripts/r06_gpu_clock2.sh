#!/bin/bash
# Round 6: (time, clock) pairs from the same window of calls, 8 interleaved passes.
set -o pipefail
O=gpurun_out/r06/clock2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/clock_attrib_probe.py --rounds 2 --reps 4 --clock-passes 8 > $O/clock_attrib.jsonl 2> $O/clock_attrib.err || exit $?
echo done
