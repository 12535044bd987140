#!/bin/bash
# Round 6: the hand-off split windows at 65-128 clients (2 waves per window)
# against the one-wave window kernels the plan picks there.
set -o pipefail
O=gpurun_out/r06/winf_k100
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python scripts/fused_probe.py --shapes 100x25000000 128x12500000 80x25000000 65x25000000 100x3125000 \
  --variants 91000808,0 91001608,0 --rounds 4 --reps 4 > $O/probe.jsonl 2> $O/probe.err || exit $?
python - <<'PY'
import json
by = {}
for l in open("gpurun_out/r06/winf_k100/probe.jsonl"):
    r = json.loads(l)
    if "ms_median" in r:
        by.setdefault((r["K"], r["P"]), {})[r["variant"]] = r["ms_median"]
for (K, P), v in sorted(by.items()):
    print(K, P, v)
PY
