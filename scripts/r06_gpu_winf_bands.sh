#!/bin/bash
# Round 6: where the hand-off split windows beat the plan's other forms below
# 369 clients (the bands were tuned on the barrier form): production plan vs
# winf<8,8> (91000808) at long and short rows.
set -o pipefail
O=gpurun_out/r06/winf_bands
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python scripts/fused_probe.py --shapes 130x5000000 140x5000000 150x5000000 160x5000000 170x5000000 \
  200x5000000 256x5000000 260x5000000 270x5000000 288x5000000 300x5000000 340x5000000 368x5000000 \
  200x1200000 300x1200000 370x1200000 500x1403477 1000x1562500 \
  --variants 91000808,0 91001616,0 --rounds 3 --reps 3 > $O/probe.jsonl 2> $O/probe.err || exit $?
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/r06/winf_bands/probe.jsonl")]
by = {}
for r in rows:
    if "ms_median" in r:
        by.setdefault((r["K"], r["P"]), {})[r["variant"]] = r["ms_median"]
for (K, P), v in sorted(by.items()):
    print(K, P, {k: v[k] for k in ("reduce-only", "fused", "S91000808b0", "S91001616b0") if k in v})
PY
