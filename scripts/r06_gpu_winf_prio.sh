#!/bin/bash
# Round 6: the hand-off windows' squares priority: by quarters (production),
# flat (16), by halves (32).
set -o pipefail
O=gpurun_out/r06/winf_prio
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python scripts/fused_probe.py --shapes 1000x12500000 600x10000000 \
  --variants 91001616,0 91161616,0 91321616,0 --rounds 4 --reps 4 > $O/probe16.jsonl 2> $O/probe16.err || exit $?
timeout -k 10 500 python scripts/fused_probe.py --shapes 500x11227812 300x10000000 \
  --variants 91000808,0 91160808,0 91320808,0 --rounds 4 --reps 4 > $O/probe8.jsonl 2> $O/probe8.err || exit $?
python - <<'PY'
import json
for f in ("probe16", "probe8"):
    by = {}
    for l in open(f"gpurun_out/r06/winf_prio/{f}.jsonl"):
        r = json.loads(l)
        if "ms_median" in r:
            by.setdefault((r["K"], r["P"]), {})[r["variant"]] = r["ms_median"]
    for k, v in sorted(by.items()):
        print(k, v)
PY
