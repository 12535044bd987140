#!/bin/bash
# Round 6: HBM traffic of the hand-off split windows (rows, 1000 x 12.5M and
# cfg4) -- two PMC passes, FETCH_SIZE and WRITE_SIZE.
set -o pipefail
O=gpurun_out/r06/winf_pmc
mkdir -p $O
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex winf --output-format csv -d $O/$C -o run -- \
    python scripts/fused_probe.py --shapes 1000x12500000 500x11227812 --variants --rounds 1 --reps 2 > $O/$C.log 2>&1 || exit $?
done
python - <<'PY'
import csv, json
from collections import defaultdict
out = {}
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    per = defaultdict(float); name = {}
    for r in csv.DictReader(open(f"gpurun_out/r06/winf_pmc/{C}/run_counter_collection.csv")):
        if r["Counter_Name"] == C:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"]); name[r["Dispatch_Id"]] = r["Kernel_Name"][:60]
    out[C] = [(name[d], per[d]) for d in sorted(per, key=int)]
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/r06/winf_pmc/summary.json", "w"), indent=1)
PY
