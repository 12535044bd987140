set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01chk}; mkdir -p $OUT
B="4,8,0 8,8,0 4,4,0 8,4,0 2,8,0 2,16,0"
G="8,4,768 16,4,768 8,2,768 16,1,768 4,8,768"
for shape in "100 390625" "100 781250" "100 1562500" "100 3125000"; do
  set -- $shape
  timeout -k 10 120 python -u scripts/buf_probe.py --K $1 --P $2 --rounds 12 --reps 8 --buf $B --glob $G >> $OUT/chunks.jsonl 2>> $OUT/err.log || { tail -30 $OUT/err.log; exit 1; }
done
python - <<'PY'
import json, os
from collections import defaultdict
d=defaultdict(dict)
for l in open(f"gpurun_out/{os.environ.get('RUN_TAG','r01chk')}/chunks.jsonl"):
    r=json.loads(l); d[(r["K"],r["P"])][r["variant"]]=r["GBps"]
names=list(next(iter(d.values())).keys())
print("variant".ljust(20), *[f"{k[0]}x{k[1]}".rjust(12) for k in d])
for n in names: print(n.ljust(20), *[str(d[k].get(n)).rjust(12) for k in d])
PY
