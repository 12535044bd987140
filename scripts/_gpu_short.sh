set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01short}; mkdir -p $OUT
for shape in "100 390625 8" "100 200000 8" "500 200000 4" "1000 100000 4" "64 500000 8" "200 300000 6"; do
  set -- $shape
  timeout -k 10 150 python -u scripts/buf_probe.py --K $1 --P $2 --chunks $3 --rounds 10 --reps 8 --buf \
     --nt 16,1,768,1 8,2,768,1 16,2,768,1 8,1,768,1 4,2,768,1 >> $OUT/short.jsonl 2>> $OUT/err.log || { tail -30 $OUT/err.log; exit 1; }
done
python - <<'PY'
import json, os
from collections import defaultdict
d=defaultdict(dict)
for l in open(f"gpurun_out/{os.environ.get('RUN_TAG','r01short')}/short.jsonl"):
    r=json.loads(l); d[(r["K"],r["P"])][r["variant"]]=(r["GBps"], r["bit_identical"])
names=list(next(iter(d.values())).keys())
print("variant".ljust(24), *[f"{k[0]}x{k[1]}".rjust(12) for k in d])
for n in names: print(n.ljust(24), *[str(d[k].get(n, ("-",))[0]).rjust(12) for k in d])
print("all identical", all(v[1] for x in d.values() for v in x.values()))
PY
