set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01buf3}; mkdir -p $OUT
B="4,8,0 8,8,0 2,16,0 4,4,0 8,4,0 2,8,0"
G="4,8,768 8,2,768 8,4,768 16,4,768"
for shape in "10 1206590" "100 600372" "100 5000000" "500 5000000" "100 10000000" "20 8000000" "1000 1000000"; do
  set -- $shape
  timeout -k 10 120 python -u scripts/buf_probe.py --K $1 --P $2 --rounds 12 --reps 8 --buf $B --glob $G >> $OUT/buf_shapes.jsonl 2>> $OUT/buf.err || { tail -30 $OUT/buf.err; exit 1; }
  echo "done $shape"
done
python - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/${RUN_TAG:-r01buf3}/buf_shapes.jsonl".replace("${RUN_TAG:-r01buf3}", __import__("os").environ.get("RUN_TAG","r01buf3")))]
from collections import defaultdict
d=defaultdict(dict)
for r in rows: d[(r["K"],r["P"])][r["variant"]]=(r["GBps"], r["bit_identical"])
for k,v in d.items():
    best=max(v.items(), key=lambda t:t[1][0])
    print(k, "prod", v["production"][0], "best", best[0], best[1][0], "all_identical", all(x[1] for x in v.values()))
PY
