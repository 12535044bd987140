set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g12
mkdir -p $O
N="seg-rows seg-tensors"
for src in tensors rows; do
  for v in U2C16b1 U2C16b2 U2C16b3 U4C8b2 U4C8b3 U4C4b2 U4C4b4 U4C4b5 U8C4b2 U2C8b2 U2C8b4 U8C2b4; do N="$N var-$src-$v"; done
done
timeout -k 10 400 python -u scripts/segments_probe.py --rounds 4 --names $N > $O/seg_sched_a.jsonl 2> $O/seg_sched_a.err
echo a ok
timeout -k 10 400 python -u scripts/segments_probe.py --rounds 4 --names $N > $O/seg_sched_b.jsonl 2> $O/seg_sched_b.err
echo b ok
python - <<'PY'
import json
rows = {}
for f in ("a", "b"):
    for l in open(f"gpurun_out/r03/g12/seg_sched_{f}.jsonl"):
        d = json.loads(l)
        if "variant" in d:
            rows.setdefault(d["variant"], []).append(d["GBps"])
for k, v in rows.items():
    print(f"{k:28s} {v}")
PY
