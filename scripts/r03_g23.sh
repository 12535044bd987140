set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g23
mkdir -p $O
N=""
for src in tensors rows; do
  for v in U2C16b1 U2C16b3 U102C16b3 U202C16b1 U202C16b3 U302C16b1 U302C16b2 U302C16b3 U402C16b2 U402C16b3 U204C4b3 U304C4b3 U304C4b4 U304C8b2 U304C8b3 U404C8b3; do N="$N var-$src-$v"; done
done
timeout -k 10 400 python -u scripts/segments_probe.py --rounds 4 --names seg-tensors $N > $O/style_a.jsonl 2> $O/style_a.err
echo a ok
timeout -k 10 400 python -u scripts/segments_probe.py --rounds 4 --names seg-tensors $N > $O/style_b.jsonl 2> $O/style_b.err
echo b ok
python - <<'PY'
import json
rows = {}
for f in ("a", "b"):
    for l in open(f"gpurun_out/r03/g23/style_{f}.jsonl"):
        d = json.loads(l)
        if "variant" in d:
            rows.setdefault(d["variant"], []).append((d["GBps"], d["bit_identical"]))
for k, v in rows.items():
    print(f"{k:28s} {v}")
PY
