set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g20
mkdir -p $O
for r in a b; do
timeout -k 10 400 python -u scripts/segments_probe.py --rounds 4 --reps 6 > $O/seg_layouts_$r.jsonl 2> $O/seg_layouts_$r.err
echo seg $r ok
done
