set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g18
mkdir -p $O
for r in a b; do
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 100x25000003 --variants 70010042,0 62000042,0 64000042,0 66000042,0 68000042,0 61000042,0 --rounds 4 --reps 6 > $O/modes_$r.jsonl 2> $O/modes_$r.err
echo $r ok
done
