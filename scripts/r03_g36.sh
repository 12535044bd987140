set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g36
mkdir -p $O
for r in a b; do
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 100x25000003 90x25000000 81x1000003 25x20000 --variants 124000042,0 380000042,0 --rounds 4 --reps 6 > $O/pairs_$r.jsonl 2> $O/pairs_$r.err
echo $r ok
done
