set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g24
mkdir -p $O
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 100x25000003 90x25000000 --variants 70010042,0 124000042,0 61000042,0 --rounds 4 --reps 6 > $O/ldsrows.jsonl 2> $O/ldsrows.err
echo ldsrows ok
