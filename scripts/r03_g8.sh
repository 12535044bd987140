set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g8
mkdir -p $O
timeout -k 10 400 python -u scripts/fused_probe.py --shapes 100x25000000 --variants 64,0 200064,0 22000128,0 23000128,0 22000256,0 23000256,0 5310256,0 --rounds 3 --reps 6 > $O/deep.jsonl 2> $O/deep.err
echo deep ok
