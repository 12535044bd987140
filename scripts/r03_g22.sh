set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g22
mkdir -p $O
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 --variants 70010042,0 92000042,0 100000042,0 68000042,0 61000042,0 --rounds 4 --reps 6 > $O/fp32sq.jsonl 2> $O/fp32sq.err
echo fp32sq ok
