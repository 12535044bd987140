set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g20
mkdir -p $O
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 80x25000000 --variants 70010042,0 70010041,0 170010041,0 70008041,0 70008042,0 61000042,0 --rounds 4 --reps 6 > $O/vec1.jsonl 2> $O/vec1.err
echo vec1 ok
bash scripts/r03_g19.sh
