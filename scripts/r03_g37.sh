set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g37
mkdir -p $O
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 70x600000 70x1500000 70x3000000 --variants 64,0 70008042,0 --rounds 3 --reps 8 > $O/k70.jsonl 2> $O/k70.err
echo k70 ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 90x600000 90x1500000 90x3000000 100x600372 100x1500000 100x3000000 --variants 64,0 124000042,0 70010042,0 --rounds 3 --reps 8 > $O/k90_100.jsonl 2> $O/k90_100.err
echo k90 ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 40x600000 40x2000000 56x600000 56x2000000 120x600000 120x2000000 --variants 70004844,0 70006442,0 70012841,0 --rounds 3 --reps 8 > $O/other.jsonl 2> $O/other.err
echo other ok
