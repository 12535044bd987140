set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g28
mkdir -p $O
B="40002,16,0 2040002,16,0 4040002,16,0 8040002,16,0 2040004,4,0 4040004,4,0 2040004,8,0 4040004,8,0"
timeout -k 10 300 python -u scripts/dist_variants.py --K 100 --P 25000000 --rounds 4 --iters 5 --glob --buf $B > $O/dist_k100.jsonl 2> $O/err1
echo k100 ok
timeout -k 10 300 python -u scripts/dist_variants.py --K 1000 --P 12500000 --rounds 3 --iters 3 --glob --buf $B > $O/dist_k1000.jsonl 2> $O/err2
echo k1000 ok
