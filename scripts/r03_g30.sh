set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g30
mkdir -p $O
B="40002,16,0 4040002,16,0 8040002,16,0 2040002,16,0"
for s in 513x10000000 1000x25000000 2000x5000000 640x3000000; do
K=${s%x*}; P=${s#*x}
timeout -k 10 300 python -u scripts/dist_variants.py --K $K --P $P --rounds 3 --iters 3 --glob --buf $B > $O/dist_$s.jsonl 2> $O/dist_$s.err
echo $s ok
done
