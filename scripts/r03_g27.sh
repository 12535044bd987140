set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g27
mkdir -p $O
for P in 1562500 3125000 781250 12500000; do
timeout -k 10 200 python -u scripts/segments_probe.py --K 100 --P $P --rounds 4 --reps 10 --names ptrs-rows seg-rows > $O/chunk_$P.jsonl 2> $O/chunk_$P.err
echo $P ok
done
timeout -k 10 300 python -u bench.py --shard-of 8 --steps 20 --warmup 5 --no-cpu-baseline > $O/shard8.json 2> $O/shard8.err
echo shard8 ok
B="40002,16,0 2040002,16,0 4040002,16,0 8040002,16,0 2040004,4,0 4040004,4,0 2040004,8,0 4040004,8,0"
timeout -k 10 300 python -u scripts/dist_variants.py --K 100 --P 25000000 --rounds 4 --iters 5 --glob --buf $B > $O/dist_k100.jsonl 2> $O/err1
echo k100 ok
timeout -k 10 300 python -u scripts/dist_variants.py --K 1000 --P 12500000 --rounds 3 --iters 3 --glob --buf $B > $O/dist_k1000.jsonl 2> $O/err2
echo k1000 ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 100x25000003 90x25000000 81x25000000 --variants 70010042,0 124000042,0 188000042,0 252000042,0 --rounds 4 --reps 6 > $O/win_groups.jsonl 2> $O/win_groups.err
echo groups ok
