set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g47
mkdir -p $O
# standalone :291 pass (K > 512 rounds): occupancy-capped schedules (3 / 4 waves per SIMD) vs production
timeout -k 10 300 python -u scripts/dist_variants.py --K 1000 --P 25000000 --glob --buf 40002,16,0 40302,16,0 40302,12,0 40402,8,0 40303,8,0 --rounds 3 --iters 3 > $O/dist_k1000_minw.jsonl 2> $O/dist_k1000_minw.err
echo k1000 ok
timeout -k 10 300 python -u scripts/dist_variants.py --K 600 --P 10000000 --glob --buf 40002,16,0 40302,16,0 40302,12,0 40402,8,0 40303,8,0 --rounds 3 --iters 5 > $O/dist_k600_minw.jsonl 2> $O/dist_k600_minw.err
echo k600 ok
