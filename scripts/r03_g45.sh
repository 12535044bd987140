set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g45
mkdir -p $O
# production window kernel (LDS rows) with 1 / 2 / 4 waves per workgroup
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 90x25000000 100x6250000 --variants 124000012,0 124000022,0 124000042,0 --rounds 3 --reps 8 > $O/win_nw.jsonl 2> $O/win_nw.err
echo probe ok
