set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g38
mkdir -p $O
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 65x20000 65x200000 70x20000 80x200000 80x1500000 --variants 64,0 70008042,0 --rounds 3 --reps 8 > $O/k65_80.jsonl 2> $O/k65_80.err
echo a ok
timeout -k 10 400 python -u scripts/fused_probe.py --shapes 85x100000 92x200000 92x1500000 95x200000 95x1500000 98x200000 98x1500000 98x6000000 95x6000000 --variants 64,0 124000042,0 --rounds 3 --reps 8 > $O/k85_98.jsonl 2> $O/k85_98.err
echo b ok
