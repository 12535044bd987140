set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g16
mkdir -p $O
FP="timeout -k 10 300 python -u scripts/fused_probe.py --rounds 3 --reps 6"
$FP --shapes 100x25000000 100x12500000 100x6250000 100x3125000 --variants 64,0 70010042,0 > $O/k100_p.jsonl 2> $O/err1
echo k100 ok
$FP --shapes 90x25000000 80x25000000 72x25000000 --variants 64,0 70010042,0 70008042,0 > $O/k72_90.jsonl 2> $O/err2
echo k72-90 ok
$FP --shapes 64x10000000 56x20000000 --variants 128,0 70006442,0 70008042,0 > $O/k56_64.jsonl 2> $O/err3
echo k56-64 ok
$FP --shapes 32x31250000 24x41666667 48x20833333 --variants 128,0 256,0 70003244,0 70004844,0 70006442,0 > $O/k24_48.jsonl 2> $O/err4
echo k24-48 ok
$FP --shapes 128x8000000 112x8000000 --variants 64,0 70012841,0 > $O/k112_128.jsonl 2> $O/err5
echo k112-128 ok
