set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g29
mkdir -p $O
timeout -k 10 400 python -u scripts/ld_probe.py --K 100 --P 25000000 --rounds 3 --reps 6 --fused --pads 0 64 128 192 256 384 512 1024 4096 > $O/pitch_k100.jsonl 2> $O/pitch_k100.err
echo k100 ok
timeout -k 10 400 python -u scripts/ld_probe.py --K 100 --P 12500000 --rounds 3 --reps 6 --fused --pads 0 64 128 256 512 > $O/pitch_k100_p12.jsonl 2> $O/pitch_k100_p12.err
echo k100 p12 ok
O2=gpurun_out/r03/g30
mkdir -p $O2
B="40002,16,0 4040002,16,0 8040002,16,0 2040002,16,0"
for s in 513x10000000 1000x25000000 2000x5000000 640x3000000; do
K=${s%x*}; P=${s#*x}
timeout -k 10 300 python -u scripts/dist_variants.py --K $K --P $P --rounds 3 --iters 3 --glob --buf $B > $O2/dist_$s.jsonl 2> $O2/dist_$s.err
echo $s ok
done
