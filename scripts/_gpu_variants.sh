set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01h}; mkdir -p $OUT
true
echo gpu parity ok
timeout -k 10 600 python bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err
echo e2e done
for cfg in "100 25000000 target" "100 6250000 chunk4" "500 11227812 resnet18gn" "37 3000001 odd" "1000 12500000 k1000" "100 600372 resnet56" "10 1206590 femnist"; do
  set -- $cfg
  timeout -k 10 400 python scripts/kernel_variants.py --set focus --K $1 --P $2 --rounds 5 --iters 10 > $OUT/focus_$3.jsonl 2> $OUT/focus_$3.err
  echo "$3 done"
done
