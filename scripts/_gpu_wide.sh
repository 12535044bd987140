set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01l}; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
for cfg in "100 25000000 target" "500 11227812 resnet18gn" "1000 12500000 k1000"; do
  set -- $cfg
  timeout -k 10 400 python scripts/kernel_variants.py --set wide --K $1 --P $2 --rounds 5 --iters 10 > $OUT/wide_$3.jsonl 2> $OUT/wide_$3.err
  echo "$3 done"
done
timeout -k 10 300 python bench.py --workload resnet56 --no-cpu-baseline > $OUT/bench_resnet56.json 2> $OUT/bench_resnet56.err
echo "resnet56: $(cut -c1-100 $OUT/bench_resnet56.json)"
