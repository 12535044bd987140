set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01m}; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
for cfg in "100 25000000 target" "500 11227812 resnet18gn" "1000 12500000 k1000" "37 3000001 odd" "100 6250000 chunk4"; do
  set -- $cfg
  timeout -k 10 400 python scripts/kernel_variants.py --set window --K $1 --P $2 --rounds 5 --iters 10 > $OUT/window_$3.jsonl 2> $OUT/window_$3.err
  echo "$3 done"
done
for w in femnist_cnn resnet56; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --graph > $OUT/bench_graph_$w.json 2> $OUT/bench_graph_$w.err
  echo "$w graph: $(cut -c1-120 $OUT/bench_graph_$w.json)"
done
