set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01p}; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "variants" > $OUT/pytest_variants.log 2>&1
echo "variant parity: $(tail -1 $OUT/pytest_variants.log)"
for cfg in "1000 7850 k1000p7850" "10000 7850 k10000p7850" "1000 600372 k1000p600k" "100 7850 k100p7850" "2 100000000 k2p100m" "10 25000000 k10p25m" "3 25000000 k3p25m" "100 150000 k100p150k"; do
  set -- $cfg
  timeout -k 10 300 python scripts/kernel_variants.py --set small --K $1 --P $2 --rounds 5 --iters 20 > $OUT/small_$3.jsonl 2> $OUT/small_$3.err
  echo "$3: $(head -1 $OUT/small_$3.jsonl | cut -c1-110)"
done
