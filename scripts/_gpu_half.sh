set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01h}; mkdir -p $OUT
for dt in bf16 f16; do
  timeout -k 10 300 python scripts/half_variants.py --dtype $dt --K 100 --P 25000000 > $OUT/half_${dt}_k100.jsonl 2> $OUT/half_${dt}_k100.err
  head -8 $OUT/half_${dt}_k100.jsonl | cut -c1-200; grep production $OUT/half_${dt}_k100.jsonl | cut -c1-250
done
timeout -k 10 300 python scripts/half_variants.py --dtype bf16 --K 500 --P 11227812 > $OUT/half_bf16_k500.jsonl 2> $OUT/half_bf16_k500.err
head -8 $OUT/half_bf16_k500.jsonl | cut -c1-200; grep production $OUT/half_bf16_k500.jsonl | cut -c1-250
