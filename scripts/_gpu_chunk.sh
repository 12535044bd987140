set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01c}; mkdir -p $OUT
for cb in 4194304 8388608 16777216 33554432; do
  FEDAVG_CHUNK_BYTES=$cb timeout -k 10 300 python bench.py --e2e --reps 7 --configs femnist_cnn,resnet56 > $OUT/e2e_cb$cb.jsonl 2> $OUT/e2e_cb$cb.err
  python -c "
import json
for l in open('$OUT/e2e_cb$cb.jsonl'):
    r=json.loads(l); print($cb, r['config'], 'e2e', r['e2e_ms_median'], 'min', r['e2e_ms_min'], 'pack', r['pack_issue_ms_median'], 'rest', r['h2d_kernel_d2h_ms_median'], 'cpu', r['cpu_ref_ms_median'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json
cut -c1-300 $OUT/bench.json
