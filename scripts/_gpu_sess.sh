set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01sess2}; mkdir -p $OUT
for sb in 4194304 0; do for tm in 5 0; do
FEDAVG_SMALL_ROUND_BYTES=$sb timeout -k 10 120 python -u bench.py --e2e --configs mnist_lr --reps 15 --train-ms $tm > $OUT/e2e_sb${sb}_tm${tm}.jsonl 2> $OUT/e2e_sb${sb}_tm${tm}.err
python -c "import json; r=json.loads(open('$OUT/e2e_sb${sb}_tm${tm}.jsonl').read()); print('sb=$sb tm=$tm', r['e2e_ms_median'], r['stream_finish_ms_median'], r['stream_bit_exact'])"
done; done
