set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01seg2}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_clients.py tests/test_gpu_fpf.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_dev.log 2>&1 || { tail -40 $OUT/pytest_dev.log; exit 1; }
echo "device tests: $(tail -1 $OUT/pytest_dev.log)"
for m in resnet56 femnist_cnn target_flat; do
  timeout -k 10 200 python -u scripts/segments_probe.py --model $m --rounds 6 --reps 6 >> $OUT/segmodel.jsonl 2>> $OUT/segmodel.err || { tail -30 $OUT/segmodel.err; exit 1; }
done
cut -c1-150 $OUT/segmodel.jsonl
timeout -k 10 600 python -u bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err || { tail -30 $OUT/e2e.err; exit 1; }
python -c "
import json
for l in open('$OUT/e2e.jsonl'):
    r=json.loads(l); print(r['config'], 'host', r['e2e_ms_median'], 'dev', r['device_clients_ms_median'], r['device_clients_GBps'], 'devstream', r['device_clients_stream_finish_ms_median'], r['device_clients_bit_exact'], r['bit_exact_vs_cpu_ref'], 'dist', r['dist_ms_median'], 'devdist', r['device_clients_dist_ms_median'])
"
