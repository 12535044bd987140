set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01seg}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_clients.py tests/test_gpu_fpf.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_dev.log 2>&1 || { tail -40 $OUT/pytest_dev.log; exit 1; }
echo "device tests: $(tail -1 $OUT/pytest_dev.log)"
timeout -k 10 600 python -u bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err || { tail -30 $OUT/e2e.err; exit 1; }
python -c "
import json
for l in open('$OUT/e2e.jsonl'):
    r=json.loads(l); print(r['config'], 'host', r['e2e_ms_median'], 'dev', r['device_clients_ms_median'], r['device_clients_GBps'], 'devstream', r['device_clients_stream_finish_ms_median'], r['device_clients_bit_exact'], r['bit_exact_vs_cpu_ref'], 'dist', r['dist_ms_median'], 'devdist', r['device_clients_dist_ms_median'], r['device_clients_dist_max_rel_vs_host'])
"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o seg -- python3 $GRAFT_REPO_ROOT/bench.py --e2e --configs resnet56,target_flat --reps 3 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
cd $GRAFT_REPO_ROOT && grep -E "segments|pack_rows_device|reduce_f32x4_var|sqdist" $OUT/prof/seg_kernel_stats.csv | cut -c1-220
