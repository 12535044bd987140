set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01dev2}; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err || { tail -30 $OUT/e2e.err; exit 1; }
python -c "
import json
for l in open('$OUT/e2e.jsonl'):
    r=json.loads(l); print(r['config'], 'host', r['e2e_ms_median'], 'dev', r['device_clients_ms_median'], r['device_clients_GBps'], 'devstream', r['device_clients_stream_finish_ms_median'], r['device_clients_bit_exact'], r['bit_exact_vs_cpu_ref'])
"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o dev -- python3 $GRAFT_REPO_ROOT/bench.py --e2e --configs resnet56,target_flat --reps 3 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
cd $GRAFT_REPO_ROOT && find $OUT/prof -name "*kernel_stats.csv" | head -3
