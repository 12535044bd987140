set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01cfg}; mkdir -p $OUT
for w in resnet18_gn synthetic_1000x100m_slice femnist_cnn resnet56; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json; r=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print('$w', r['value'], r['roofline']['kernel'][:50], r['roofline']['frac'], r['parity']['ok'])"
done
timeout -k 10 200 python -u scripts/buf_probe.py --K 500 --P 11227812 --rounds 8 --buf 2,16,0 --glob 4,8,768 > $OUT/buf_cfg4.jsonl 2>> $OUT/buf.err
timeout -k 10 300 python -u scripts/buf_probe.py --K 1000 --P 12500000 --rounds 4 --reps 4 --buf 2,16,0 --glob 4,8,768 > $OUT/buf_cfg5.jsonl 2>> $OUT/buf.err
cut -c1-150 $OUT/buf_cfg4.jsonl $OUT/buf_cfg5.jsonl
