set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01v}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
for b in 0 64; do
  FEDAVG_D2H_BLOCKS=$b timeout -k 10 300 python scripts/stream_probe.py --rounds 8 > $OUT/stream_b$b.jsonl 2> $OUT/stream_b$b.err
  echo "blocks=$b $(python -c "import json; r=[json.loads(l) for l in open('$OUT/stream_b$b.jsonl')]; print('finish ms', [round(x['finish_ms'],3) for x in r])")"
done
timeout -k 10 300 python scripts/upload_probe.py --reps 3 > $OUT/upload.jsonl 2> $OUT/upload.err
cat $OUT/upload.jsonl
timeout -k 10 600 python bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err
cat $OUT/e2e.jsonl
