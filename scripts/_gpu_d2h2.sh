set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01u}; mkdir -p $OUT
for b in 0 64 128 256 0 64; do
  FEDAVG_D2H_BLOCKS=$b timeout -k 10 300 python scripts/stream_probe.py --rounds 10 > $OUT/stream_b$b.jsonl 2> $OUT/stream_b$b.err
  echo "blocks=$b $(python -c "import json; r=[json.loads(l) for l in open('$OUT/stream_b$b.jsonl')][1:]; print('finish ms', [round(x['finish_ms'],3) for x in r])")"
done
timeout -k 10 300 python scripts/upload_probe.py --reps 3 > $OUT/upload.jsonl 2> $OUT/upload.err
cat $OUT/upload.jsonl
