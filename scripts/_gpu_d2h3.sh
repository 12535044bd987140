set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01d3}; mkdir -p $OUT
for b in 0 64; do
  FEDAVG_D2H_BLOCKS=$b timeout -k 10 300 python scripts/stream_probe.py --rounds 6 --keep-results > $OUT/stream_keep_b$b.jsonl 2> $OUT/stream_keep_b$b.err
  echo "keep-results blocks=$b"; python -c "import json; [print(round(json.loads(l)['finish_ms'],3), json.loads(l)['finish_phases_ms']) for l in open('$OUT/stream_keep_b$b.jsonl')]"
done
