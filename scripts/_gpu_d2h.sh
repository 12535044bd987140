# Streaming finish vs the D2H path: runtime hipMemcpyAsync (blocks=0) or the
# zero-copy kernel with a bounded grid; then the GPU tests and e2e.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01w}; mkdir -p $OUT
for b in 0 16 32 64 128; do
  FEDAVG_D2H_BLOCKS=$b timeout -k 10 300 python scripts/stream_probe.py --rounds 5 > $OUT/stream_b$b.jsonl 2> $OUT/stream_b$b.err
  echo "blocks=$b $(python -c "import json,sys; r=[json.loads(l) for l in open('$OUT/stream_b$b.jsonl')][1:]; print('finish ms', [round(x['finish_ms'],3) for x in r])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof -o stream -- python scripts/stream_probe.py > $OUT/stream_prof.jsonl 2> $OUT/stream_prof.err
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 600 python bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err
cat $OUT/e2e.jsonl
