# Session-2 checks: GPU tests, the D2H path sweep (runtime blit vs zero-copy
# kernel), input-distribution upload rates, e2e, and a 2-rank rehearsal of the
# N>1 bench path (gloo, both ranks on cuda:0; the driver uses RCCL).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01t}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 300 python scripts/upload_probe.py > $OUT/upload.jsonl 2> $OUT/upload.err
cat $OUT/upload.jsonl
for b in 0 64; do
  FEDAVG_D2H_BLOCKS=$b timeout -k 10 300 python scripts/stream_probe.py --rounds 5 > $OUT/stream_b$b.jsonl 2> $OUT/stream_b$b.err
  echo "blocks=$b $(python -c "import json; r=[json.loads(l) for l in open('$OUT/stream_b$b.jsonl')][1:]; print('finish ms', [round(x['finish_ms'],3) for x in r])")"
done
timeout -k 10 600 python bench.py --e2e --reps 5 > $OUT/e2e.jsonl 2> $OUT/e2e.err
cat $OUT/e2e.jsonl
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 3 --warmup 1 > $OUT/rehearsal_gloo2.json 2> $OUT/rehearsal_gloo2.err
echo "gloo2 rehearsal: $(tail -1 $OUT/rehearsal_gloo2.json | cut -c1-400)"
