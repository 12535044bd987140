set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01k}; mkdir -p $OUT
# 2-rank rehearsal of the distributed bench path on one GPU (gloo; the driver uses RCCL, one GPU per rank)
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/rehearsal_gloo2.json 2> $OUT/rehearsal_gloo2.err
echo "gloo2 rehearsal ok: $(tail -1 $OUT/rehearsal_gloo2.json | cut -c1-200)"
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 2 --steps 5 --warmup 2 --no-gather > $OUT/rehearsal_gloo2_nogather.json 2> $OUT/rehearsal_gloo2_nogather.err
echo "gloo2 no-gather ok"
for w in femnist_cnn resnet56 resnet18_gn synthetic_1000x100m_slice; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  echo "$w: $(cut -c1-160 $OUT/bench_$w.json)"
done
