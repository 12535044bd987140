set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g42
mkdir -p $O
# final-tree readiness of the N>1 path on a 1-GPU box: N ranks on cuda:0 over gloo (the driver's runs use RCCL, one GPU per rank)
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/rehearsal_gloo2.json 2> $O/rehearsal_gloo2.err
echo gloo2 ok
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 4 --steps 10 --warmup 3 --no-cpu-baseline > $O/rehearsal_gloo4.json 2> $O/rehearsal_gloo4.err
echo gloo4 ok
timeout -k 10 300 python -u bench.py --shard-of 8 --steps 20 --warmup 5 --no-cpu-baseline > $O/shard8.json 2> $O/shard8.err
echo shard8 ok
