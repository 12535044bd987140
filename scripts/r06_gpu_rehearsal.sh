#!/bin/bash
# Round 6: the N > 1 bench path on one GPU (gloo, N ranks on cuda:0): the line
# with the north_star block and the prediction, at N = 2 and 8.
set -o pipefail
O=gpurun_out/r06/rehearsal
mkdir -p $O
export TMPDIR=/tmp FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1
for N in 2 8; do
  timeout -k 10 600 python bench.py --gpus $N --steps 5 --warmup 2 > $O/rehearsal_gloo$N.json 2> $O/rehearsal_gloo$N.err || { tail -20 $O/rehearsal_gloo$N.err; exit 1; }
  echo "N=$N ok"
done
