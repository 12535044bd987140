set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke: $(tail -1 $OUT/smoke.log)"
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-200 $OUT/bench.json; python -c "import json; r=json.load(open('$OUT/bench.json')); print(r['roofline'])"
FEDAVG_DIST_BACKEND=gloo FEDAVG_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 3 --warmup 1 > $OUT/rehearsal_gloo2.json 2> $OUT/rehearsal_gloo2.err
python -c "import json; r=json.loads(open('$OUT/rehearsal_gloo2.json').read().strip().splitlines()[-1]); print('gloo2', r['config']['chunks'], r['parity'], r['roofline'])"
