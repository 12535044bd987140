#!/bin/bash
# Round 6: zero-copy split windows, workgroups per CU (FEDAVG_SEGWINN_PER_CU)
# at 3, 4, 5 and 8 waves per workgroup.
set -o pipefail
O=gpurun_out/r06/zc_percu
mkdir -p $O
export TMPDIR=/tmp
for K in 129 200 257 300 500; do
  for C in 0 1 2 3 4 6; do
    FEDAVG_SEGWINN_PER_CU=$C timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 10 > $O/k${K}_c$C.log 2>&1 || exit $?
  done
done
python - <<'PY'
import json
for K in (129, 200, 257, 300, 500):
    row = []
    for C in (0, 1, 2, 3, 4, 6):
        r = [json.loads(l) for l in open(f"gpurun_out/r06/zc_percu/k{K}_c{C}.log") if l.startswith("{")][0]
        row.append(f"c{C}={r['round_gpu_us_median']}")
    print(K, " ".join(row))
PY
