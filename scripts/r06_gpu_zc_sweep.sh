#!/bin/bash
# Round 6: zero-copy device rounds against the rows kernel on the same values
# (packed layout) across client counts, resnet18_gn-shaped clients.
set -o pipefail
O=gpurun_out/r06/zc_sweep
mkdir -p $O
export TMPDIR=/tmp
for K in 8 16 17 32 64 65 100 128 129 257 384; do
  timeout -k 10 240 python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --clients $K --calls 10 > $O/sep_k$K.log 2>&1 || exit $?
  timeout -k 10 240 python scripts/segwin_layout_probe.py --layout packed --config resnet18_gn --clients $K --calls 10 > $O/packed_k$K.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob
for K in (8, 16, 17, 32, 64, 65, 100, 128, 129, 257, 384):
    s = [json.loads(l) for l in open(f"gpurun_out/r06/zc_sweep/sep_k{K}.log") if l.startswith("{")][0]
    p = [json.loads(l) for l in open(f"gpurun_out/r06/zc_sweep/packed_k{K}.log") if l.startswith("{")][0]
    print(K, "zero-copy", s["round_gpu_us_median"], "rows", p.get("rows_gpu_us_median"), "packed-round", p["round_gpu_us_median"],
          "same_out", s["out_checksum"] == p["out_checksum"])
PY
