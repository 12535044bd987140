#!/bin/bash
# Round 6: tight polls in production, the band from 160 clients without the
# 257-288 gap, >= 16 windows per workgroup: tests, the band sweep at the new
# plan (production "fused" vs winf), zero-copy cfg4.
set -o pipefail
O=gpurun_out/r06/winf_v2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_window.py \
  tests/test_gpu_fused.py tests/test_gpu_device_round.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 600 python scripts/fused_probe.py --shapes 160x5000000 200x1200000 260x5000000 288x5000000 \
  368x600000 260x600000 200x800000 1000x12500000 600x10000000 500x11227812 \
  --variants 91000808,0 91011616,0 --rounds 3 --reps 3 > $O/probe.jsonl 2> $O/probe.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/zc -o run -- \
  python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --calls 20 > $O/zc.log 2>&1 || exit $?
find $O -name '*kernel_trace.csv' -delete
python - <<'PY'
import json
by = {}
for l in open("gpurun_out/r06/winf_v2/probe.jsonl"):
    r = json.loads(l)
    if "ms_median" in r:
        by.setdefault((r["K"], r["P"]), {})[r["variant"]] = r["ms_median"]
for (K, P), v in sorted(by.items()):
    print(K, P, {k: v[k] for k in ("reduce-only", "fused", "S91000808b0", "S91011616b0") if k in v})
PY
grep -h '^{' $O/zc.log
grep -h segwinf $O/zc/run_kernel_stats.csv | cut -c1-40,120-
