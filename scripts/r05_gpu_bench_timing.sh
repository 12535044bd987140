#!/usr/bin/env bash
# Round 5: bench lines with the whole-region event pair (no per-launch
# attached events) -- target, FEMNIST, resnet56 -- and the target under
# rocprofv3 --kernel-trace --stats for the per-launch agreement.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g32}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
log start
for w in target femnist_cnn resnet56; do
  timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  log "$w: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])" "$OUT/bench_$w.json")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python bench.py --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
find "$OUT/prof" -name "*kernel_trace.csv" -delete
log "under rocprof: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])" "$OUT/prof_bench.json")"
log done
