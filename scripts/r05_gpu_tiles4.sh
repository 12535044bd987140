#!/usr/bin/env bash
# Round 5: why the segments tile kernel (device round) runs ~45% over the rows
# tile kernel on the SAME bytes (resnet56_flat, packed [K, ld] layout): the
# dispatch records (grid, LDS, registers) and SQ / TCC counters of both.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${RUN_TAG:-g14}
mkdir -p "$OUT"
log() { echo "[r05] $(date -u +%T) $*" | tee -a "$OUT/progress.log"; }
keep() {  # the fused kernels' rows only (the trace of torch's init kernels is large)
  python - "$1" <<'EOF'
import csv, sys, glob, os
for f in glob.glob(os.path.join(sys.argv[1], "**", "*.csv"), recursive=True):
    if not (f.endswith("kernel_trace.csv") or f.endswith("counter_collection.csv")):
        continue
    rows = list(csv.reader(open(f)))
    if not rows:
        continue
    hdr = rows[0]
    name = hdr.index("Kernel_Name")
    kept = [r for r in rows[1:] if "reduce_sqdist" in r[name] or "finalize" in r[name]]
    with open(f[:-4] + "_fused.csv", "w", newline="") as o:
        w = csv.writer(o)
        w.writerow(hdr)
        w.writerows(kept)
    os.remove(f)
EOF
}
PROBE="python scripts/segwin_layout_probe.py --layout packed --config resnet56_flat --calls 20"
log start
for LA in 1 0; do
  D="$OUT/trace_la$LA"
  FEDAVG_SEG_LADDR=$LA FEDAVG_SEGWIN_MIN_PER_WAVE=1000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$D" -o run -- $PROBE > "$D.log" 2>&1
  keep "$D"
  log "trace la=$LA: $(grep -h '"layout"' "$D.log" | cut -c1-250)"
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum"
P3="WRITE_SIZE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  D="$OUT/pmc$i"
  FEDAVG_SEGWIN_MIN_PER_WAVE=1000000 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$D" -o run \
      -- $PROBE > "$D.log" 2>&1
  keep "$D"
  log "pmc$i done"
done
log done
