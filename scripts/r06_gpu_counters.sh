#!/bin/bash
# Round 6: (1) K = 100 fused window: time + shader clock of the production kernel,
# its fp32-squares and loads-only forms and the plain reduce, interleaved;
# (2) SQ counter passes on the split-row window (1000 x 12.5M, packed rows) and
# its zero-copy form (cfg4 resnet18_gn x 500, separate allocations).
set -o pipefail
O=gpurun_out/r06/counters
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/clock_attrib_probe.py --rounds 4 --reps 6 > $O/clock_attrib.jsonl 2> $O/clock_attrib.err || exit $?
echo "clock probe done"
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA"
P2="SQ_WAVE_CYCLES,SQ_INSTS_VMEM_RD,SQ_INST_CYCLES_VMEM_RD,SQ_INST_LEVEL_VMEM,SQ_VMEM_TA_ADDR_FIFO_FULL,SQ_VMEM_TA_CMD_FIFO_FULL,SQ_ACTIVE_INST_VMEM,SQ_WAIT_INST_LDS"
P3="SQ_WAVE_CYCLES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_INSTS_SMEM,SQ_ACTIVE_INST_MISC,SQ_INST_LEVEL_LDS"
n=0
for PASS in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-include-regex winn --output-format csv -d $O/rows_p$n -o run -- \
    python scripts/fused_probe.py --shapes 1000x12500000 --variants --rounds 1 --reps 2 > $O/rows_p$n.log 2>&1 || exit $?
  echo "rows pass $n done"
  timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-include-regex segwinn --output-format csv -d $O/zc_p$n -o run -- \
    python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --calls 4 > $O/zc_p$n.log 2>&1 || exit $?
  echo "zero-copy pass $n done"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rows_stats -o run -- \
  python scripts/fused_probe.py --shapes 1000x12500000 --variants --rounds 2 --reps 4 > $O/rows_stats.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/zc_stats -o run -- \
  python scripts/segwin_layout_probe.py --layout separate --config resnet18_gn --calls 12 > $O/zc_stats.log 2>&1 || exit $?
find $O -name "*kernel_trace.csv" -delete
echo all done
