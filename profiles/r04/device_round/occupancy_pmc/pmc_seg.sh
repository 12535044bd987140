set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmc_seg
mkdir -p $O
P="python scripts/segwin_layout_probe.py --config resnet56 --calls 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_sep -o run -- $P --layout separate > $O/stats_sep.log 2>&1 || exit 1
echo stats_sep ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_packed -o run -- $P --layout packed > $O/stats_packed.log 2>&1 || exit 1
echo stats_packed ok
for L in separate packed; do
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex reduce_ --output-format csv -d $O/fetch_$L -o run -- $P --layout $L > $O/fetch_$L.log 2>&1 || exit 1
echo fetch_$L ok
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU --kernel-include-regex reduce_ --output-format csv -d $O/sq_$L -o run -- $P --layout $L > $O/sq_$L.log 2>&1 || exit 1
echo sq_$L ok
done
find $O -name '*trace*.csv' -size +20M -delete
