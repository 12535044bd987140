set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g32
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/stats.log 2>&1
echo stats ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "reduce_" --output-format csv -d $O/fetch -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "reduce_" --output-format csv -d $O/write -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1
echo write ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "win_kernel" --output-format csv -d $O/sq -o run -- python scripts/fused_probe.py --shapes 100x25000000 --variants --rounds 1 --reps 3 > $O/sq.log 2>&1
echo sq ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "segments" --output-format csv -d $O/seg_fetch -o run -- python scripts/segments_probe.py --rounds 1 --reps 3 --names seg-tensors > $O/seg_fetch.log 2>&1
echo seg fetch ok
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-include-regex "segments" --output-format csv -d $O/seg_utcl1 -o run -- python scripts/segments_probe.py --rounds 1 --reps 3 --names seg-rows seg-tensors > $O/seg_utcl1.log 2>&1
echo seg utcl1 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seg_stats -o run -- python scripts/segments_probe.py --rounds 2 --reps 5 --names seg-rows seg-tensors > $O/seg_stats.log 2>&1
echo seg stats ok
