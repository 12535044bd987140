set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g21
mkdir -p $O
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 --variants 70010042,0 76000042,0 76000082,0 60000082,0 61000042,0 --rounds 4 --reps 6 > $O/sync.jsonl 2> $O/sync.err
echo sync ok
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*\|GRBM_[A-Z_0-9]*" $O/counters.txt | sort -u > $O/counter_names.txt || true
echo list ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "win_kernel|reduce_f32x4_buf" --output-format csv -d $O/sq -o run -- python scripts/fused_probe.py --shapes 100x25000000 --variants 70010042,0 61000042,0 --rounds 1 --reps 3 > $O/sq.log 2>&1
echo sq ok
