set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g13
mkdir -p $O
timeout -k 10 300 python -u scripts/segments_probe.py --model target_flat --rounds 4 --sched 2,16,1 2,16,2 4,4,3 4,4,2 4,4,1 4,8,1 2,8,1 1,16,2 > $O/flat.jsonl 2> $O/flat.err
echo flat ok
timeout -k 10 400 python -u scripts/segments_probe.py --model resnet18_gn --rounds 4 --sched 2,16,1 2,16,2 4,4,3 4,4,2 4,4,1 4,8,2 > $O/r18.jsonl 2> $O/r18.err
echo r18 ok
timeout -k 10 300 python -u scripts/segments_probe.py --model resnet56 --rounds 4 --sched 4,1,8 4,1,4 4,1,2 4,4,2 4,4,1 > $O/r56.jsonl 2> $O/r56.err
echo r56 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o flat -- python -u scripts/segments_probe.py --model target_flat --rounds 2 --sched 2,16,1 2,16,2 4,4,3 > $O/flat_prof.jsonl 2> $O/flat_prof.err
echo prof ok
cat $O/flat.jsonl $O/r18.jsonl $O/r56.jsonl
find $O/prof -name "*kernel_stats.csv" | head -3
