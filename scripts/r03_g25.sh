set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g25
mkdir -p $O
SP="timeout -k 10 300 python -u scripts/segments_probe.py --rounds 4 --reps 6"
$SP --model target_flat --sched 4,4,3 204,4,3 304,4,3 204,8,3 204,4,2 302,16,1 > $O/target_flat.jsonl 2> $O/err1
echo target ok
$SP --model resnet18_gn --sched 4,4,3 204,4,3 304,4,3 204,4,2 302,16,1 > $O/resnet18_gn.jsonl 2> $O/err2
echo r18 ok
$SP --model resnet56 --sched 4,1,8 204,1,8 304,1,8 > $O/resnet56.jsonl 2> $O/err3
echo r56 ok
$SP --model femnist_cnn --sched 4,1,8 204,1,8 304,1,8 > $O/femnist.jsonl 2> $O/err4
echo femnist ok
