set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g6
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo bench default ok
timeout -k 10 200 python -u bench.py --shard-of 8 --steps 30 --warmup 5 --no-cpu-baseline > $O/shard8_auto.json 2> $O/shard8_auto.err
echo shard8 ok
timeout -k 10 200 python -u bench.py --shard-of 4 --steps 30 --warmup 5 --no-cpu-baseline > $O/shard4_auto.json 2> $O/shard4_auto.err
echo shard4 ok
timeout -k 10 300 python -u bench.py --workload resnet18_gn --steps 20 --warmup 5 --no-cpu-baseline > $O/cfg4_n1.json 2> $O/cfg4_n1.err
echo cfg4 ok
