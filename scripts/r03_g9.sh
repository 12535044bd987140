set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g9
mkdir -p $O
timeout -k 10 200 python -u scripts/stream_install_probe.py --K 10 --P 7850 --keys 2 --rounds 30 --delay-ms 1 > $O/stream_mnist.jsonl 2> $O/stream_mnist.err
echo mnist ok
timeout -k 10 200 python -u scripts/stream_install_probe.py --K 10 --P 1206590 --keys 8 --rounds 20 --delay-ms 2 > $O/stream_femnist.jsonl 2> $O/stream_femnist.err
echo femnist ok
for w in femnist_cnn resnet56; do
  for r in 1 2; do
    timeout -k 10 200 python -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_${w}_$r.json 2> $O/bench_${w}_$r.err
    echo $w $r ok
  done
done
timeout -k 10 600 python -u bench.py --workload synthetic_1000x100m --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err
echo cfg5 ok
