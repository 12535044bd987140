set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_autostream.py tests/test_gpu_model_shapes.py tests/test_gpu_parity.py -k "autostream or side_stream or session or golden or model" -x -v --timeout 150 --timeout-method thread > $O/pytest_new.log 2>&1
echo tests ok
timeout -k 10 300 python -u scripts/fused_tiled_probe.py > $O/tiled.jsonl 2> $O/tiled.err
echo tiled ok
timeout -k 10 400 python -u scripts/stream_install_probe.py --rounds 3 > $O/stream_install.jsonl 2> $O/stream_install.err
echo stream ok
for c in 1 2 3 4 5 6; do
  timeout -k 10 200 python -u bench.py --shard-of 8 --chunks $c --steps 30 --warmup 5 --no-cpu-baseline > $O/shard8_c$c.json 2> $O/shard8_c$c.err
  echo shard8 c$c ok
done
