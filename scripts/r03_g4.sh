set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 150 --timeout-method thread > $O/pytest_fused.log 2>&1
echo fused tests ok
timeout -k 10 400 python -u scripts/stream_install_probe.py --rounds 5 > $O/stream_install.jsonl 2> $O/stream_install.err
echo stream ok
timeout -k 10 500 python -u scripts/fused_probe.py --shapes 8x125000000 16x62500000 24x41666688 32x31250000 48x20833344 --variants 256,0 128,0 200256,0 200128,0 --rounds 2 --reps 5 > $O/rule_small.jsonl 2> $O/rule_small.err
echo small ok
timeout -k 10 500 python -u scripts/fused_probe.py --shapes 129x7750016 160x6250000 192x5208320 224x4464320 --variants 64,0 32,0 200032,0 1800064,0 --rounds 2 --reps 5 > $O/rule_mid.jsonl 2> $O/rule_mid.err
echo mid ok
timeout -k 10 500 python -u scripts/fused_probe.py --shapes 384x5000000 448x5000000 512x5000000 640x3000000 --variants 1800032,0 3400032,0 --rounds 2 --reps 4 > $O/rule_big.jsonl 2> $O/rule_big.err
echo big ok
