set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g26
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo gpu tests ok
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 python -u scripts/segments_probe.py --rounds 4 --reps 6 --names seg-rows seg-tensors ptrs-rows ptrs-tensors seg-skewed-tensors seg-2mib-pitch > $O/seg_prod.jsonl 2> $O/seg_prod.err
echo seg ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 90x25000000 --variants 70010042,0 --rounds 4 --reps 6 > $O/fused_prod.jsonl 2> $O/fused_prod.err
echo fused ok
