set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g44
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo gpu tests ok
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo bench ok
cat $O/bench_default.json
