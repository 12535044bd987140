set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g43
mkdir -p $O
# split-row windows with 16-B loads (50 rows x 4 columns per lane, 1 KiB row segments per wave)
timeout -k 10 300 python -u -m pytest tests/test_gpu_window.py -k split_row -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo tests ok
timeout -k 10 300 python -u scripts/fused_probe.py --shapes 100x25000000 90x25000000 100x6250000 --variants 80005004,0 80005002,0 61000042,0 --rounds 3 --reps 8 > $O/win2_vec4.jsonl 2> $O/win2_vec4.err
echo probe ok
bash scripts/r03_g42.sh
