set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g5
mkdir -p $O
timeout -k 10 300 python -u scripts/buf_probe.py --K 100 --P 1562560 --chunks 2 --rounds 4 --reps 8 --buf 4,6,0 2,6,0 8,6,0 4,4,0 8,4,0 2,12,0,128 4,6,0,128 --nt 4,6,0,1 8,4,0,1 > $O/chunk_1p56m.jsonl 2> $O/c1.err
echo c1 ok
timeout -k 10 300 python -u scripts/buf_probe.py --K 100 --P 1041728 --chunks 3 --rounds 4 --reps 8 --buf 4,4,0 8,4,0 16,4,0 4,6,0 2,6,0 --nt 16,4,0,1 4,6,0,1 > $O/chunk_1p04m.jsonl 2> $O/c2.err
echo c2 ok
timeout -k 10 300 python -u scripts/buf_probe.py --K 100 --P 781312 --chunks 4 --rounds 4 --reps 8 --buf 8,3,0 4,3,0 16,3,0 4,4,0 8,4,0 16,4,0 --nt 16,4,0,1 8,3,0,1 > $O/chunk_781k.jsonl 2> $O/c3.err
echo c3 ok
timeout -k 10 300 python -u -m pytest tests/test_gpu_fpf.py tests/test_gpu_autostream.py tests/test_gpu_fused.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
echo tests ok
