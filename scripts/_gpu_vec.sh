set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01vec}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "vec_buffer or half or f64 or vec_dtypes" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
timeout -k 10 300 python -u scripts/vec_buf_probe.py > $OUT/vec.jsonl 2> $OUT/vec.err || { tail -30 $OUT/vec.err; exit 1; }
cut -c1-170 $OUT/vec.jsonl
