set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01buf}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "buffer_descriptor or schedule_variants or reduce_f32_exact" > $OUT/pytest_buf.log 2>&1 || { tail -40 $OUT/pytest_buf.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest_buf.log)"
timeout -k 10 300 python -u scripts/buf_probe.py > $OUT/buf.jsonl 2> $OUT/buf.err || { tail -30 $OUT/buf.err; exit 1; }
cut -c1-160 $OUT/buf.jsonl
