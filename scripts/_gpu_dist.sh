set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01dist}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "sqdist or schedule or buffer_descriptor" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
timeout -k 10 200 python -u scripts/dist_variants.py --rounds 6 > $OUT/dist.jsonl 2> $OUT/dist.err || { tail -30 $OUT/dist.err; exit 1; }
cut -c1-170 $OUT/dist.jsonl
timeout -k 10 200 python -u scripts/buf_probe.py --K 100 --P 10000000 --rounds 10 --buf 2,16,0 --glob 4,8,768 > $OUT/buf10m.jsonl 2>> $OUT/dist.err
cut -c1-170 $OUT/buf10m.jsonl
