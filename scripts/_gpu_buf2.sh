set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01buf2}; mkdir -p $OUT
timeout -k 10 300 python -u scripts/buf_probe.py --rounds 8 --buf 2,16,0 2,16,512 2,16,768 2,16,1024 2,16,1536 4,8,0 8,8,0 4,16,0 \
   --glob 2,16,0 4,8,0 2,16,768 > $OUT/buf.jsonl 2> $OUT/buf.err || { tail -30 $OUT/buf.err; exit 1; }
cut -c1-160 $OUT/buf.jsonl
timeout -k 10 300 python -u scripts/buf_probe.py --rounds 8 --K 500 --P 5000000 --buf 2,16,0 4,8,0 2,16,768 --glob 2,16,0 > $OUT/buf_k500.jsonl 2>> $OUT/buf.err || { tail -30 $OUT/buf.err; exit 1; }
cut -c1-160 $OUT/buf_k500.jsonl
timeout -k 10 300 python -u scripts/buf_probe.py --rounds 8 --K 10 --P 1206590 --buf 2,16,0 4,8,0 --glob 2,16,0 > $OUT/buf_k10.jsonl 2>> $OUT/buf.err || { tail -30 $OUT/buf.err; exit 1; }
cut -c1-160 $OUT/buf_k10.jsonl
