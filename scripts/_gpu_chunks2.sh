set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01chk2}; mkdir -p $OUT
for P in 390625 781250 1562500; do
  timeout -k 10 150 python -u scripts/buf_probe.py --K 100 --P $P --chunks 8 --rounds 12 --reps 8 --buf 8,4,0 4,4,0 \
     --nt 16,4,768,0 16,4,768,1 8,4,768,1 8,2,768,1 16,1,768,1 8,4,768,0 >> $OUT/chunks_rot.jsonl 2>> $OUT/err.log || { tail -30 $OUT/err.log; exit 1; }
done
cut -c1-150 $OUT/chunks_rot.jsonl
