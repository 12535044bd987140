set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01segm}; mkdir -p $OUT
for m in resnet56 femnist_cnn target_flat; do
  timeout -k 10 200 python -u scripts/segments_probe.py --model $m --rounds 6 --reps 6 >> $OUT/segmodel.jsonl 2>> $OUT/segmodel.err || { tail -30 $OUT/segmodel.err; exit 1; }
done
cut -c1-170 $OUT/segmodel.jsonl
