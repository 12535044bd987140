set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01xcd; mkdir -p $OUT
timeout -k 10 200 python -u scripts/xcd_probe.py > $OUT/xcd_target.jsonl 2> $OUT/xcd.err
timeout -k 10 200 python -u scripts/xcd_probe.py --K 500 --P 11227812 > $OUT/xcd_k500.jsonl 2>> $OUT/xcd.err
cat $OUT/xcd_target.jsonl $OUT/xcd_k500.jsonl
