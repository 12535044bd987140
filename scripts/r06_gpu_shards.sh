#!/bin/bash
# Round 6: per-rank kernel fractions of the strong-scaled plans at N = 2/4/8
# (bench.py --shard-of N: rank 0's shard, its chunks, no exchange) for the
# target, cfg4 and cfg5 -- the inputs of DESIGN.md section 7's 8-GPU
# prediction; then the K = 100 clock attribution with 5 clock passes.
set -o pipefail
O=gpurun_out/r06/shards
mkdir -p $O
export TMPDIR=/tmp
for W in target resnet18_gn synthetic_1000x100m; do
  for N in 2 4 8; do
    timeout -k 10 300 python bench.py --shard-of $N --workload $W --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/${W}_s$N.json 2> $O/${W}_s$N.err || exit $?
    echo "$W shard-of $N: $(tail -c 300 $O/${W}_s$N.json | head -c 120)"
  done
done
for C in 1 2 4 8; do
  timeout -k 10 300 python bench.py --shard-of 8 --workload target --chunks $C --steps 20 --warmup 5 --no-cpu-baseline \
    > $O/target_s8_c$C.json 2> $O/target_s8_c$C.err || exit $?
done
timeout -k 10 300 python scripts/clock_attrib_probe.py --rounds 4 --reps 6 --clock-passes 6 > $O/clock_attrib.jsonl 2> $O/clock_attrib.err || exit $?
echo done
