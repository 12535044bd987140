set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03/g11
mkdir -p $O
N="seg-rows seg-tensors seg-skewed-tensors seg-2mib-pitch seg-pow2-pitch rows-pow2-pitch var-tensors-U2C16b3 var-skewed-U2C16b3 var-rows-U2C16b3 var-skewed-U4C4b3"
timeout -k 10 300 python -u scripts/segments_probe.py --rounds 6 --names $N > $O/seg_skew_a.jsonl 2> $O/seg_skew_a.err
echo a ok
timeout -k 10 300 python -u scripts/segments_probe.py --rounds 6 --names $N > $O/seg_skew_b.jsonl 2> $O/seg_skew_b.err
echo b ok
cat $O/seg_skew_a.jsonl $O/seg_skew_b.jsonl
