set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-r01d4}; mkdir -p $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o stream -- python3 $GRAFT_REPO_ROOT/scripts/stream_probe.py --rounds 4 > $GRAFT_REPO_ROOT/$OUT/stream.jsonl 2> $GRAFT_REPO_ROOT/$OUT/stream.err
cd $GRAFT_REPO_ROOT && ls $OUT/prof && python -c "import json; [print(round(json.loads(l)['finish_ms'],3)) for l in open('$OUT/stream.jsonl')]"
