set -euo pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${RUN_TAG:-r01utcl}; mkdir -p $OUT
cd /tmp
for v in seg-rows seg-tensors; do
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-include-regex segments \
     --output-format csv -d $OUT/pmc_$v -o run -- python3 $GRAFT_REPO_ROOT/scripts/segments_probe.py --only $v --rounds 1 --reps 3 > $OUT/pmc_$v.log 2>&1
  echo "pass $v ok"
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, os, collections
out = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", os.environ.get("RUN_TAG", "r01utcl"))
for v in ("seg-rows", "seg-tensors"):
    f = glob.glob(f"{out}/pmc_{v}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in acc.items()}, "dispatch-rows", {k: len(x) for k, x in acc.items()})
PY
