"""Summarise rocprofv3 --pmc CSV passes (SQ counters) per kernel: mean per
dispatch of every counter, over the passes given.

    python scripts/sq_counter_table.py DIR [DIR ...] [--regex winn] [--json out.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--regex", default=".")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    meta = {}
    for d in args.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if not re.search(args.regex, k):
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta[k] = {"grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]), "lds": int(r["LDS_Block_Size"]),
                           "vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]), "sgpr": int(r["SGPR_Count"])}
    out = {}
    for k, cs in vals.items():
        short = re.sub(r"\(.*", "", k.replace("void ", "").replace("(anonymous namespace)::", ""))
        out[short] = {"meta": meta[k], "counters": {c: sum(v) / len(v) for c, v in sorted(cs.items())},
                      "dispatches": {c: len(v) for c, v in sorted(cs.items())}}
        print(short, meta[k])
        for c, v in sorted(cs.items()):
            print(f"  {c:28s} {sum(v) / len(v):.4e}  (n={len(v)})")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
