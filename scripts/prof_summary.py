"""Summarise rocprofv3 output of scripts/gpu_check.sh into profiles/.

    python scripts/prof_summary.py gpurun_out/<tag> --round r01 --workload target --K 100 --P 25000000 --launches 4

Reads (recursively) the ``*_kernel_stats.csv`` of the ``--kernel-trace
--stats`` pass and the ``*_counter_collection.csv`` of the two separate PMC
passes (FETCH_SIZE, WRITE_SIZE), and writes

  profiles/<round>_<workload>_kernel_stats.csv   (copy of rocprof's summary)
  profiles/<round>_<workload>_pmc.json           (per-kernel counter means)
  profiles/traffic_<workload>.json               (what bench.py attaches)

HBM traffic per launch follows MI355X_MICROARCH.md section HBM: FETCH_SIZE
and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read, so
``hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024``.
"""
from __future__ import annotations

import argparse
import csv
import json
import shutil
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def find(base: Path, suffix: str):
    return sorted(base.rglob(f"*{suffix}"))


def read_csv(p: Path):
    with open(p, newline="") as f:
        return list(csv.DictReader(f))


def counter_means(paths, kernel_regex="reduce_"):
    vals = defaultdict(list)
    meta = {}
    for p in paths:
        for row in read_csv(p):
            name = row.get("Kernel_Name", "")
            # the reduce kernels only: bench.py's round_with_distances side measurement
            # also runs the fused reduce_sqdist and the :291 kernels
            if kernel_regex not in name or "sqdist" in name:
                continue
            vals[(name, row["Counter_Name"])].append(float(row["Counter_Value"]))
            meta[name] = {k: row.get(k) for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count", "SGPR_Count",
                                                   "LDS_Block_Size", "Scratch_Size")}
    return {f"{n}|{c}": sum(v) / len(v) for (n, c), v in vals.items()}, meta, {
        f"{n}|{c}": len(v) for (n, c), v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--workload", default="target")
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--launches", type=int, default=1, help="round-split launches per reduce call")
    args = ap.parse_args()
    base = Path(args.outdir)
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    tag = f"{args.round}_{args.workload}"

    stats = find(base / "prof_stats", "kernel_stats.csv")
    if stats:
        shutil.copy(stats[0], prof / f"{tag}_kernel_stats.csv")
        rows = read_csv(stats[0])
        for r in rows:
            if "reduce_" in r.get("Name", "") and "sqdist" not in r.get("Name", ""):
                print(f"[stats] {r['Name'][:90]} calls={r['Calls']} avg={float(r['AverageNs'])/1e3:.1f} us")

    fetch, meta, nf = counter_means(find(base / "prof_fetch", "counter_collection.csv"))
    write, _, nw = counter_means(find(base / "prof_write", "counter_collection.csv"))
    pmc = {"fetch_size_kib": fetch, "write_size_kib": write, "dispatches": {**nf, **nw}, "kernels": meta,
           "note": "means over dispatches; separate --pmc passes; units KiB (rocprofv3 derived counters)"}
    (prof / f"{tag}_pmc.json").write_text(json.dumps(pmc, indent=1))

    # dominant kernel = the reduce kernel with the most FETCH_SIZE
    best = None
    for key, fv in fetch.items():
        name = key.split("|")[0]
        wv = write.get(f"{name}|WRITE_SIZE")
        if wv is None:
            continue
        if best is None or fv > best[1]:
            best = (name, fv, wv)
    if best:
        name, fv, wv = best
        hbm = (2.0 * fv + wv) * 1024.0
        alg = (4 * args.K * args.P + 4 * args.P + 4 * args.K) // args.launches
        traffic = {
            "kernel": name,
            "FETCH_SIZE_KiB": fv,
            "WRITE_SIZE_KiB": wv,
            "hbm_bytes_per_launch": int(hbm),
            "algorithmic_bytes_per_launch": alg,
            "traffic_over_algorithmic": round(hbm / alg, 4),
            "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024  (gfx950 FETCH_SIZE half-count correction)",
            "source": f"profiles/{tag}_pmc.json",
        }
        (prof / f"traffic_{args.workload}.json").write_text(json.dumps(traffic, indent=1))
        print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
