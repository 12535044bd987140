"""PMC traffic of the per-rank kernel at every chunk geometry the N > 1 sweep
can pick (bench.chunk_candidates: 1, 2, 4, 8 chunks), from the separate
``rocprofv3 --pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE`` passes of
``bench.py --shard-of N --chunks C`` (scripts/r05_gpu_stream.sh):

    python scripts/shard_traffic_summary.py gpurun_out/r05/g1 --round r05

writes profiles/traffic_target_shard{N}.json (what bench.attach_traffic reads:
one ``launches`` entry per chunk geometry, so a SCALE line never transplants a
ratio) and profiles/<round>/shard_pmc/pmc_s{N}_c{C}.json (the per-kernel means).
HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md:
FETCH_SIZE counts half the bytes of 16-B/lane streaming reads on gfx950).
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def dominant(csv_path: Path, counter: str):
    """(kernel name, grid, mean counter value, dispatches) of the most-dispatched
    reduce launch shape (the timed kernel; parity/clock side launches are rarer)."""
    groups = defaultdict(list)
    with open(csv_path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if "reduce_" not in name or "sqdist" in name or row["Counter_Name"] != counter:
                continue
            groups[(name, int(row["Grid_Size"]))].append(float(row["Counter_Value"]))
    (name, grid), vals = max(groups.items(), key=lambda kv: len(kv[1]))
    return name, grid, sum(vals) / len(vals), len(vals)


def bench_line(log: Path) -> dict:
    for line in log.read_text(errors="replace").splitlines():
        if line.startswith('{"metric"'):
            return json.loads(line)
    raise SystemExit(f"{log}: no bench line")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--round", default="r05")
    ap.add_argument("--workload", default="target")
    args = ap.parse_args()
    base = Path(args.outdir)
    pdir = ROOT / "profiles" / args.round / "shard_pmc"
    pdir.mkdir(parents=True, exist_ok=True)
    by_n = defaultdict(list)
    for d in sorted(base.glob("pmc_s*_c*_FETCH_SIZE")):
        m = re.match(r"pmc_s(\d+)_c(\d+)_FETCH_SIZE", d.name)
        n, c = int(m.group(1)), int(m.group(2))
        wdir = base / f"pmc_s{n}_c{c}_WRITE_SIZE"
        fcsv = next(d.rglob("*counter_collection.csv"))
        wcsv = next(wdir.rglob("*counter_collection.csv"))
        kname, grid, fetch, nf = dominant(fcsv, "FETCH_SIZE")
        kname_w, grid_w, write, nw = dominant(wcsv, "WRITE_SIZE")
        assert (kname, grid) == (kname_w, grid_w), (kname, grid, kname_w, grid_w)
        line = bench_line(base / f"pmc_s{n}_c{c}_FETCH_SIZE.log")
        roof = line["roofline"]
        alg = int(roof["bytes_per_launch"])
        hbm = (2.0 * fetch + write) * 1024.0
        entry = {"kernel": kname, "grid_threads": grid, "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
                 "dispatches": {"FETCH_SIZE": nf, "WRITE_SIZE": nw}, "hbm_bytes_per_launch": int(hbm),
                 "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round(hbm / alg, 4),
                 "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024  (gfx950 FETCH_SIZE half-count correction)",
                 "geometry": f"rank 0 of the {n}-GPU strong-scaled {args.workload} (100 x 25M): {c} chunk(s) of "
                             f"{line['config']['chunk_cols']:,} columns",
                 "chunks": c, "chunk_cols": line["config"]["chunk_cols"],
                 "source": f"profiles/{args.round}/shard_pmc/pmc_s{n}_c{c}.json"}
        (pdir / f"pmc_s{n}_c{c}.json").write_text(json.dumps({**entry, "bench_line_of_fetch_pass": line}, indent=1))
        by_n[n].append(entry)
    for n, entries in sorted(by_n.items()):
        entries.sort(key=lambda e: e["chunks"])
        out = {**entries[0], "launches": entries[1:],
               "collected": f"round {args.round[1:]}: bench.py --shard-of {n} --chunks {{1,2,4,8}} under separate "
                            f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({base})"}
        path = ROOT / "profiles" / f"traffic_{args.workload}_shard{n}.json"
        path.write_text(json.dumps(out, indent=1))
        print(path.name, [(e["chunks"], e["chunk_cols"], e["traffic_over_algorithmic"]) for e in entries])


if __name__ == "__main__":
    main()
