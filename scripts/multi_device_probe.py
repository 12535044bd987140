"""The host path over N column shards (multi.ShardedAggregator) against one
GPU (DeviceAggregator), host state_dicts in, host state_dict out.

    python scripts/multi_device_probe.py [--K 100] [--P 25000000] [--shards 1,2,8] [--reps 3]

On a one-GPU box every shard maps to cuda:0 and shares its one PCIe link, so
the e2e time here is NOT the N-GPU time; what this measures is the part
that does not scale with links: the host packing (fedavg_pack_rows into
pinned staging, the same threads as the drop-in), timed alone, and the
single-link H2D/D2H rates.  Prediction for N GPUs, each on its own x16 link:
    e2e_N ~= max(pack, (rows bytes / N) / H2D link rate) + reduce_N + (P bytes / N) / D2H link rate
One JSON line per leg.
"""
from __future__ import annotations

import argparse
import copy
import json
import sys
import time
from collections import OrderedDict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

import mfl_amd
from mfl_amd.layout import KeyTable


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--shards", default="1,2,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pack-threads", default="",
                    help="also time the packer alone at these thread counts (e.g. 16,32,64): the host rate an "
                         "N-GPU job with more host cores would get")
    ap.add_argument("--skip-dropin", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, P = args.K, args.P
    base = torch.randn(P) * 0.05
    clients = [OrderedDict(w=base + (i * 1e-3 - 0.05)) for i in range(K)]
    counts = [int(c) for c in np.random.default_rng(1234).integers(1, 1000, size=K)]
    ref = None
    # the packer alone: K rows into pinned staging with the drop-in's thread count
    table = KeyTable(clients[0])
    g = table.groups[torch.float32]
    host = torch.empty((K, g.ld), dtype=torch.float32, pin_memory=True)
    ptrs, _ = table.collect(clients)
    lib = mfl_amd._lib.load()
    threads = max(1, torch.get_num_threads())
    ts = []
    for _ in range(args.reps + 1):
        t0 = time.perf_counter()
        items = table.pack_items(g, ptrs, 0, g.ld)
        mfl_amd._lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], host.data_ptr(), 4, threads), "pack")
        ts.append(time.perf_counter() - t0)
    pack_s = float(np.median(ts[1:]))
    print(json.dumps({"leg": "pack_only", "K": K, "P": P, "threads": threads, "ms": round(pack_s * 1e3, 2),
                      "GBps": round(4 * K * P / pack_s / 1e9, 1)}), flush=True)
    import os

    for nt in [int(x) for x in args.pack_threads.split(",") if x.strip()]:
        ts = []
        items = table.pack_items(g, ptrs, 0, g.ld)
        for _ in range(args.reps + 1):
            t0 = time.perf_counter()
            mfl_amd._lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], host.data_ptr(), 4, nt),
                               "pack")
            ts.append(time.perf_counter() - t0)
        s_nt = float(np.median(ts[1:]))
        print(json.dumps({"leg": "pack_threads", "K": K, "P": P, "threads": nt, "ms": round(s_nt * 1e3, 2),
                          "GBps": round(4 * K * P / s_nt / 1e9, 1), "affinity_cpus": len(os.sched_getaffinity(0)),
                          "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}), flush=True)
    # single-link rates: the staging rows H2D, the model D2H
    d = torch.empty((K, g.ld), dtype=torch.float32, device=dev)
    out_h = torch.empty(P, dtype=torch.float32, pin_memory=True)
    for what, fn, nbytes in (("h2d_rows", lambda: d.copy_(host, non_blocking=True), 4 * K * g.ld),
                             ("d2h_model", lambda: out_h.copy_(d[0, :P], non_blocking=True), 4 * P)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        s = (time.perf_counter() - t0) / args.reps
        print(json.dumps({"leg": what, "ms": round(s * 1e3, 2), "GBps": round(nbytes / s / 1e9, 1)}), flush=True)
    del d, host
    torch.cuda.empty_cache()
    for n in ([] if args.skip_dropin else [int(x) for x in args.shards.split(",")]):
        agg = mfl_amd.default_aggregator(dev) if n == 1 else mfl_amd.ShardedAggregator([0] * n)
        times, prof = [], None
        for r in range(args.reps + 1):
            wl = [(c, OrderedDict(sd)) for c, sd in zip(counts, clients)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = agg.aggregate(wl)
            times.append(time.perf_counter() - t0)
            prof = dict(agg.last_profile)
            if ref is None:
                ref = out["w"].clone()
            same = torch.equal(out["w"].view(torch.int32), ref.view(torch.int32))
        print(json.dumps({"leg": "dropin", "shards": n, "K": K, "P": P,
                          "e2e_ms_median": round(float(np.median(times[1:])) * 1e3, 2),
                          "bit_identical_to_1gpu": bool(same), "last_profile": prof,
                          "note": "all shards on cuda:0 (one PCIe link)" if n > 1 else "one GPU"}), flush=True)


if __name__ == "__main__":
    main()
