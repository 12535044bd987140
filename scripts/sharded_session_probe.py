"""A streamed round over N column shards (multi.ShardedRoundSession) at K
clients x P fp32, host clients: add() every client, then finish(); the
finish's host phases per round (issue per shard, verify, wait), against the
single-device RoundSession on the same clients.  On a one-GPU box every
shard maps to cuda:0 (one PCIe link, the device's hardware queues shared by
all shards' streams), so this rehearses the N-GPU finish's host side and
bits, not its link rates.

    python scripts/sharded_session_probe.py [--K 100 --P 25000000] [--shards 1,2,4,8] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import OrderedDict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

import mfl_amd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, P = args.K, args.P
    base = torch.randn(P) * 0.05
    clients = [OrderedDict(w=base + (i * 1e-3 - 0.05)) for i in range(K)]
    counts = [int(c) for c in np.random.default_rng(7).integers(1, 1000, size=K)]
    ref = None
    for n in [int(x) for x in args.shards.split(",")]:
        agg = mfl_amd.default_aggregator(dev) if n == 1 else mfl_amd.ShardedAggregator([0] * n)
        agg.warm_up() if n == 1 else None
        for r in range(args.rounds):
            sess = agg.begin_round(clients[0], K)
            t0 = time.perf_counter()
            for c, sd in zip(counts, clients):
                sess.add(c, sd)
            t1 = time.perf_counter()
            torch.cuda.synchronize()  # every upload landed: the finish alone below
            t2 = time.perf_counter()
            wl = [(c, OrderedDict(sd)) for c, sd in zip(counts, clients)]
            sess.dicts = [sd for _, sd in wl]
            out = sess.finish(wl)
            t3 = time.perf_counter()
            if ref is None:
                ref = out["w"].clone()
            same = torch.equal(out["w"].view(torch.int32), ref.view(torch.int32))
            print(json.dumps({"shards": n, "round": r, "add_all_ms": round((t1 - t0) * 1e3, 2),
                              "uploads_drain_ms": round((t2 - t1) * 1e3, 2), "finish_ms": round((t3 - t2) * 1e3, 3),
                              "finish_profile": sess.finish_profile, "add_profile": sess.add_profile,
                              "bit_identical_to_first": bool(same),
                              "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")}), flush=True)


if __name__ == "__main__":
    main()
