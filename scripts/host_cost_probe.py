"""Host cost of a device-resident round at the BASELINE model shapes.

    python scripts/host_cost_probe.py [--configs resnet56 femnist_cnn target_flat] [--rounds 20]

Clients' state_dicts live in HBM (client.py:96 without the .cpu()); each
round calls the drop-in's aggregate (fedavg_trainer.py:217) and then
client_distances (:291) on fresh shallow copies of the clients' dicts (the
reference deep-copies at :199, so every round's dicts are new objects; the
tensors are reused).  Per round: wall ms of the :217 call and of :291, each
ended by torch.cuda.synchronize (the GPU work included), and the host phases
of :217 (prepare = reference checks + the native state_dict walk; issue =
tables, weights, kernels; the rest = result views and bookkeeping).  One
JSON line per (config, round) and a summary with medians over rounds >= 2.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from collections import OrderedDict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd
from model_shapes import CONFIGS

A = sys.modules[mfl_amd.DeviceAggregator.__module__]


def device_clients(name, dev, seed=0):
    K, shapes = CONFIGS[name]
    g = torch.Generator(device=dev).manual_seed(seed)
    dicts = []
    for i in range(K):
        sd = OrderedDict()
        for k, s in shapes:
            k = "".join(list(k))  # each client's own key strings, as every state_dict() call builds them
            if k.endswith("num_batches_tracked"):
                sd[k] = torch.tensor(1000 + i, dtype=torch.int64, device=dev)
            else:
                sd[k] = torch.randn(s, generator=g, device=dev) * 0.05
        dicts.append(sd)
    counts = [int(c) for c in np.random.default_rng(1234).integers(1, 1001, size=K)]
    return counts, dicts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["resnet56", "femnist_cnn", "target_flat"])
    ap.add_argument("--rounds", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    agg = mfl_amd.default_aggregator(dev)
    phases = {}
    orig_prepare = A.prepare
    orig_dev = A.DeviceAggregator._reduce_groups_device

    def timed_prepare(*a, **k):
        t0 = time.perf_counter()
        out = orig_prepare(*a, **k)
        phases["prepare_ms"] = (time.perf_counter() - t0) * 1e3
        return out

    def timed_dev(self, *a, **k):
        t0 = time.perf_counter()
        out = orig_dev(self, *a, **k)
        phases["issue_ms"] = (time.perf_counter() - t0) * 1e3
        return out

    A.prepare = timed_prepare
    A.DeviceAggregator._reduce_groups_device = timed_dev
    try:
        for name in args.configs:
            counts, dicts = device_clients(name, dev)
            recs = []
            for r in range(args.rounds):
                w_locals = [(n, OrderedDict(sd)) for n, sd in zip(counts, dicts)]  # :199's new dict objects
                torch.cuda.synchronize()
                phases.clear()
                t0 = time.perf_counter()
                out = agg.aggregate(w_locals)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                d = mfl_amd.client_distances(w_locals, out, device=dev)
                t3 = time.perf_counter()
                torch.cuda.synchronize()
                t4 = time.perf_counter()
                rec = {"config": name, "K": len(dicts), "keys": len(dicts[0]), "round": r,
                       "aggregate_wall_ms": round((t2 - t0) * 1e3, 4),
                       "aggregate_host_ms": round((t1 - t0) * 1e3, 4),
                       "distances_wall_ms": round((t4 - t2) * 1e3, 4),
                       "distances_host_ms": round((t3 - t2) * 1e3, 4),
                       "round_wall_ms": round((t4 - t0) * 1e3, 4),
                       **{k: round(v, 4) for k, v in phases.items()},
                       "distances_type": type(d).__name__}
                rec["rest_ms"] = round(rec["aggregate_host_ms"] - rec.get("prepare_ms", 0) - rec.get("issue_ms", 0), 4)
                recs.append(rec)
                print(json.dumps(rec), flush=True)
            tail = recs[2:] or recs
            summ = {"summary": True, "config": name}
            for k in ("aggregate_wall_ms", "aggregate_host_ms", "distances_wall_ms", "round_wall_ms", "prepare_ms",
                      "issue_ms", "rest_ms"):
                vals = [r[k] for r in tail if k in r]
                if vals:
                    summ[k] = round(float(np.median(vals)), 4)
            print(json.dumps(summ), flush=True)
            del dicts, out
            torch.cuda.empty_cache()
    finally:
        A.prepare = orig_prepare
        A.DeviceAggregator._reduce_groups_device = orig_dev


if __name__ == "__main__":
    main()
