"""Where the time of a tiny drop-in call goes (MNIST-LR shape, K=10 x P=7,850).

    python scripts/small_e2e_probe.py [--reps 300]

Times, per call of DeviceAggregator.aggregate, the host phases with
perf_counter: prepare (weights, KeyTable, validation + pointer walk), pack +
H2D issue, reduce + D2H + sync, unpack; plus the reference's CPU loop on the
same inputs.  Medians in microseconds, one JSON line.
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
sys.path.insert(0, str(ROOT / "oracle"))

import numpy as np
import torch

import mfl_amd
A = sys.modules["mfl_amd.aggregate"]  # the module (the package re-exports a function of that name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--K", type=int, default=10)
    args = ap.parse_args()
    import fedavg_oracle as O

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator().manual_seed(0)
    shapes = [("linear.weight", (10, 784)), ("linear.bias", (10,))]
    dicts = [OrderedDict((k, torch.randn(s, generator=g) * 0.05) for k, s in shapes) for _ in range(args.K)]
    counts = list(range(100, 100 + args.K))
    agg = mfl_amd.DeviceAggregator(dev)
    phases = {"prepare": [], "reduce_groups": [], "total": [], "cpu_ref": []}
    orig_prepare, orig_reduce = A.prepare, A.DeviceAggregator._reduce_groups

    def t_prepare(*a, **k):
        t0 = time.perf_counter()
        r = orig_prepare(*a, **k)
        phases["prepare"].append(time.perf_counter() - t0)
        return r

    def t_reduce(self, *a, **k):
        t0 = time.perf_counter()
        r = orig_reduce(self, *a, **k)
        phases["reduce_groups"].append(time.perf_counter() - t0)
        return r

    A.prepare = t_prepare
    A.DeviceAggregator._reduce_groups = t_reduce
    prof = []
    phases.update({"native_one_call": [], "dropin_functional": []})
    fresh = lambda: [(counts[0], OrderedDict(dicts[0]))] + list(zip(counts[1:], dicts[1:]))  # noqa: E731
    for r in range(args.reps):
        wl = fresh()
        agg._fast_small = None  # the general path (prepare + _reduce_groups)
        t0 = time.perf_counter()
        agg.aggregate(wl)
        phases["total"].append(time.perf_counter() - t0)
        prof.append(dict(agg.last_profile))
        wl = fresh()  # the next round: the native one-call path (fedavg_collect_ext.small_round)
        t0 = time.perf_counter()
        out = agg.aggregate(wl)
        phases["native_one_call"].append(time.perf_counter() - t0)
        assert out is wl[0][1]
        wl = fresh()  # what install()'d FedAvgTrainer.aggregate runs: the functional form
        t0 = time.perf_counter()
        mfl_amd.aggregate(wl, device=dev)
        phases["dropin_functional"].append(time.perf_counter() - t0)
        wl2 = fresh()
        t0 = time.perf_counter()
        O.aggregate_torch(wl2)
        phases["cpu_ref"].append(time.perf_counter() - t0)
    out = {k: round(float(np.median(v[10:])) * 1e6, 1) for k, v in phases.items()}
    out["native_fast_rounds"] = agg.fast_rounds
    out["dropin_vs_cpu"] = round(out["cpu_ref"] / out["dropin_functional"], 3)
    for k in prof[0]:
        out[k + "_us"] = round(float(np.median([p[k] for p in prof[10:]])) * 1e3, 1)
    out["K"] = args.K
    out["P"] = 7850
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
