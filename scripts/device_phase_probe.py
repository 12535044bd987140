"""Where a device-resident round's host time goes, call by call.

    python scripts/device_phase_probe.py [--configs resnet56 target_flat] [--rounds 30]

Same round as scripts/host_cost_probe.py (clients' state_dicts in HBM, fresh
shallow dicts per round, :217 then :291), with perf_counter wrappers around
each step the drop-in takes on the host: the reference checks and native
walk (prepare / try_collect), the pointer-table gather, the int-key pre-pass,
the weights upload, the table workspace wait, each native library call, and
the result views.  One JSON line per round, then medians over rounds >= 3.
"""
from __future__ import annotations

import argparse
import inspect
import json
import sys
import time
from collections import OrderedDict, defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd
from host_cost_probe import device_clients

A = sys.modules[mfl_amd.DeviceAggregator.__module__]
L = sys.modules[A.KeyTable.__module__]
_lib = A._lib

acc = defaultdict(float)


def timed(name, fn):
    def wrap(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] += (time.perf_counter() - t0) * 1e3
    wrap.__wrapped__ = fn
    return wrap


def patch(obj, attr, name=None):
    raw = inspect.getattr_static(obj, attr) if isinstance(obj, type) else getattr(obj, attr)
    w = timed(name or attr, getattr(obj, attr))
    setattr(obj, attr, staticmethod(w) if isinstance(raw, staticmethod) else w)
    return (obj, attr, raw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["resnet56", "target_flat"])
    ap.add_argument("--rounds", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    agg = mfl_amd.default_aggregator(dev)
    lib = _lib.load()
    D = A.DeviceAggregator
    undo = []
    for obj, attr, name in [(A, "prepare", None), (L.KeyTable, "try_collect", None), (D, "_client_device", None),
                            (D, "_reduce_groups_device", None), (D, "_device_round", None),
                            (D, "_stage_ws", None), (L.KeyTable, "unpack_into", None),
                            (L.KeyTable, "forget_tensors", None), (A._Weights, "upload", "weights_upload")]:
        if hasattr(obj, attr):
            undo.append(patch(obj, attr, name))
    for fn in ("fedavg_device_round_f32", "fedavg_reduce_sqdist_segments_partials", "fedavg_device_round_workspace",
               "fedavg_device_round_scratch", "fedavg_reduce_segments_f32", "fedavg_pack_rows_device"):
        undo.append(patch(lib, fn, "lib." + fn))
    try:
        for name in args.configs:
            counts, dicts = device_clients(name, dev)
            recs = []
            for r in range(args.rounds):
                w_locals = [(n, OrderedDict(sd)) for n, sd in zip(counts, dicts)]
                torch.cuda.synchronize()
                acc.clear()
                t0 = time.perf_counter()
                out = agg.aggregate(w_locals)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                rec = {"config": name, "round": r, "aggregate_host_ms": round((t1 - t0) * 1e3, 4),
                       "aggregate_wall_ms": round((t2 - t0) * 1e3, 4),
                       **{k: round(v, 4) for k, v in acc.items()}}
                recs.append(rec)
                print(json.dumps(rec), flush=True)
            tail = recs[3:] or recs
            keys = sorted({k for r in tail for k in r if k not in ("config", "round")})
            summ = {"summary": True, "config": name, "K": len(dicts), "keys": len(dicts[0])}
            for k in keys:
                summ[k] = round(float(np.median([r.get(k, 0.0) for r in tail])), 4)
            print(json.dumps(summ), flush=True)
            del dicts, out, w_locals
            torch.cuda.empty_cache()
    finally:
        for obj, attr, orig in reversed(undo):
            setattr(obj, attr, orig)


if __name__ == "__main__":
    main()
