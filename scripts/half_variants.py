"""A/B the packed fp16/bf16 exact kernel's schedules in ONE process,
interleaved (CDNA guide rule 24), device-resident.

    python scripts/half_variants.py [--K 100 --P 25000000] [--dtype bf16] [--rounds 3] [--iters 10]

One JSON line per variant: median ms per call, GB/s of algorithmic bytes
((K+1)*P*2 + 4K), and whether its output is bit-identical to the production
kernel's (fedavg_reduce_bf16 / _f16).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
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
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    K, P = args.K, args.P
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    ld = (P + 63) // 64 * 64
    x = torch.empty((K, ld), dtype=dt, device=dev)
    for k in range(K):
        x[k].normal_(0, 0.05)
    counts = np.random.default_rng(1234).integers(1, 1001, size=K)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights([int(c) for c in counts]), torch.float32, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ref = mfl_amd.reduce_packed(x, w, P)
    vals = [ctypes.c_int() for _ in range(4)]
    mfl_amd._lib.check(lib.fedavg_half_schedule(K, P, *[ctypes.byref(v) for v in vals]), "schedule")
    prod = dict(zip(("unroll", "cols", "nontemporal", "launches"), (v.value for v in vals)))
    variants = [("production " + json.dumps(prod), None)]
    for U, C in [(1, 8), (2, 8), (4, 8), (2, 4), (4, 4), (8, 4), (4, 2), (8, 2), (1, 16), (2, 16), (16, 1)]:
        for mb in (512, 768, 1024, 0):
            variants.append((f"U{U} C{C} mb{mb}", (U, C, mb)))
    outs = {}

    def run(name, v):
        if v is None:
            return mfl_amd.reduce_packed(x, w, P, out=outs.setdefault(name, torch.empty(P, dtype=dt, device=dev)))
        o = outs.setdefault(name, torch.empty(P, dtype=dt, device=dev))
        U, C, mb = v
        mfl_amd._lib.check(lib.fedavg_reduce_half_variant(1 if dt == torch.bfloat16 else 0, x.data_ptr(), K, P, ld,
                                                          w.data_ptr(), o.data_ptr(), U, C, mb, stream), name)
        return o

    for name, v in variants:
        run(name, v)
    torch.cuda.synchronize()
    times = {name: [] for name, _ in variants}
    for _ in range(args.rounds):
        for name, v in variants:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                run(name, v)
            e.record()
            e.synchronize()
            times[name].append(s.elapsed_time(e) / args.iters)
    alg = (K + 1) * P * 2 + 4 * K
    rows = []
    for name, v in variants:
        ms = float(np.median(times[name]))
        same = torch.equal(outs[name].view(torch.int16), ref.view(torch.int16))
        rows.append({"variant": name, "dtype": args.dtype, "K": K, "P": P, "ms_median": round(ms, 4),
                     "GBps": round(alg / ms / 1e6, 1), "frac_of_8TBps": round(alg / ms / 1e6 / 8000, 4),
                     "bit_identical": bool(same)})
    for r in sorted(rows, key=lambda r: -r["GBps"]):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
