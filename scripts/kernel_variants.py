"""A/B every schedule variant of the exact fp32 kernel in ONE process,
interleaved round by round (CDNA guide rule 24), on device-resident inputs.

    python scripts/kernel_variants.py [--K 100 --P 25000000] [--rounds 5] [--iters 10]

Prints one JSON line per variant (median / min ms per launch, GB/s of
algorithmic bytes) sorted fastest first, and checks every variant's output is
bit-identical to the default kernel's.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

import mfl_amd
from mfl_amd import _lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--set", default="all", choices=["all", "focus", "wide", "window", "small"])
    ap.add_argument("--no-tiled", action="store_true")
    args = ap.parse_args()
    K, P = args.K, args.P
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _lib.load_probe()
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((K, ld), generator=g, device=dev) * 0.05
    ntiles = (P + 1023) // 1024
    tiled = None
    if args.set == "all" and not args.no_tiled:
        tiled = torch.zeros((ntiles, K, 1024), device=dev)
        full_cols = min(ntiles * 1024, ld) // 1024 * 1024
        tiled[: full_cols // 1024] = x[:, :full_cols].reshape(K, full_cols // 1024, 1024).permute(1, 0, 2)
        if full_cols < P:
            rem = P - full_cols
            tiled[full_cols // 1024, :, :rem] = x[:, full_cols:P]
    counts = np.random.default_rng(1234).integers(1, 1001, size=K)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights([int(c) for c in counts]), torch.float32, dev)
    stream = torch.cuda.current_stream().cuda_stream
    ref = mfl_amd.reduce_packed(x, w, P)

    variants = [("default", None)]
    if args.set == "small":
        for U, C in [(8, 1), (16, 1), (32, 1), (8, 2), (16, 2), (32, 2), (8, 4), (16, 4), (4, 8)]:
            for mb in (768, 100000):
                variants.append((f"split U{U} C{C} nt1 mb{mb}", (U, 1, C, 4, mb)))
        unrolls = []
    elif args.set == "window":
        for U, C in [(4, 8), (8, 8), (8, 4), (2, 16), (4, 4)]:
            for G in (512, 768, 1024):
                variants.append((f"window U{U} C{C} nt1 G{G}", (U, 1, C, 5, G)))
        for U, C, mb in [(4, 8, 768), (8, 8, 768), (8, 4, 512)]:
            variants.append((f"split U{U} C{C} nt1 mb{mb}", (U, 1, C, 4, mb)))
        unrolls = []
    elif args.set == "wide":
        for U, C in [(4, 8), (2, 8), (8, 8), (2, 16), (1, 16), (8, 4)]:
            for mb in (384, 512, 640, 768, 896, 1024, 1280):
                variants.append((f"split U{U} C{C} nt1 mb{mb}", (U, 1, C, 4, mb)))
        unrolls = []
    elif args.set == "focus":
        for U, C in [(8, 4), (4, 8), (8, 2), (8, 1)]:
            for nt in (0, 1):
                variants.append((f"var U{U} C{C} nt{nt} pipe0 mb0", (U, nt, C, 0, 0)))
        for U, C in [(8, 4), (4, 4), (4, 8), (8, 2)]:
            variants.append((f"bal U{U} C{C} nt1 mb0", (U, 1, C, 3, 0)))
        for U, C in [(4, 4), (2, 4), (8, 2), (4, 2), (8, 1), (16, 1), (2, 8)]:
            variants.append((f"glds U{U} C{C} nt1", (U, 1, C, 2, 0)))
        for U, C in [(2, 4), (4, 4), (8, 4), (16, 4), (2, 8), (4, 8), (8, 2), (16, 2), (4, 2), (8, 1), (16, 1)]:
            for nt in (0, 1):
                for mb in (0, 512, 768):
                    variants.append((f"split U{U} C{C} nt{nt} mb{mb}", (U, nt, C, 4, mb)))
        unrolls = []
    else:
        unrolls = None
    unrolls = ([8] if args.quick else [4, 8, 16]) if unrolls is None else unrolls
    for U in unrolls:
        for C in (1, 2, 4):
            for nt in (0, 1):
                for pipe in (0, 1):
                    if U == 16 and C == 4 and pipe:
                        continue  # spills
                    for mb in ((0,) if args.quick else (0, 2048)):
                        variants.append((f"var U{U} C{C} nt{nt} pipe{pipe} mb{mb}", (U, nt, C, pipe, mb)))
    if args.set == "all":
        for U in (2, 4):
            for nt in (0, 1):
                variants.append((f"var U{U} C8 nt{nt} pipe0 mb0", (U, nt, 8, 0, 0)))
        for U, C in [(2, 1), (4, 1), (8, 1), (16, 1), (2, 2), (4, 2), (8, 2), (2, 4), (4, 4), (2, 8)]:
            for nt in (0, 1):
                variants.append((f"glds U{U} C{C} nt{nt}", (U, nt, C, 2, 0)))
        variants.append(("tiled U8", ("tiled", 8)))

    outs = {}

    def launch(v, out):
        name, spec = v
        if spec is None:
            mfl_amd.reduce_packed(x, w, P, out)
        elif spec[0] == "tiled":
            _lib.check(lib.fedavg_reduce_tiled_f32(tiled.data_ptr(), K, P, w.data_ptr(), out.data_ptr(),
                                                   spec[1], stream), name)
        else:
            U, nt, C, pipe, mb = spec
            _lib.check(lib.fedavg_reduce_f32_variant(x.data_ptr(), K, P, ld, w.data_ptr(), out.data_ptr(),
                                                     U, nt, C, pipe, mb, stream), name)

    times = {v[0]: [] for v in variants}
    out = torch.empty(P, device=dev)
    for v in variants:  # warm-up + correctness
        out.zero_()
        launch(v, out)
        torch.cuda.synchronize()
        outs[v[0]] = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
    for r in range(args.rounds):
        order = variants if r % 2 == 0 else variants[::-1]
        for v in order:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                launch(v, out)
            e.record()
            e.synchronize()
            times[v[0]].append(s.elapsed_time(e) / args.iters)
    alg = 4 * K * P + 4 * P + 4 * K
    rows = []
    for name, ts in times.items():
        med = float(np.median(ts))
        rows.append({"variant": name, "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                     "GBps": round(alg / med / 1e6, 1), "frac_of_8TBps": round(alg / med / 1e6 / 8000, 4),
                     "bit_identical": outs[name], "K": K, "P": P})
    rows.sort(key=lambda r: r["ms_median"])
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
