"""fp16 / bf16 / fp64 reduce through buffer descriptors vs production.

    python scripts/vec_buf_probe.py [--K 100 --P 25000000] [--rounds 6] [--reps 4]

fedavg_reduce_vec_buf (tuning hook) against the production kernel
(mfl_amd.reduce_packed) on the same [K, ld] rows of each dtype, interleaved,
bit-identity checked.  One JSON line per (dtype, variant): median ms and GB/s
of algorithmic bytes (K*P*e + P*e + K*weight bytes).
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

CODES = {torch.float16: 0, torch.bfloat16: 1, torch.float64: 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--dtypes", nargs="*", default=["bfloat16", "float16", "float64"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    stream = torch.cuda.current_stream(dev).cuda_stream
    K, P = args.K, args.P
    for name in args.dtypes:
        dt = getattr(torch, name)
        e = torch.tensor([], dtype=dt).element_size()
        Pd = P if dt != torch.float64 else P // 2  # fp64: the same row bytes as fp32 at P
        ld = (Pd + 63) // 64 * 64
        g = torch.Generator(device=dev).manual_seed(11)
        x = (torch.randn((K, ld), generator=g, device=dev) * 0.05).to(dt)
        wdt = torch.float64 if dt == torch.float64 else torch.float32
        w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), wdt, dev)
        variants = {"production": None}
        for u, c, b in [(8, 4, 768), (4, 8, 768), (2, 16, 768), (2, 16, 0), (4, 4, 768)]:
            variants[f"buf-U{u}C{c}b{b}"] = (u, c, b)
        outs = {n: torch.empty(Pd, dtype=dt, device=dev) for n in variants}

        def run(n):
            v = variants[n]
            if v is None:
                mfl_amd.reduce_packed(x, w, Pd, outs[n])
                return
            mfl_amd._lib.check(lib.fedavg_reduce_vec_buf(CODES[dt], x.data_ptr(), K, Pd, ld, w.data_ptr(),
                                                         outs[n].data_ptr(), v[0], v[1], v[2], stream), n)

        for n in variants:
            run(n)
        torch.cuda.synchronize()
        iv = torch.int64 if dt == torch.float64 else torch.int16
        same = {n: bool(torch.equal(outs[n].view(iv), outs["production"].view(iv))) for n in variants}
        times = {n: [] for n in variants}
        for _ in range(args.rounds):
            for n in variants:
                for _ in range(args.reps):
                    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    run(n)
                    t.record()
                    times[n].append((s, t))
            torch.cuda.synchronize()
        alg = e * K * Pd + e * Pd + w.element_size() * K
        for n in variants:
            ms = float(np.median([s.elapsed_time(t) for s, t in times[n]]))
            print(json.dumps({"dtype": name, "variant": n, "K": K, "P": Pd, "ms_median": round(ms, 4),
                              "GBps": round(alg / ms / 1e6, 1), "bit_identical": same[n]}), flush=True)
        del x, outs


if __name__ == "__main__":
    main()
