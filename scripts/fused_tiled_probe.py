"""Is the fused kernel's tile walk limited by the spread of its K row segments?

    python scripts/fused_tiled_probe.py [--K 100 --P 25000000] [--rounds 3] [--reps 6]

The same register-staged tile walk (reduce_sqdist_rs_kernel, probe codes of
fedavg_reduce_sqdist_f32_variant) over two layouts of the same values,
interleaved in one process:
  rows   [K, ld]              (the C ABI's layout: a tile's K row segments
                               are ld * 4 bytes apart, one per client row)
  tiled  [ceil(P/S)][K][S]    (a tile's K x S floats are contiguous)
Variants: full (average + sums), loads only, and the production fused kernel
and the row reduce on the row-major buffer as references.  One JSON line per
variant: median ms (HIP events), GB/s of the round's bytes counted once.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    probe = mfl_amd._lib.load_probe()
    K, P = args.K, args.P
    S = 64
    assert P % S == 0
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(K + P)
    x = torch.randn((K, ld), generator=g, device=dev) * 0.05
    xt = x[:, :P].reshape(K, P // S, S).permute(1, 0, 2).contiguous()  # [ntiles][K][S]
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    n_ws = K * 256 * 8
    work = torch.empty(n_ws, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs, sums = {}, {}

    def variant(code, buf, name):
        def run():
            o = outs.setdefault(name, torch.empty(P, device=dev))
            s = sums.setdefault(name, torch.empty(K, dtype=torch.float64, device=dev))
            mfl_amd._lib.check(probe.fedavg_reduce_sqdist_f32_variant(
                buf.data_ptr(), K, P, ld, w.data_ptr(), o.data_ptr(), work.data_ptr(), n_ws, s.data_ptr(), code, 0,
                stream), name, probe)
        return run

    def reduce_only():
        mfl_amd.reduce_packed(x, w, P, outs.setdefault("reduce-only", torch.empty(P, device=dev)))

    def fused():
        o, s = mfl_amd.reduce_with_sqdist(x, w, P, outs.setdefault("fused", torch.empty(P, device=dev)))
        sums["fused"] = s

    runs = {"reduce-only": reduce_only, "fused": fused,
            "rs-rows": variant(200064, x, "rs-rows"), "rs-tiled": variant(1200064, xt, "rs-tiled"),
            "rs-rows-loads": variant(300064, x, "rs-rows-loads"),
            "rs-tiled-loads": variant(1300064, xt, "rs-tiled-loads"),
            "rs-rows-loads-S128": variant(310128, x, "rs-rows-loads-S128"),
            "rs-tiled-loads-S128": variant(1310128, xt, "rs-tiled-loads-S128"),
            "rs-rows-xcd": variant(2200064, x, "rs-rows-xcd"), "rs-rows-xcd-loads": variant(2300064, x, "rs-rows-xcd-loads"),
            "rs-rows-cu": variant(4200064, x, "rs-rows-cu"), "rs-rows-cu-loads": variant(4300064, x, "rs-rows-cu-loads")}
    for fn in runs.values():
        fn()
    torch.cuda.synchronize()
    times = {n: [] for n in runs}
    for _ in range(args.rounds):
        for n, fn in runs.items():
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                times[n].append((a, b))
        torch.cuda.synchronize()
    ref = outs["reduce-only"].view(torch.int32)
    alg = 4 * K * P + 4 * P + 4 * K
    for n in runs:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[n]]))
        rec = {"K": K, "P": P, "variant": n, "ms_median": round(ms, 4), "round_GBps": round(alg / ms / 1e6, 1),
               "bit_identical_out": bool(torch.equal(outs[n].view(torch.int32), ref))}
        if n in sums and "fused" in sums:
            rec["sumsq_max_rel_vs_fused"] = float(((sums[n] - sums["fused"]).abs() / sums["fused"]).max().item())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
