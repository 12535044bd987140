"""Fused aggregate + :291 pass vs the two production passes, on the same rows.

    python scripts/fused_probe.py [--shapes 100x25000000 10x1206590 ...] [--rounds 4] [--reps 6]

Per shape, interleaved in one process:
  two-pass     fedavg_reduce_f32 then fedavg_client_sqdist_f32 on its output
               (what a round costs today: :217 then :291),
  reduce-only  fedavg_reduce_f32 alone (the floor for one read of the rows),
  fused        fedavg_reduce_sqdist_f32 (production rule),
  S<cols>b<n>  fedavg_reduce_sqdist_f32_variant (tile width, workgroups/CU).
Every fused form must give the reduce's bits and sums within 1e-12 of the
two-pass sums.  One JSON line per (shape, variant): median ms (HIP events),
GB/s of the ROUND's algorithmic bytes counted once (4KP + 4P + 4K: the rows
are read once by a fused pass, twice by the two passes).
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
    ap.add_argument("--shapes", nargs="*", default=["100x25000000", "10x1206590", "100x600372", "64x10000000",
                                                      "127x8000000", "20x25000000"])
    ap.add_argument("--variants", nargs="*", default=["64,0", "128,0", "256,0", "128,2", "64,4"])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    probe = mfl_amd._lib.load_probe()
    for shape in args.shapes:
        K, P = (int(v) for v in shape.split("x"))
        ld = (P + 63) // 64 * 64
        g = torch.Generator(device=dev).manual_seed(K + P)
        x = torch.randn((K, ld), generator=g, device=dev) * 0.05
        w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
        n_ws = max(K * 256 * 8, mfl_amd._lib.load().fedavg_reduce_sqdist_workspace(K, P))
        work = torch.empty(n_ws, dtype=torch.float64, device=dev)
        outs, sums = {}, {}

        def two_pass():
            o = mfl_amd.reduce_packed(x, w, P, outs.setdefault("two-pass", torch.empty(P, device=dev)))
            sums["two-pass"] = mfl_amd.client_sqdist(x, o, P)

        def reduce_only():
            mfl_amd.reduce_packed(x, w, P, outs.setdefault("reduce-only", torch.empty(P, device=dev)))

        def fused():
            o, s = mfl_amd.reduce_with_sqdist(x, w, P, outs.setdefault("fused", torch.empty(P, device=dev)))
            sums["fused"] = s

        def variant(cols, bpc, name):
            def run():
                o = outs.setdefault(name, torch.empty(P, device=dev))
                s = sums.setdefault(name, torch.empty(K, dtype=torch.float64, device=dev))
                mfl_amd._lib.check(probe.fedavg_reduce_sqdist_f32_variant(
                    x.data_ptr(), K, P, ld, w.data_ptr(), o.data_ptr(), work.data_ptr(), n_ws, s.data_ptr(), cols, bpc,
                    torch.cuda.current_stream(dev).cuda_stream), name, probe)
            return run

        runs = {"two-pass": two_pass, "reduce-only": reduce_only}
        if K <= 1024:
            runs["fused"] = fused
            for v in args.variants:
                cols, bpc = (int(t) for t in v.split(","))
                name = f"S{cols}b{bpc}"
                runs[name] = variant(cols, bpc, name)
        for n, fn in list(runs.items()):
            try:
                fn()
            except mfl_amd.FedAvgLibraryError as e:  # e.g. two tiles beyond the CU's LDS
                print(json.dumps({"K": K, "P": P, "variant": n, "skipped": str(e)}), flush=True)
                del runs[n]
        torch.cuda.synchronize()
        times = {n: [] for n in runs}
        for _ in range(args.rounds):
            for n, fn in runs.items():
                for _ in range(args.reps):
                    s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s0.record()
                    fn()
                    e0.record()
                    times[n].append((s0, e0))
            torch.cuda.synchronize()
        ref_out = outs["reduce-only"].view(torch.int32)
        ref_sum = sums["two-pass"]
        alg = 4 * K * P + 4 * P + 4 * K
        for n in runs:
            ms = float(np.median([a.elapsed_time(b) for a, b in times[n]]))
            rec = {"K": K, "P": P, "variant": n, "ms_median": round(ms, 4), "round_GBps": round(alg / ms / 1e6, 1),
                   "bit_identical_out": bool(torch.equal(outs[n].view(torch.int32), ref_out))}
            if n in sums:
                rec["sumsq_max_rel_vs_two_pass"] = float(((sums[n] - ref_sum).abs() / ref_sum).max().item())
            print(json.dumps(rec), flush=True)
        del x, work, outs, sums
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
