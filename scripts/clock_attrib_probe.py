"""Time AND shader clock of the K = 100 fused window beside its variants, in
ONE process, interleaved (round 6: settles whether the fused pass's deficit
against the plain reduce is clock or cycles).

    python scripts/clock_attrib_probe.py [--K 100 --P 25000000] [--rounds 4] [--reps 6]

Variants (all on the same resident [K, ld] rows):
  reduce        fedavg_reduce_f32 alone (the bench's kernel)
  fused         the production plan (reduce_sqdist_win_kernel<100,2,4,64>: fp64 squares)
  fp32_squares  the same kernel with its squares in fp32 (MODE 4 + 64, probe: sums differ)
  loads_only    the same grid and loads, no chain, no squares (MODE 1 + 64, probe: wrong results)

Per variant: median ms over rounds x reps (HIP events around each call);
then, in interleaved passes, the clock the chip holds under back-to-back
calls (bench.shader_clock_mhz: d(s_memtime)/d(s_memrealtime) on a side
stream) together with those same calls' time, so every pass gives one
(time, clock) pair from one window and cycles per call = ms x MHz of that
pair; and the fp32-squares sums' max relative difference from the fp64 ones.
One JSON line per variant, then a summary line.
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

import bench
import mfl_amd

CODES = {"fused_mode64": 60000000 + 64 * 1000000 + 42, "fp32_squares": 60000000 + 68 * 1000000 + 42,
         "loads_only": 60000000 + 65 * 1000000 + 42}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--clock-calls", type=int, default=30)
    ap.add_argument("--clock-passes", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    probe = mfl_amd._lib.load_probe()
    K, P = args.K, args.P
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(K + P)
    x = torch.randn((K, ld), generator=g, device=dev) * 0.05
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    n_ws = max(K * 256 * 8 * 4, mfl_amd._lib.load().fedavg_reduce_sqdist_workspace(K, P))
    work = torch.empty(n_ws, dtype=torch.float64, device=dev)
    outs = {n: torch.empty(P, device=dev) for n in ("reduce", "fused", *CODES)}
    sums = {n: torch.empty(K, dtype=torch.float64, device=dev) for n in ("fused", *CODES)}
    stream = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731

    def variant(name):
        code = CODES[name]

        def run():
            mfl_amd._lib.check(probe.fedavg_reduce_sqdist_f32_variant(
                x.data_ptr(), K, P, ld, w.data_ptr(), outs[name].data_ptr(), work.data_ptr(), n_ws,
                sums[name].data_ptr(), code, 0, stream()), name, probe)
        return run

    def fused():
        _, s = mfl_amd.reduce_with_sqdist(x, w, P, outs["fused"])
        sums["fused"].copy_(s)

    runs = {"reduce": lambda: mfl_amd.reduce_packed(x, w, P, outs["reduce"]), "fused": fused}
    runs.update({n: variant(n) for n in CODES})
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
    clocks, pair_ms = {}, {}
    for _ in range(args.clock_passes):  # interleaved passes of the clock probe, each timing its own calls
        for n, fn in runs.items():
            c = bench.shader_clock_mhz(fn, calls=args.clock_calls)
            clocks.setdefault(n, []).append(c["clock_mhz"])
            pair_ms.setdefault(n, []).append(c["ms_per_call_in_window"])
    alg = 4 * K * P + 4 * P + 4 * K
    ref = outs["reduce"].view(torch.int32)
    summary = {}
    for n in runs:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[n]]))
        mhz = float(np.median(clocks[n]))
        # cycles from (time, clock) pairs measured over the same window of calls
        cyc = [m * c / 1e3 for m, c in zip(pair_ms[n], clocks[n])]
        rec = {"K": K, "P": P, "variant": n, "ms_median": round(ms, 4), "GBps": round(alg / ms / 1e6, 1),
               "frac_of_8TBps": round(alg / ms / 1e6 / 8000.0, 4), "clock_mhz": mhz, "clock_samples": clocks[n],
               "window_ms_samples": pair_ms[n], "mcycles_per_call": round(float(np.median(cyc)), 3),
               "mcycles_samples": [round(x, 3) for x in cyc],
               "out_bits_equal_reduce": bool(torch.equal(outs[n].view(torch.int32), ref))}
        if n in sums and n not in ("fused", "loads_only"):
            rec["sums_max_rel_vs_fused"] = float(((sums[n] - sums["fused"]).abs() / sums["fused"].abs()).max())
        summary[n] = (float(np.median(pair_ms[n])), mhz, float(np.median(cyc)))
        print(json.dumps(rec), flush=True)
    base_ms, base_mhz, base_cyc = summary["reduce"]
    print(json.dumps({"summary": {n: {"window_ms_over_reduce": round(ms / base_ms, 4),
                                      "clock_over_reduce": round(mhz / base_mhz, 4),
                                      "cycles_over_reduce": round(cyc / base_cyc, 4)}
                                  for n, (ms, mhz, cyc) in summary.items()}}), flush=True)


if __name__ == "__main__":
    main()
