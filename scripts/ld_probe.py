"""Row pitch (ld) of the [K, ld] client rows vs the production reduce's rate.

    python scripts/ld_probe.py [--K 100 --P 25000000] [--rounds 4] [--reps 8]

The staging rows are padded to a multiple of 64 elements (256 B).  This
probe views one device buffer at several pitches (P rounded to 64, and +256 B
... +128 KiB of padding per row) and times the production exact reduce on
each, interleaved over --rounds rounds in one process: does the distance
between the clients' rows (their DRAM channel/bank mapping) change the read
stream's rate?  One JSON line per pitch; outputs must be bit-identical.
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
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--pads", nargs="*", type=int, default=[0, 64, 256, 1024, 4096, 32768])
    ap.add_argument("--fused", action="store_true",
                    help="also time the fused aggregate + :291 pass (reduce_with_sqdist) at every pitch")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, P = args.K, args.P
    base_ld = (P + 63) // 64 * 64
    pads = args.pads  # elements of padding per row
    buf = torch.empty(K * (base_ld + max(pads)), device=dev)
    g = torch.Generator(device=dev).manual_seed(1)
    src = torch.randn((K, P), generator=g, device=dev) * 0.05
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    outs, views = {}, {}
    for pad in pads:
        ld = base_ld + pad
        views[pad] = buf[:K * ld].view(K, ld)
        outs[pad] = torch.empty(P, device=dev)

    times = {pad: [] for pad in pads}
    ftimes = {pad: [] for pad in pads}
    ref = None
    for _ in range(args.rounds):
        for pad in pads:
            x = views[pad]
            x[:, :P].copy_(src)  # the same rows at this pitch
            mfl_amd.reduce_packed(x, w, P, outs[pad])  # warm-up / parity
            torch.cuda.synchronize()
            if ref is None:
                ref = outs[pad].clone()
            same = torch.equal(outs[pad].view(torch.int32), ref.view(torch.int32))
            for _ in range(args.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                mfl_amd.reduce_packed(x, w, P, outs[pad])
                e.record()
                times[pad].append((s, e, same))
            if args.fused:
                for _ in range(args.reps):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    o2, _ = mfl_amd.reduce_with_sqdist(x, w, P)
                    e.record()
                    ftimes[pad].append((s, e, torch.equal(o2.view(torch.int32), ref.view(torch.int32))))
            torch.cuda.synchronize()
    alg = 4 * K * P + 4 * P + 4 * K
    for pad in pads:
        ms = float(np.median([s.elapsed_time(e) for s, e, _ in times[pad]]))
        print(json.dumps({"ld": base_ld + pad, "pad_elems": pad, "row_pitch_bytes": 4 * (base_ld + pad), "K": K,
                          "P": P, "ms_median": round(ms, 4), "GBps": round(alg / ms / 1e6, 1),
                          "bit_identical": all(t[2] for t in times[pad])}), flush=True)
        if args.fused:
            fms = float(np.median([s.elapsed_time(e) for s, e, _ in ftimes[pad]]))
            print(json.dumps({"ld": base_ld + pad, "pad_elems": pad, "fused_ms_median": round(fms, 4),
                              "fused_GBps": round(alg / fms / 1e6, 1),
                              "fused_bit_identical": all(t[2] for t in ftimes[pad])}), flush=True)


if __name__ == "__main__":
    main()
