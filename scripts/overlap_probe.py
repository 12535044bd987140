"""Does a collective-sized kernel find CUs while the reduce runs?  (1 GPU)

    python scripts/overlap_probe.py [--K 100] [--cols 25000000] [--reps 8]
                                    [--hold-us 0] [--copy-frac 1.0]

Mimics one rank of the N=8 P-sharded step on a single MI355X: the exact
reduce over C column chunks on the compute stream and, after each chunk, a
stand-in for RCCL's all-gather kernel on a side stream ordered after that
chunk's reduce.  The stand-in (fedavg_probe_busy_copy) holds ~294 registers
per wave like RCCL's generic kernel on gfx950 (261 VGPR + 17 AGPR in its code
object) and copies the 7/8 x chunk bytes one rank receives at N = 8 (times
--copy-frac), then stays resident until --hold-us / C microseconds after it
started: with a small copy fraction and a hold it behaves like a collective
bound by xGMI rather than HBM (resident, waiting, light on HBM).  A wave
that size fits on a SIMD only next to <= 218 registers of other waves, so
whether it can run beside the reduce depends on the reduce's registers per
wave x waves per SIMD.

For each chunk count, reduce schedule and side-stream priority: the reduce
alone, the copy alone, and both (median ms per step).  One JSON line each.
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
    ap.add_argument("--cols", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--copy-blocks", default="32,64")
    ap.add_argument("--hold-us", type=int, default=0, help="per step, split over the chunks")
    ap.add_argument("--copy-frac", type=float, default=1.0)
    ap.add_argument("--chunk-list", default="4,8")
    ap.add_argument("--production-only", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    K = args.K
    cols = (args.cols + 511) // 512 * 512
    x = torch.empty((K, cols), device=dev)
    for k in range(K):
        x[k].normal_(0, 0.05)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    out = torch.empty(cols, device=dev)
    ref = mfl_amd.reduce_packed(x, w, cols).clone()
    src = torch.ones(7 * cols // 4 + 64, device=dev)
    dst = torch.empty_like(src)

    def mk(prio):
        h = ctypes.c_void_p()
        mfl_amd._lib.check(lib.fedavg_stream_create_masked(0, prio, ctypes.byref(h)), "stream")
        return torch.cuda.ExternalStream(h.value, device=dev)

    comp, side_lo, side_hi = mk(0), mk(0), mk(-1)

    def step(C, tuned, side, legs, copy_blocks):
        S = cols // C
        cbytes = int(7 * S * 4 * args.copy_frac) // 16 * 16
        for c in range(C):
            with torch.cuda.stream(comp):
                if "r" in legs:
                    mfl_amd.reduce_packed(x[:, c * S:(c + 1) * S], w, S, out[c * S:(c + 1) * S], tuned=tuned)
                ev = torch.cuda.Event()
                ev.record(comp)
            if "c" in legs:
                side.wait_event(ev)
                mfl_amd._lib.check(lib.fedavg_probe_busy_copy(src.data_ptr(), dst.data_ptr(), cbytes, copy_blocks,
                                                              args.hold_us // C, side.cuda_stream), "copy")
        torch.cuda.current_stream().wait_stream(comp)
        torch.cuda.current_stream().wait_stream(side)

    configs = []
    for C in [int(c) for c in args.chunk_list.split(",")]:
        S = cols // C
        prod = mfl_amd._lib.f32_schedule(K, S)
        scheds = [("production U%d C%d mb768" % (prod["unroll"], prod["cols"]), None),
                  ("U2 C4 mb512", (2, 1, 4, 4, 512)), ("U2 C4 mb768", (2, 1, 4, 4, 768)),
                  ("U2 C8 mb768", (2, 1, 8, 4, 768)), ("U4 C4 mb512", (4, 1, 4, 4, 512))]
        if args.production_only:
            scheds = scheds[:1]
        for sname, tuned in scheds:
            configs.append((C, sname, tuned))
    rows = []
    for cb in [int(b) for b in args.copy_blocks.split(",")]:
        for C, sname, tuned in configs:
            legsets = [("reduce_only", "r", side_lo), ("copy_only", "c", side_lo), ("overlap", "rc", side_lo),
                       ("overlap_hiprio", "rc", side_hi)]
            for _, legs, side in legsets:  # warm-up
                step(C, tuned, side, legs, cb)
            torch.cuda.synchronize()
            res = {name: [] for name, _, _ in legsets}
            for _ in range(args.reps):
                for name, legs, side in legsets:
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    step(C, tuned, side, legs, cb)
                    e.record()
                    e.synchronize()
                    res[name].append(s.elapsed_time(e))
            assert torch.equal(out, ref), "reduce result changed"
            r = {k: round(float(np.median(v)), 4) for k, v in res.items()}
            serial = r["reduce_only"] + r["copy_only"]
            row = {"chunks": C, "schedule": sname, "copy_blocks": cb, "hold_us": args.hold_us,
                   "copy_frac": args.copy_frac, **r,
                   "hidden_frac": round((serial - r["overlap"]) / min(r["reduce_only"], r["copy_only"]), 3),
                   "hidden_frac_hiprio": round((serial - r["overlap_hiprio"]) / min(r["reduce_only"], r["copy_only"]), 3)}
            rows.append(row)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
