"""The :291 distance pass on device-resident clients (zero-copy segments) by schedule.

    python scripts/segments_dist_probe.py --model resnet56 [--sched 4,1 4,4 ...] [--rounds 6 --reps 10]

K separately allocated device state_dicts of a scripts/model_shapes.py model;
fedavg_client_sqdist_segments_f32 (production) against
fedavg_client_sqdist_segments_f32_variant (U, C) schedules, interleaved; the
per-client sums must agree to 1e-12 relative (the fp64 partial grouping
depends on the unit size).  One JSON line per variant: median ms per call
(HIP events, table staging included) -- run under rocprofv3 --stats for the
kernel time alone.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd
from model_shapes import CONFIGS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet56")
    ap.add_argument("--sched", nargs="*", default=["1,4", "4,4", "8,4", "4,1", "8,1", "4,2", "8,2", "4,8"])
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    K, shapes = CONFIGS[args.model]
    g = torch.Generator(device=dev).manual_seed(9)
    clients = [[torch.randn(shp, generator=g, device=dev) * 0.05 for _, shp in shapes] for _ in range(K)]
    numel = np.array([t.numel() for t in clients[0]], dtype=np.int64)
    offset = np.concatenate([[0], np.cumsum(numel)[:-1]]).astype(np.int64)
    kind = np.zeros(len(numel), dtype=np.int64)
    ptrs = np.array([[t.data_ptr() for t in sd] for sd in clients], dtype=np.int64)
    P, nk = int(numel.sum()), len(numel)
    glob = torch.randn(P, generator=g, device=dev) * 0.05
    need = lib.fedavg_segments_workspace(K, nk)
    max_parts = K * 4 * int(sum((n + 1023) // 1024 for n in numel))  # the narrowest units
    stream = torch.cuda.current_stream(dev)
    variants = [None] + [tuple(int(t) for t in v.split(",")) for v in args.sched]
    names = ["production" if v is None else f"U{v[0]}C{v[1]}" for v in variants]
    bufs = {n: (torch.empty(need, dtype=torch.uint8, pin_memory=True), torch.empty(need, dtype=torch.uint8, device=dev),
                torch.empty(max_parts, dtype=torch.float64, device=dev), torch.empty(K, dtype=torch.float64, device=dev))
            for n in names}
    a = (ptrs.ctypes.data, numel.ctypes.data, offset.ctypes.data, kind.ctypes.data, nk, K, glob.data_ptr())

    def run(n, v):
        h, d, parts, sumsq = bufs[n]
        if v is None:
            rc = lib.fedavg_client_sqdist_segments_f32(*a, parts.data_ptr(), parts.numel(), sumsq.data_ptr(),
                                                       h.data_ptr(), d.data_ptr(), need, stream.cuda_stream)
        else:
            rc = lib.fedavg_client_sqdist_segments_f32_variant(*a, parts.data_ptr(), parts.numel(), sumsq.data_ptr(),
                                                               h.data_ptr(), d.data_ptr(), need, v[0], v[1],
                                                               stream.cuda_stream)
        mfl_amd._lib.check(rc, n, lib)

    for n, v in zip(names, variants):
        run(n, v)
    torch.cuda.synchronize()
    ref = bufs["production"][3].cpu().numpy()
    rel = {n: float(np.max(np.abs(bufs[n][3].cpu().numpy() - ref) / np.abs(ref))) for n in names}
    times = {n: [] for n in names}
    for _ in range(args.rounds):
        for n, v in zip(names, variants):
            for _ in range(args.reps):
                s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                run(n, v)
                e0.record()
                times[n].append((s0, e0))
            torch.cuda.synchronize()  # the pinned table of the next call
    alg = 4 * K * P + 4 * P
    for n in names:
        ms = float(np.median([s0.elapsed_time(e0) for s0, e0 in times[n]]))
        print(json.dumps({"model": args.model, "variant": n, "K": K, "P": P, "keys": nk, "ms_median": round(ms, 4),
                          "GBps": round(alg / ms / 1e6, 1), "max_rel_vs_production": rel[n]}), flush=True)
        assert rel[n] <= 1e-12, (n, rel[n])


if __name__ == "__main__":
    main()
