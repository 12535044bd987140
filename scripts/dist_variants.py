"""A/B the schedules of the :291 distance pass (fedavg_client_sqdist_variant)
in ONE process, interleaved, device-resident.

    python scripts/dist_variants.py [--K 100 --P 25000000] [--rounds 3] [--iters 5]

One JSON line per variant: median ms per call (both launches: the per-wave
partials and the fixed-order finalize), GB/s of algorithmic bytes (4KP + 4P
read), and the max relative difference of its fp64 sums from the production
schedule's (every schedule is deterministic; the wave partition changes the
fp64 summation order only).
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
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--glob", nargs="*", default=["4,8,0", "4,8,768"], help="U,C,max_blocks of the global form")
    ap.add_argument("--buf", nargs="*", default=["2,16,0", "2,16,512", "1,16,0", "1,16,768", "1,12,0", "2,12,0",
                                                 "2,12,512", "4,8,0", "2,8,0"],
                    help="U,C,max_blocks of the buffer-descriptor form")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    K, P = args.K, args.P
    ld = (P + 63) // 64 * 64
    x = torch.empty((K, ld), device=dev)
    for k in range(K):
        x[k].normal_(0, 0.05)
    glob = x[:, :P].mean(0).contiguous()
    n_ws = K * 4 * (((P + 3) // 4 + 255) // 256)  # per-wave partials at one 16-B slice per thread (the most)
    work = torch.empty(n_ws, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ap_glob = [tuple(int(t) for t in v.split(",")) for v in args.glob]
    ap_buf = [tuple(int(t) for t in v.split(",")) for v in args.buf]
    variants = [("production", None)] + [(f"U{u} C{c} mb{mb}", (u, c, mb)) for u, c, mb in ap_glob]
    # the buffer-descriptor form (fedavg_client_sqdist_buf)
    variants += [(f"buf U{u} C{c} mb{mb}", ("buf", u, c, mb)) for u, c, mb in ap_buf]
    outs = {name: torch.empty(K, dtype=torch.float64, device=dev) for name, _ in variants}

    def run(name, v):
        o = outs[name]
        if v is None:
            rc = lib.fedavg_client_sqdist_f32(x.data_ptr(), K, P, ld, glob.data_ptr(), work.data_ptr(), n_ws,
                                              o.data_ptr(), stream)
        elif v[0] == "buf":
            rc = lib.fedavg_client_sqdist_buf(x.data_ptr(), K, P, ld, glob.data_ptr(), work.data_ptr(), n_ws,
                                              o.data_ptr(), v[1], v[2], v[3], stream)
        else:
            rc = lib.fedavg_client_sqdist_variant(x.data_ptr(), K, P, ld, glob.data_ptr(), work.data_ptr(), n_ws,
                                                  o.data_ptr(), v[0], v[1], v[2], stream)
        mfl_amd._lib.check(rc, name)

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
    alg = 4 * K * P + 4 * P
    ref = outs["production"].cpu().numpy()
    rows = []
    for name, v in variants:
        ms = float(np.median(times[name]))
        rel = float(np.max(np.abs(outs[name].cpu().numpy() - ref) / np.abs(ref)))
        rows.append({"variant": name, "K": K, "P": P, "ms_median": round(ms, 4), "GBps": round(alg / ms / 1e6, 1),
                     "frac_of_8TBps": round(alg / ms / 1e6 / 8000, 4), "max_rel_vs_production": rel})
    for r in sorted(rows, key=lambda r: -r["GBps"]):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
