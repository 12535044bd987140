"""A/B the FPF2 index pass (fedavg_trainer.py:272) in ONE process: the
one-block-per-row kernel (fedavg_fpf_index_f32) against the column-window
schedules (fedavg_fpf_index_variant), device-resident, interleaved.

    python scripts/fpf_index_variants.py [--n 1000] [--P 99990] [--rounds 5] [--iters 20]

One JSON line per variant: median us per call, GB/s of local_w_diffs read
(n * P * 4 bytes), max relative difference from the row kernel.
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
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--P", type=int, default=99_990)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    n, P = args.n, args.P
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(0)
    D = torch.randn((n, ld), generator=g, device=dev) * 0.01
    D[:, P:] = 0
    A = torch.rand(ld, generator=g, device=dev) + 0.5
    G = torch.rand(n, generator=g, device=dev) + 0.5
    ws_n = lib.fedavg_fpf_index_workspace(n, P)
    ws = torch.empty(ws_n, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    variants = [("row kernel", None)] + [
        (f"U{u} C{c} groups{gr}", (u, c, gr)) for u, c in [(4, 1), (8, 1), (16, 1), (8, 2), (4, 4), (8, 4), (4, 8)]
        for gr in (0, 8, 32)]
    outs = {name: torch.empty(n, device=dev) for name, _ in variants}

    def run(name, v):
        o = outs[name]
        if v is None:
            rc = lib.fedavg_fpf_index_f32(D.data_ptr(), n, ld, P, A.data_ptr(), G.data_ptr(), o.data_ptr(), s)
        else:
            rc = lib.fedavg_fpf_index_variant(D.data_ptr(), n, ld, P, A.data_ptr(), G.data_ptr(), o.data_ptr(),
                                              ws.data_ptr(), ws_n, v[0], v[1], v[2], s)
        mfl_amd._lib.check(rc, name)

    for name, v in variants:
        run(name, v)
    torch.cuda.synchronize()
    times = {name: [] for name, _ in variants}
    for _ in range(args.rounds):
        for name, v in variants:
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(args.iters):
                run(name, v)
            en.record()
            en.synchronize()
            times[name].append(st.elapsed_time(en) / args.iters)
    ref = outs["row kernel"].double().cpu()
    rows = []
    for name, v in variants:
        ms = float(np.median(times[name]))
        rel = float(((outs[name].double().cpu() - ref).abs() / ref.abs().clamp_min(1e-30)).max())
        rows.append({"variant": name, "n": n, "P": P, "us_median": round(ms * 1e3, 2),
                     "GBps": round(4 * n * P / ms / 1e6, 1), "max_rel_vs_row_kernel": rel})
    for r in sorted(rows, key=lambda r: r["us_median"]):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
