"""Can the streaming finish's reduce write the model straight into pinned host memory?

    python scripts/d2h_direct_probe.py [--K 100] [--P 25000000] [--reps 8]

The streaming finish (session.RoundSession.finish -> aggregate.reduce_and_fetch)
reduces the rows in column chunks into HBM and copies each chunk to the pinned
result on a D2H stream; on this system that copy is a runtime blit kernel that
shares the CUs with the next chunk's reduce (~2.7 ms at
100 x 25M).  This probe times, on the same resident rows:
  fetch  : the production chunked reduce + D2H (fused :291 sums included);
  direct : ONE fused launch whose output pointer IS the pinned host buffer
           (the kernel's stores cross PCIe as they are produced; no copy);
  direct_plain / dev_plain / dev_fused : the plain reduce into host memory and
           the device-only kernels, for scale.
Wall time per call (host clock, synchronised), medians over --reps after one
warm-up; the outputs' bits and the sums are compared with the production form.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

import mfl_amd
from mfl_amd import _lib
from mfl_amd.aggregate import reduce_and_fetch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    K, P = args.K, args.P
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    ld = (P + 63) // 64 * 64
    rows = torch.empty((K, ld), device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    for i in range(K):
        rows[i].normal_(0.0, 0.05, generator=g)
    counts = np.random.default_rng(1234).integers(1, 1001, K)
    w = torch.tensor([c / counts.sum() for c in counts], dtype=torch.float32, device=dev)
    cur = torch.cuda.current_stream(dev)
    d2h = torch.cuda.Stream(dev)
    host_a = torch.empty(P, pin_memory=True)
    host_b = torch.empty(P, pin_memory=True)
    host_c = torch.empty(P, pin_memory=True)
    out_dev = torch.empty(P, device=dev)
    n_ws = lib.fedavg_reduce_sqdist_workspace(K, P)
    work = torch.empty(max(n_ws, 1), dtype=torch.float64, device=dev)
    sums_b = torch.empty(K, dtype=torch.float64, device=dev)
    sums_d = torch.empty(K, dtype=torch.float64, device=dev)

    def fetch():
        sums = {}
        reduce_and_fetch(rows, w, P, d2h, out_host=host_a, sums=sums)
        d2h.synchronize()
        cur.synchronize()
        return sums[torch.float32]

    def fused(out_ptr, sums):
        _lib.check(lib.fedavg_reduce_sqdist_f32(rows.data_ptr(), K, P, ld, w.data_ptr(), out_ptr, work.data_ptr(),
                                                n_ws, sums.data_ptr(), cur.cuda_stream), "fedavg_reduce_sqdist_f32")
        cur.synchronize()

    def plain(out_ptr):
        _lib.check(lib.fedavg_reduce_f32(rows.data_ptr(), K, P, ld, w.data_ptr(), out_ptr, cur.cuda_stream),
                   "fedavg_reduce_f32")
        cur.synchronize()

    from mfl_amd.aggregate import column_chunks

    chunks = column_chunks(P)
    sums_parts = [torch.empty(K, dtype=torch.float64, device=dev) for _ in chunks]
    host_e = torch.empty(P, pin_memory=True)

    def direct_chunked():  # the finish's chunking (uploads pipeline per chunk), each chunk straight to host
        for (c0, c1), sp in zip(chunks, sums_parts):
            n = c1 - c0
            ws = lib.fedavg_reduce_sqdist_workspace(K, n)
            _lib.check(lib.fedavg_reduce_sqdist_f32(rows.data_ptr() + 4 * c0, K, n, ld, w.data_ptr(),
                                                    host_e.data_ptr() + 4 * c0, work.data_ptr(), ws, sp.data_ptr(),
                                                    cur.cuda_stream), "fedavg_reduce_sqdist_f32")
        cur.synchronize()

    legs = {
        "fetch": fetch,
        "direct_chunked": direct_chunked,
        "direct": lambda: fused(host_b.data_ptr(), sums_b),
        "dev_fused": lambda: fused(out_dev.data_ptr(), sums_d),
        "direct_plain": lambda: plain(host_c.data_ptr()),
        "dev_plain": lambda: plain(out_dev.data_ptr()),
    }
    times = {k: [] for k in legs}
    sums_a = None
    for r in range(args.reps + 1):
        for name, fn in legs.items():  # interleaved: every leg sees the same clock
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = fn()
            t = (time.perf_counter() - t0) * 1e3
            if name == "fetch":
                sums_a = res
            if r:
                times[name].append(t)
    rec = {"K": K, "P": P, "reps": args.reps}
    for name, ts in times.items():
        rec[f"{name}_ms_median"] = round(float(np.median(ts)), 4)
        rec[f"{name}_ms_min"] = round(float(np.min(ts)), 4)
    rec["direct_bits_equal"] = bool(torch.equal(host_a.view(torch.int32), host_b.view(torch.int32)))
    rec["direct_plain_bits_equal"] = bool(torch.equal(host_a.view(torch.int32), host_c.view(torch.int32)))
    rec["chunks"] = len(chunks)
    rec["direct_chunked_bits_equal"] = bool(torch.equal(host_a.view(torch.int32), host_e.view(torch.int32)))
    tot = sums_parts[0]
    for sp in sums_parts[1:]:
        tot = tot + sp
    rec["direct_chunked_sums_equal_fetch"] = bool(torch.equal(tot, sums_a))
    rec["direct_sums_max_rel"] = float(((sums_a - sums_b).abs() / sums_a.abs().clamp_min(1e-300)).max())
    rec["dev_sums_equal_direct"] = bool(torch.equal(sums_b, sums_d))
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
