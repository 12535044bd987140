"""Does a chunk's second read (the :291 squares) come from the Infinity Cache?

    python scripts/mall_reread_probe.py [--K 100] [--P 25000000] [--reps 5]

The fused aggregate + :291 pass holds every row of a window in registers
until the average is known (77 % of HBM peak at
100 x 25M, bound by two waves per SIMD).  The alternative is two passes per
column chunk small enough to stay in the 256 MB Infinity Cache (MALL): the
exact reduce of the chunk (default-policy loads, so the lines are allocated),
then the production :291 kernel over the same chunk, whose reads should hit
the cache.  This probe times, on the same resident rows (HIP events around
the whole 25M columns, medians over --reps, interleaved):
  fused   : fedavg_reduce_sqdist_f32, one launch (production);
  twopass : fedavg_reduce_f32 then fedavg_client_sqdist_f32 over all columns;
  pairs_W_ntX : per chunk of W columns, fedavg_reduce_f32_variant (U4 x C4,
           nontemporal X) then fedavg_client_sqdist_f32 on that chunk.
The averages' bits are compared with the fused pass; the sums to 1e-12 rel.
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

import mfl_amd  # noqa: F401
from mfl_amd import _lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--widths", default="262144,524288,1048576,2097152")
    args = ap.parse_args()
    K, P = args.K, args.P
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    probe = _lib.load_probe()
    ld = (P + 63) // 64 * 64
    rows = torch.empty((K, ld), device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    for i in range(K):
        rows[i].normal_(0.0, 0.05, generator=g)
    counts = np.random.default_rng(1234).integers(1, 1001, K)
    w = torch.tensor([c / counts.sum() for c in counts], dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    out_ref = torch.empty(P, device=dev)
    sums_ref = torch.empty(K, dtype=torch.float64, device=dev)
    n_ws = lib.fedavg_reduce_sqdist_workspace(K, P)
    work = torch.empty(max(n_ws, 1), dtype=torch.float64, device=dev)

    def fused():
        _lib.check(lib.fedavg_reduce_sqdist_f32(rows.data_ptr(), K, P, ld, w.data_ptr(), out_ref.data_ptr(),
                                                work.data_ptr(), n_ws, sums_ref.data_ptr(), s), "fused")

    out_t = torch.empty(P, device=dev)
    sums_t = torch.empty(K, dtype=torch.float64, device=dev)
    d_ws = lib.fedavg_client_sqdist_workspace(K, P)
    d_work = torch.empty(max(d_ws, 1), dtype=torch.float64, device=dev)

    def twopass():
        _lib.check(lib.fedavg_reduce_f32(rows.data_ptr(), K, P, ld, w.data_ptr(), out_t.data_ptr(), s), "reduce")
        _lib.check(lib.fedavg_client_sqdist_f32(rows.data_ptr(), K, P, ld, out_t.data_ptr(), d_work.data_ptr(), d_ws,
                                                sums_t.data_ptr(), s), "sqdist")

    legs = {"fused": (fused, out_ref, lambda: sums_ref), "twopass": (twopass, out_t, lambda: sums_t)}
    for W in [int(x) for x in args.widths.split(",")]:
        chunks = [(c0, min(P, c0 + W)) for c0 in range(0, P, W)]
        for nt in (0, 1):
            out_c = torch.empty(P, device=dev)
            parts = torch.empty((len(chunks), K), dtype=torch.float64, device=dev)
            c_ws = max(lib.fedavg_client_sqdist_workspace(K, c1 - c0) for c0, c1 in chunks)
            c_work = torch.empty(max(c_ws, 1), dtype=torch.float64, device=dev)

            def pairs(chunks=chunks, nt=nt, out_c=out_c, parts=parts, c_ws=c_ws, c_work=c_work):
                for j, (c0, c1) in enumerate(chunks):
                    n = c1 - c0
                    _lib.check(probe.fedavg_reduce_f32_variant(rows.data_ptr() + 4 * c0, K, n, ld, w.data_ptr(),
                                                               out_c.data_ptr() + 4 * c0, 4, nt, 4, 0, 0, s), "variant")
                    _lib.check(lib.fedavg_client_sqdist_f32(rows.data_ptr() + 4 * c0, K, n, ld,
                                                            out_c.data_ptr() + 4 * c0, c_work.data_ptr(), c_ws,
                                                            parts[j].data_ptr(), s), "sqdist chunk")

            legs[f"pairs_{W}_nt{nt}"] = (pairs, out_c, lambda parts=parts: parts.sum(0))
    times = {k: [] for k in legs}
    for r in range(args.reps + 1):
        for name, (fn, _, _) in legs.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1))
    rec = {"K": K, "P": P, "reps": args.reps}
    for name, (_, out, sums) in legs.items():
        rec[name] = {"ms_median": round(float(np.median(times[name])), 4), "ms_min": round(float(np.min(times[name])), 4),
                     "bits_equal": bool(torch.equal(out.view(torch.int32), out_ref.view(torch.int32))),
                     "sums_max_rel": float(((sums() - sums_ref).abs() / sums_ref.abs()).max())}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
