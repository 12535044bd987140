"""A/B of fedavg_reduce_sqdist_f32 between the product library and an
alternate build of the same sources (a candidate change), interleaved in one
process on the same rows -- box-to-box variance cancels.

    python scripts/ab_fused_lib.py ALT.so [--shapes 100x25000000 ...] [--rounds 4] [--reps 6]

One JSON line per (shape, library): median ms (HIP events around each call)
and whether the averages and sums are bit-identical between the two builds.
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


def bind(path):
    lib = ctypes.CDLL(str(path))
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.fedavg_reduce_sqdist_workspace.restype = i64
    lib.fedavg_reduce_sqdist_workspace.argtypes = [i64, i64]
    lib.fedavg_reduce_sqdist_f32.restype = ctypes.c_int
    lib.fedavg_reduce_sqdist_f32.argtypes = [vp, i64, i64, i64, vp, vp, vp, i64, vp, vp]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("alt")
    ap.add_argument("--shapes", nargs="*", default=["100x25000000", "100x600372", "64x10000000", "20x25000000",
                                                      "200x10000000"])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    libs = {"product": bind(mfl_amd._lib.library_path() if hasattr(mfl_amd._lib, "library_path")
                            else mfl_amd._lib.LIB_PATH), "alt": bind(args.alt)}
    for shape in args.shapes:
        K, P = (int(v) for v in shape.split("x"))
        ld = (P + 63) // 64 * 64
        g = torch.Generator(device=dev).manual_seed(K + P)
        x = torch.randn((K, ld), generator=g, device=dev) * 0.05
        w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
        res = {}
        for name, lib in libs.items():
            n_ws = lib.fedavg_reduce_sqdist_workspace(K, P)
            res[name] = (torch.empty(P, device=dev), torch.empty(K, dtype=torch.float64, device=dev),
                         torch.empty(max(n_ws, 1), dtype=torch.float64, device=dev), n_ws)
        stream = torch.cuda.current_stream(dev).cuda_stream

        def run(name):
            o, s, ws, n_ws = res[name]
            rc = libs[name].fedavg_reduce_sqdist_f32(x.data_ptr(), K, P, ld, w.data_ptr(), o.data_ptr(), ws.data_ptr(),
                                                     n_ws, s.data_ptr(), stream)
            if rc:
                raise RuntimeError(f"{name}: rc {rc}")

        for name in libs:
            run(name)
        torch.cuda.synchronize()
        times = {n: [] for n in libs}
        for _ in range(args.rounds):
            for name in libs:
                for _ in range(args.reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    run(name)
                    b.record()
                    times[name].append((a, b))
            torch.cuda.synchronize()
        same_out = bool(torch.equal(res["product"][0].view(torch.int32), res["alt"][0].view(torch.int32)))
        same_sums = bool(torch.equal(res["product"][1], res["alt"][1]))
        for name in libs:
            ms = float(np.median([a.elapsed_time(b) for a, b in times[name]]))
            print(json.dumps({"K": K, "P": P, "lib": name, "ms_median": round(ms, 4), "out_bits_equal": same_out,
                              "sums_equal": same_sums}), flush=True)
        del x, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
