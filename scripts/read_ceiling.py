"""HBM read ceiling on this MI355X next to the production reduce.

    python scripts/read_ceiling.py [--gib 10] [--rounds 3] [--reps 10]

Streams one device buffer of the target's size (K=100 x P=25M fp32 = 10 GB)
with the read-only probe kernels (fedavg_probe_read_f32x4: grid-stride or
block-contiguous, nontemporal or default loads, several grid sizes and
launch splits) and runs the production exact reduce over the same bytes,
interleaved over --rounds rounds in one process.  One JSON line per variant:
median launch-sequence time (HIP events) and GB/s of bytes read.
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
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    K, P = args.K, args.P
    ld = (P + 63) // 64 * 64
    x = torch.empty((K, ld), device=dev)
    for k in range(K):
        x[k].normal_(0, 0.05)
    nvec = x.numel() // 4
    sink = torch.zeros(1 << 16, device=dev)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    out = torch.empty(P, device=dev)
    stream = torch.cuda.current_stream(dev)
    variants = [("reduce production", None)]
    for b in (1024, 2048, 4096, 8192, 16384):
        variants.append((f"probe grid-stride nt G{b}", (0, b, 1)))
    for b in (512, 763, 1024, 2048, 4096):
        variants.append((f"probe block-contig nt G{b}", (1, b, 1)))
    variants += [("probe block-contig nt G763 x4 launches", (1, 763, 4)),
                 ("probe block-contig nt G1018 x3 launches", (1, 1018, 3)),
                 ("probe block-contig default G1024", (2, 1024, 1)),
                 ("probe block-contig default G4096", (2, 4096, 1))]

    def run(v):
        if v is None:
            mfl_amd.reduce_packed(x, w, P, out)
        else:
            mode, blocks, launches = v
            mfl_amd._lib.check(lib.fedavg_probe_read_f32x4(x.data_ptr(), nvec, mode, blocks, launches,
                                                           sink.data_ptr(), stream.cuda_stream), "probe")

    times = {name: [] for name, _ in variants}
    for name, v in variants:  # warm-up
        run(v)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for name, v in variants:
            for _ in range(args.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run(v)
                e.record()
                times[name].append((s, e))
        torch.cuda.synchronize()
    for name, v in variants:
        ms = float(np.median([s.elapsed_time(e) for s, e in times[name]]))
        nbytes = 4 * K * P + 4 * P + 4 * K if v is None else 16 * nvec
        print(json.dumps({"variant": name, "ms_median": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                          "frac_of_8TBps": round(nbytes / ms / 1e6 / 8000, 4), "bytes": nbytes}), flush=True)


if __name__ == "__main__":
    main()
