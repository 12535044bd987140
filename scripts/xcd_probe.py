"""XCD-aware workgroup order vs the production launch order.

    python scripts/xcd_probe.py [--K 100 --P 25000000] [--rounds 5] [--reps 10]

Runs the production exact reduce (U4 x C8 nt, round-split launches) and the
same kernel with an XCD-aware workgroup order (fedavg_reduce_f32_xcd: XCD x
takes one contiguous run of column slices instead of every 8th slice),
interleaved over --rounds rounds in one process, on the same buffer.  One
JSON line per variant: median time per call (HIP events) and GB/s of
algorithmic bytes; the outputs must be bit-identical.
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
    ap.add_argument("--rounds", type=int, default=5)
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
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    outs = {"production": torch.empty(P, device=dev), "xcd-aware": torch.empty(P, device=dev)}
    stream = torch.cuda.current_stream(dev)

    def run(name):
        if name == "production":
            mfl_amd.reduce_packed(x, w, P, outs[name])
        else:
            mfl_amd._lib.check(lib.fedavg_reduce_f32_xcd(x.data_ptr(), K, P, ld, w.data_ptr(), outs[name].data_ptr(),
                                                         0, stream.cuda_stream), "xcd")

    names = list(outs)
    for n in names:
        run(n)
    torch.cuda.synchronize()
    same = torch.equal(outs["production"].view(torch.int32), outs["xcd-aware"].view(torch.int32))
    times = {n: [] for n in names}
    for _ in range(args.rounds):
        for n in names:
            for _ in range(args.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run(n)
                e.record()
                times[n].append((s, e))
        torch.cuda.synchronize()
    alg = 4 * K * P + 4 * P + 4 * K
    for n in names:
        ms = float(np.median([s.elapsed_time(e) for s, e in times[n]]))
        print(json.dumps({"variant": n, "K": K, "P": P, "ms_median": round(ms, 4), "GBps": round(alg / ms / 1e6, 1),
                          "bit_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
