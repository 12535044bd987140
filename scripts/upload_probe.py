"""Input distribution rate: one rank's P-shard of a
pinned host [K, P] client buffer uploaded with one strided DMA per column
segment (distributed.upload_segments -> fedavg_upload_shard), next to a
contiguous H2D of the same byte count.

    python scripts/upload_probe.py [--K 100] [--P 25000000] [--chunks 8] [--reps 5]

One JSON line per world size G in {1, 2, 4, 8}: rank 0's columns of the
block-cyclic plan (what each rank of a G-GPU node uploads over its own PCIe
link), GB/s = shard bytes / median time.
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
from mfl_amd.distributed import plan_shards, upload_segments


def timed(fn, reps):
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts[1:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--chunks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mfl_amd._lib.load()
    K, P = args.K, args.P
    host = torch.empty((K, P), dtype=torch.float32, pin_memory=True)
    host.view(-1)[::4096] = 1.0
    for G in (1, 2, 4, 8):
        plan = plan_shards(P, G, 0, 1 if G == 1 else args.chunks)
        segs = plan.local_segments()
        nbytes = 4 * K * sum(n for _, _, n in segs)
        dst = torch.empty((K, plan.local_cols), dtype=torch.float32, device=dev)
        t_2d = timed(lambda: upload_segments(dst, host, segs), args.reps)
        # checked before the contiguous copy below overwrites dst; compared as bits
        # (the pinned buffer is uninitialised, so it may hold NaN patterns)
        ok = all(torch.equal(dst[:, l:l + n][:, ::997].cpu().view(torch.int32),
                             host[:, g:g + n][:, ::997].view(torch.int32)) for l, g, n in segs)
        flat = dst.view(-1)[:nbytes // 4]
        src = host.view(-1)[:nbytes // 4]
        t_c = timed(lambda: flat.copy_(src, non_blocking=True), args.reps)
        print(json.dumps({"G": G, "K": K, "P": P, "chunks": plan.chunks, "segments": len(segs),
                          "shard_bytes": nbytes, "strided_ms": round(t_2d * 1e3, 3),
                          "strided_GBps": round(nbytes / t_2d / 1e9, 2), "contiguous_ms": round(t_c * 1e3, 3),
                          "contiguous_GBps": round(nbytes / t_c / 1e9, 2), "sampled_equal": ok}), flush=True)
        del dst


if __name__ == "__main__":
    main()
