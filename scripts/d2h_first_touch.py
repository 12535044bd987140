"""Why the first rounds of the DMA D2H engine are slow.

    python scripts/d2h_first_touch.py [--mb 100] [--bufs 4]

Each round of the drop-in copies the averaged model into a NEW pinned host
buffer (the result views keep the previous one alive).  This probe separates
the costs on fresh and reused pinned buffers of the target's output size:
the pinned allocation itself (torch's caching host allocator), the first
copy into a buffer and later copies into it, for both engines of
fedavg_copy_to_host (0 = hipMemcpyAsync DMA, 64 = zero-copy kernel).
One JSON line per measurement (wall ms around the call + stream sync).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch

import mfl_amd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=100)
    ap.add_argument("--bufs", type=int, default=4)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load()
    n = args.mb * 1_000_000 // 4
    src = torch.randn(n, device=dev)
    s = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()

    def copy(dst, blocks):
        t0 = time.perf_counter()
        mfl_amd._lib.check(lib.fedavg_copy_to_host(src.data_ptr(), dst.data_ptr(), n * 4, blocks, s.cuda_stream), "d2h")
        s.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for blocks in (0, 64):
        keep = []
        for b in range(args.bufs):
            t0 = time.perf_counter()
            dst = torch.empty(n, dtype=torch.float32, pin_memory=True)
            alloc = (time.perf_counter() - t0) * 1e3
            first = copy(dst, blocks)
            again = [copy(dst, blocks) for _ in range(3)]
            ok = torch.equal(dst, src.cpu())
            keep.append(dst)  # live, like the previous rounds' results
            print(json.dumps({"engine": "dma" if blocks == 0 else f"kernel{blocks}", "buffer": b,
                              "pinned_alloc_ms": round(alloc, 3), "first_copy_ms": round(first, 3),
                              "later_copies_ms": [round(a, 3) for a in again], "MB": args.mb, "correct": ok}),
                  flush=True)
        del keep
        # freed buffers go back to torch's pinned cache: the next allocation reuses one
        t0 = time.perf_counter()
        dst = torch.empty(n, dtype=torch.float32, pin_memory=True)
        alloc = (time.perf_counter() - t0) * 1e3
        first = copy(dst, blocks)
        print(json.dumps({"engine": "dma" if blocks == 0 else f"kernel{blocks}", "buffer": "recycled",
                          "pinned_alloc_ms": round(alloc, 3), "first_copy_ms": round(first, 3), "MB": args.mb}),
              flush=True)
        del dst


if __name__ == "__main__":
    main()
