"""Which engine moves a device -> pinned-host copy, by host allocation kind.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o d2h \
        -- python scripts/d2h_engine_probe.py [--mb 12.5] [--reps 10]

A streaming round's finish (aggregate.reduce_and_fetch) overlaps chunk c's
D2H with chunk c+1's reduce.  The rocprofv3 timeline of that finish shows
every D2H as a runtime blit KERNEL (__amd_rocclr_copyBuffer) running beside
the reduce, both ~2x slower than alone.  This probe copies the same device
buffer into host memory allocated four ways -- torch's pinned tensor,
hipHostMalloc default / non-coherent / write-combined, and a pageable buffer
registered with hipHostRegister -- each with its own byte count so the trace
tells them apart, and with the runtime copy kind and the NoCU kind.  Prints
one JSON line per (allocation, kind): bytes, median copy time (HIP events),
GB/s.
"""
from __future__ import annotations

import argparse
import ctypes
import json

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=12.5)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    hip = ctypes.CDLL("libamdhip64.so")
    base = int(args.mb * 1e6) // 4096 * 4096
    src = torch.randn(base // 4 + 8192, device=dev)
    stream = torch.cuda.current_stream(dev)
    kinds = {"d2h": 2, "nocu": 1024}
    allocs = []
    t = torch.empty(base + 65536, dtype=torch.uint8, pin_memory=True)
    allocs.append(("torch_pinned", t.data_ptr(), t))
    for name, flags in (("hostmalloc_default", 0x0), ("hostmalloc_noncoherent", 0x80000000),
                        ("hostmalloc_wc", 0x4)):
        p = ctypes.c_void_p()
        rc = hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(base + 65536), ctypes.c_uint(flags))
        if rc == 0:
            allocs.append((name, p.value, None))
    pageable = np.empty(base + 65536, dtype=np.uint8)
    rc = hip.hipHostRegister(ctypes.c_void_p(pageable.ctypes.data), ctypes.c_size_t(pageable.nbytes), ctypes.c_uint(0))
    if rc == 0:
        allocs.append(("host_register", pageable.ctypes.data, pageable))
    for i, (name, ptr, _) in enumerate(allocs):
        for j, (kname, kind) in enumerate(kinds.items()):
            nbytes = base + (i * len(kinds) + j) * 4096  # a distinct size per variant: tells them apart in the trace
            ts = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                rc = hip.hipMemcpyAsync(ctypes.c_void_p(ptr), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(nbytes),
                                        ctypes.c_int(kind), ctypes.c_void_p(stream.cuda_stream))
                b.record(stream)
                if rc != 0:
                    break
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
            ms = float(np.median(ts)) if ts else None
            print(json.dumps({"alloc": name, "kind": kname, "bytes": nbytes, "rc": rc,
                              "ms_median": None if ms is None else round(ms, 4),
                              "GBps": None if not ms else round(nbytes / ms / 1e6, 1)}), flush=True)
    torch.cuda.synchronize()
    for name, ptr, _ in allocs:
        if name.startswith("hostmalloc"):
            hip.hipHostFree(ctypes.c_void_p(ptr))
    if any(n == "host_register" for n, _, _ in allocs):
        hip.hipHostUnregister(ctypes.c_void_p(pageable.ctypes.data))


if __name__ == "__main__":
    main()
