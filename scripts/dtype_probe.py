"""Throughput of the exact fp32 / fp64 / fp16 / bf16 production kernels on the
BASELINE target shape (K = 100 clients x 25M elements), HIP events over
back-to-back launches, algorithmic bytes (K+1) * P * elem + K * wbytes."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import mfl_amd

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
P = int(sys.argv[2]) if len(sys.argv) > 2 else 25_000_000
n = np.random.default_rng(1234).integers(1, 1001, size=K)
wts = mfl_amd.sample_weights([int(v) for v in n])
for dt in (torch.float32, torch.float64, torch.float16, torch.bfloat16):
    ld = (P + 63) // 64 * 64
    x = (torch.randn((K, ld), device=dev) * 0.05).to(dt)
    w = mfl_amd.weights_tensor(wts, dt, dev)
    out = torch.empty(P, dtype=dt, device=dev)
    for _ in range(3):
        mfl_amd.reduce_packed(x, w, P, out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 10
    s.record()
    for _ in range(iters):
        mfl_amd.reduce_packed(x, w, P, out)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / iters
    eb = x.element_size()
    alg = (K + 1) * P * eb + K * w.element_size()
    print(json.dumps({"dtype": str(dt).replace("torch.", ""), "K": K, "P": P, "ms": round(ms, 4),
                      "GBps": round(alg / ms / 1e6, 1), "frac": round(alg / ms / 1e6 / 8000, 4)}), flush=True)
    del x
