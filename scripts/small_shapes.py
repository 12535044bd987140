"""Per-launch time of the exact kernel on small / latency-bound shapes
(back-to-back launches, HIP events), next to the split-client tolerance
variant: where does the sequential client chain, not HBM, set the time?"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import mfl_amd

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for K, P in [(10, 7850), (100, 7850), (1000, 7850), (100, 600_372), (1000, 600_372), (10, 1_206_590),
             (10000, 7850), (2, 100_000_000)]:
    ld = (P + 63) // 64 * 64
    x = torch.randn((K, ld), device=dev) * 0.05
    n = np.random.default_rng(1).integers(1, 1001, size=K)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights([int(v) for v in n]), torch.float32, dev)
    out = torch.empty(P, device=dev)
    res = {"K": K, "P": P, "MB": round(4 * K * P / 1e6, 1)}
    for name, kw in [("exact", {}), ("splitk4", {"splits": 4}), ("splitk8", {"splits": 8})]:
        for _ in range(3):
            mfl_amd.reduce_packed(x, w, P, out, **kw)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        iters = 50
        s.record()
        for _ in range(iters):
            mfl_amd.reduce_packed(x, w, P, out, **kw)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / iters
        res[f"{name}_us"] = round(ms * 1e3, 2)
        res[f"{name}_GBps"] = round((4 * K * P + 4 * P) / ms / 1e6, 1)
    print(json.dumps(res), flush=True)
    del x
