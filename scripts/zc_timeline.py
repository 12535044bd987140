"""Per-wave timeline of the zero-copy split windows (reduce_sqdist_segwinf_kernel,
FEDAVG_SEGWINF_STAMPS=1: the MODE 8 build) on a resnet18_gn-shaped device round.

    python scripts/zc_timeline.py [--clients 129 257 500] [--calls 5]

Same stamps and summary as scripts/winn_timeline.py (the rows kernel), so the
two can be set side by side at one client count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

os.environ["FEDAVG_SEGWINF_STAMPS"] = "1"  # read once, at the library's first device round

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd
from host_cost_probe import device_clients
from winn_timeline import MAGIC, WINS, stamps_of, summarize


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="resnet18_gn")
    ap.add_argument("--clients", nargs="*", type=int, default=[129, 257, 500])
    ap.add_argument("--calls", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load()
    counts_all, dicts_all = device_clients(args.config, dev)
    for Kc in args.clients:
        counts, dicts = counts_all[:Kc], dicts_all[:Kc]
        table = mfl_amd.KeyTable(dicts[0])
        g = table.groups[torch.float32]
        ptrs, _ = table.collect(dicts, dev)
        K, n_cols = ptrs.shape
        ki = np.ascontiguousarray(g.key_index, dtype=np.int64)
        numel = np.ascontiguousarray(g.numel, dtype=np.int64)
        offset = np.ascontiguousarray(g.offset, dtype=np.int64)
        kind = np.ascontiguousarray(g.kind, dtype=np.int64)
        n = len(numel)
        total = sum(counts)
        w64 = np.array([c / total for c in counts], dtype=np.float64)
        out = torch.empty(g.P, device=dev)
        partials = torch.zeros(max(1, lib.fedavg_reduce_sqdist_segments_partials(K)), dtype=torch.float64, device=dev)
        sumsq = torch.empty(K, dtype=torch.float64, device=dev)
        scr = torch.empty(max(1, lib.fedavg_device_round_scratch(numel.ctypes.data, kind.ctypes.data, n, K)), device=dev)
        need = lib.fedavg_device_round_workspace(K, n)
        ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
        ws_d = torch.empty(need, dtype=torch.uint8, device=dev)
        ms = []
        for _ in range(args.calls):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.fedavg_device_round_f32(ptrs.ctypes.data, n_cols, ki.ctypes.data, numel.ctypes.data,
                                             offset.ctypes.data, kind.ctypes.data, n, K, w64.ctypes.data,
                                             out.data_ptr(), partials.data_ptr(), partials.numel(), sumsq.data_ptr(),
                                             scr.data_ptr(), scr.numel(), ws_h.data_ptr(), ws_d.data_ptr(), need, None)
            e1.record()
            e1.synchronize()
            mfl_amd._lib.check(rc if rc < 0 else 0, "device round", lib)
            ms.append(e0.elapsed_time(e1))
        wv = partials.view(torch.int64).cpu().numpy()
        G = next((g_ for g_ in range(1, 8193) if K * g_ < wv.size and wv[K * g_] == MAGIC), None)
        ns = (K + 63) // 64
        if G is None:
            print(json.dumps({"K": K, "error": "no stamp header (not the split windows?)", "rc": rc}), flush=True)
            continue
        nsmax = 8 if ns <= 8 else 16
        units = int(sum((int(v) + 63) // 64 for v in numel))
        st = stamps_of(wv, K, G, nsmax, ns)
        rec = {"K": K, "config": args.config, "grid": G, "windows_per_block": round(units / G, 1),
               "round_ms_median": round(float(np.median(ms)), 4),
               "cycles_median": summarize(st, ns, min(WINS, units // G))}
        print(json.dumps(rec), flush=True)
        del ptrs, out, partials
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
