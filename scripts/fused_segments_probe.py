"""Device-resident round (zero-copy, separate client tensors): aggregate + :291
as two passes (fedavg_reduce_segments_f32 + fedavg_client_sqdist_segments_f32)
vs the fused pass (fedavg_reduce_sqdist_segments_f32), through the drop-in.

    python scripts/fused_segments_probe.py [--configs flat resnet56 femnist] [--reps 10]

One JSON line per (config, mode): median ms of aggregate + client_distances
on the device (HIP events around both, host conversion of the norms
excluded), and whether the averages are bit-identical between modes.
"""
from __future__ import annotations

import argparse
import json
import sys
from collections import OrderedDict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd

A = sys.modules[mfl_amd.DeviceAggregator.__module__]  # the module (mfl_amd.aggregate is the function)


def clients_for(name, dev):
    if name == "flat":
        K, shapes = 100, [("w", (25_000_000,))]
    elif name == "flat200":
        K, shapes = 200, [("w", (10_000_000,))]
    elif name.startswith("flatk"):  # flatk64: 64 clients of one 25M key
        K, shapes = int(name[5:]), [("w", (25_000_000,))]
    elif name == "resnet18_gn_k100":  # the cfg4 layout (all fp32 keys) at 100 clients
        from model_shapes import CONFIGS
        K, shapes = 100, CONFIGS["resnet18_gn"][1]
    else:
        from model_shapes import CONFIGS
        K, shapes = CONFIGS[name]
    g = torch.Generator(device=dev).manual_seed(7)
    out = []
    for i in range(K):
        sd = {}
        for n, shp in shapes:
            sd[n] = (torch.randint(0, 1000, shp, generator=g, device=dev) if n.endswith("num_batches_tracked")
                     else torch.randn(shp, generator=g, device=dev) * 0.05)
        out.append((i + 1, sd))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["flat", "resnet56", "femnist_cnn"])
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name in args.configs:
        base = clients_for(name, dev)
        K = len(base)
        P = sum(t.numel() for t in base[0][1].values())
        res = {}
        for mode in ("two-pass", "fused"):
            A.FUSE_DISTANCES = mode == "fused"
            agg = mfl_amd.DeviceAggregator(dev)
            times = []
            for r in range(args.reps + 2):
                # fresh (weak-referenceable, like state_dict()'s) dicts: client 0's receives the average
                w_locals = [(n, OrderedDict(sd)) for n, sd in base]
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                w_glob = agg.aggregate(w_locals)
                # client_distances without its host conversion: the device sums
                last = agg._last
                if "sumsq" in last and torch.float32 in last["sumsq"]:
                    s = last["sumsq"][torch.float32]
                else:
                    keep0 = agg._client0_tensors(last)
                    dicts = [keep0 if sd is w_glob else sd for _, sd in w_locals]
                    s = agg._sqdist_segments(last["table"], dicts, last["dev"][torch.float32][1])
                b.record()
                if r >= 2:
                    times.append((a, b))
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in times]))
            res[mode] = (ms, {k: v.clone() for k, v in w_glob.items()}, s.clone())
        A.FUSE_DISTANCES = True
        same = all(torch.equal(res["fused"][1][k].view(-1).view(torch.int32) if res["fused"][1][k].is_floating_point()
                               else res["fused"][1][k], res["two-pass"][1][k].view(-1).view(torch.int32)
                               if res["two-pass"][1][k].is_floating_point() else res["two-pass"][1][k])
                   for k in res["fused"][1])
        s2, s1 = res["two-pass"][2][1:], res["fused"][2][1:]
        rel = float(((s1 - s2).abs() / s2.abs().clamp_min(1e-300)).max()) if K > 1 else 0.0
        for mode in ("two-pass", "fused"):
            print(json.dumps({"config": name, "K": K, "P": P, "mode": mode, "ms_median": round(res[mode][0], 4),
                              "round_GBps": round((4 * K * P + 4 * P) / res[mode][0] / 1e6, 1),
                              "averages_bit_identical": same, "sums_max_rel": rel}), flush=True)
        del base, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
