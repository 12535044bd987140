"""End-to-end rate of the drop-in: host state_dicts in, host state_dict out.

    python bench.py --e2e [--configs mnist_lr,femnist_cnn,resnet56,target_flat] [--reps 5]

The reference's aggregate starts and ends in host memory (client.py:96
returns ``net.cpu().state_dict()``; fedavg_trainer.py:219 loads the result
into the CPU-resident global model), so this measures the whole drop-in:
validation, packing into pinned staging rows overlapped with per-client H2D,
the HIP kernel, D2H and unpacking -- next to the reference's torch CPU loop
(oracle restatement) on the same inputs in the same process, and checks the
two agree bit for bit.  It also times the streaming form (RoundSession):
clients added one by one as they would arrive from the round loop (with a
simulated per-client training time, --train-ms, between arrivals), and the
time from the last arrival to the averaged model (the part left on the
round's critical path).  Last, the same rounds with the clients' tensors
already on the GPU (device in, device out; see tests/test_gpu_device_clients.py).
One JSON line per config.
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import time
from collections import OrderedDict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

import mfl_amd
from model_shapes import CONFIGS, resnet56_shapes  # noqa: F401


def make_clients(K, shapes, seed=0):
    g = torch.Generator().manual_seed(seed)
    base = {k: torch.randn(s, generator=g) * 0.05 for k, s in shapes if not k.endswith("num_batches_tracked")}
    counts = [int(v) for v in np.random.default_rng(1234).integers(1, 1001, size=K)]
    dicts = []
    for i in range(K):
        sd = OrderedDict()
        for k, s in shapes:
            if k.endswith("num_batches_tracked"):
                sd[k] = torch.tensor(1000 + i, dtype=torch.int64)
            else:
                sd[k] = base[k] + torch.randn(s, generator=g) * 1e-3
        dicts.append(sd)
    return counts, dicts


def fresh(counts, dicts):
    # aggregate mutates w_locals[0][1]; give each rep its own first dict
    return [(counts[0], OrderedDict(dicts[0]))] + list(zip(counts[1:], dicts[1:]))


def run(name, reps, cpu_aggregate, cpu_distances, train_ms=0.0):
    K, shapes = CONFIGS[name]
    P = sum(math.prod(s) for _, s in shapes)
    counts, dicts = make_clients(K, shapes)
    alg = 4 * K * P + 4 * P + 4 * K
    agg = mfl_amd.DeviceAggregator(torch.device("cuda", 0))
    gpu_t, prof = [], []
    for r in range(reps + 1):
        wl = fresh(counts, dicts)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = agg.aggregate(wl)
        t = time.perf_counter() - t0
        if r:
            gpu_t.append(t)
            prof.append(dict(agg.last_profile))
    # post-aggregate distances (fedavg_trainer.py:291) on the round's device rows
    has_bool = any(t.dtype == torch.bool for t in dicts[0].values())
    dist_t = []
    if not has_bool:
        for r in range(reps + 1):
            t0 = time.perf_counter()
            norms = agg.client_distances(wl, out)
            t = time.perf_counter() - t0
            if r:
                dist_t.append(t)
    cpu_t, cpu_dist_t = [], []
    cpu_reps = max(1, min(reps, int(20.0 / max(alg / 5e9, 1e-3))))
    for r in range(cpu_reps + 1):
        wl_ref = fresh(counts, dicts)
        t0 = time.perf_counter()
        ref = cpu_aggregate(wl_ref)
        t = time.perf_counter() - t0
        if r:
            cpu_t.append(t)
    for r in range(min(cpu_reps, 2) + 1):
        t0 = time.perf_counter()
        ref_norms = cpu_distances(wl_ref, ref)
        t = time.perf_counter() - t0
        if r:
            cpu_dist_t.append(t)
    dist_rel = float(np.max(np.abs(norms - ref_norms) / np.maximum(np.abs(ref_norms), 1e-30))) if dist_t else None
    # streaming rounds (mfl_amd.RoundSession): clients are added as they
    # "arrive"; what remains after the last arrival is the round's critical path
    crit, add_ms = [], []
    for r in range(reps + 1):
        wl = fresh(counts, dicts)
        torch.cuda.synchronize()
        sess = agg.begin_round(wl[0][1], K)
        for n, sd in wl:
            if train_ms:
                time.sleep(train_ms / 1e3)  # the client's local training (client.py:38-96) would run here
            sess.add(n, sd)
        t0 = time.perf_counter()
        sout = sess.finish(wl)
        t = time.perf_counter() - t0
        if r:
            crit.append(t)
            add_ms.append(sess.add_ms)
    same_stream = all(torch.equal(sout[k].reshape(-1).view(torch.int32), out[k].reshape(-1).view(torch.int32))
                      for k in out)
    # device-resident clients (client.py:96 without the .cpu()): state_dicts
    # already in HBM, averaged model returned in HBM -- one packing kernel,
    # the weights, the reduce; timed to the device result being complete
    dev = torch.device("cuda", 0)
    ddicts = [OrderedDict((k, v.to(dev)) for k, v in sd.items()) for sd in dicts]
    dev_t, dcrit, ddist_t = [], [], []
    for r in range(reps + 1):
        wl = fresh(counts, ddicts)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dout = agg.aggregate(wl)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        if r:
            dev_t.append(t)
        if not has_bool:  # :291 right after, on the clients' own tensors
            t0 = time.perf_counter()
            dnorms = agg.client_distances(wl, dout)
            t = time.perf_counter() - t0
            if r:
                ddist_t.append(t)
    same_dev = all(torch.equal(dout[k].cpu().reshape(-1).view(torch.int32), out[k].reshape(-1).view(torch.int32))
                   for k in out)
    for r in range(reps + 1):
        wl = fresh(counts, ddicts)
        torch.cuda.synchronize()
        sess = agg.begin_round(wl[0][1], K)
        for n, sd in wl:
            if train_ms:
                time.sleep(train_ms / 1e3)
            sess.add(n, sd)
        t0 = time.perf_counter()
        dsout = sess.finish(wl)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        if r:
            dcrit.append(t)
    same_dev = same_dev and all(torch.equal(dsout[k].cpu().reshape(-1).view(torch.int32),
                                            out[k].reshape(-1).view(torch.int32)) for k in out)
    del ddicts, wl, dout, dsout
    # the same clients written into ONE buffer in the packed layout
    # (mfl_amd.client_arena): the aggregate runs the row kernel on them
    arena_t, arena_dist_t, arena_same = [], [], None
    if all(t.dtype == torch.float32 for t in dicts[0].values()):
        rows, adicts = mfl_amd.client_arena(dicts[0], K, dev)
        for a, sd in zip(adicts, dicts):
            for k, v in sd.items():
                a[k].copy_(v)
        before = agg.arena_rounds
        for r in range(reps + 1):
            wl = [(counts[0], OrderedDict(adicts[0]))] + list(zip(counts[1:], adicts[1:]))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            aout = agg.aggregate(wl)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            if r:
                arena_t.append(t)
            t0 = time.perf_counter()
            agg.client_distances(wl, aout)
            t = time.perf_counter() - t0
            if r:
                arena_dist_t.append(t)
        arena_same = (agg.arena_rounds - before == reps + 1) and all(
            torch.equal(aout[k].cpu().reshape(-1).view(torch.int32), out[k].reshape(-1).view(torch.int32)) for k in out)
        del rows, adicts, wl, aout
    gd = float(np.median(dev_t))
    same = all(torch.equal(out[k].reshape(-1).view(torch.int32), ref[k].reshape(-1).view(torch.int32)) for k in ref)
    g, c = float(np.median(gpu_t)), float(np.median(cpu_t))
    return {
        "config": name, "K": K, "P": P, "keys": len(shapes),
        "e2e_ms_median": round(g * 1e3, 3), "e2e_ms_min": round(min(gpu_t) * 1e3, 3),
        "e2e_GBps": round(alg / g / 1e9, 2),
        "pack_issue_ms_median": round(float(np.median([p["pack_issue_ms"] for p in prof])), 3),
        "h2d_kernel_d2h_ms_median": round(float(np.median([p["h2d_kernel_d2h_ms"] for p in prof])), 3),
        "cpu_ref_ms_median": round(c * 1e3, 3), "cpu_ref_GBps": round(alg / c / 1e9, 2),
        "cpu_threads": torch.get_num_threads(), "speedup_vs_cpu": round(c / g, 2),
        "bit_exact_vs_cpu_ref": bool(same), "reps": reps,
        "stream_finish_ms_median": round(float(np.median(crit)) * 1e3, 3),
        "stream_add_ms_total_median": round(float(np.median(add_ms)), 3),
        "stream_bit_exact": bool(same_stream),
        "stream_train_ms_per_client": train_ms,
        "device_clients_ms_median": round(gd * 1e3, 3), "device_clients_GBps": round(alg / gd / 1e9, 2),
        "device_clients_stream_finish_ms_median": round(float(np.median(dcrit)) * 1e3, 3),
        "device_clients_bit_exact": bool(same_dev),
        "arena_clients_ms_median": round(float(np.median(arena_t)) * 1e3, 3) if arena_t else None,
        "arena_clients_GBps": round(alg / float(np.median(arena_t)) / 1e9, 2) if arena_t else None,
        "arena_clients_dist_ms_median": round(float(np.median(arena_dist_t)) * 1e3, 3) if arena_dist_t else None,
        "arena_clients_bit_exact_and_row_path": arena_same,
        "device_clients_dist_ms_median": round(float(np.median(ddist_t)) * 1e3, 3) if ddist_t else None,
        "device_clients_dist_max_rel_vs_host": (float(np.max(np.abs(dnorms - norms) / np.maximum(np.abs(norms), 1e-30)))
                                                if ddist_t and dist_t else None),
        "dist_ms_median": round(float(np.median(dist_t)) * 1e3, 3) if dist_t else None,
        "cpu_dist_ms_median": round(float(np.median(cpu_dist_t)) * 1e3, 3),
        "dist_max_rel_vs_cpu_ref": dist_rel,
    }


def main(cpu_aggregate, cpu_distances, argv=None):
    """Entry point for ``python bench.py --e2e ...``: bench.py hands in its CPU
    baseline (the reference's torch loop and :291 norms, oracle/)."""
    ap = argparse.ArgumentParser(prog="bench.py --e2e")
    ap.add_argument("--configs", default="mnist_lr,femnist_cnn,resnet56,target_flat")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--train-ms", type=float, default=5.0,
                    help="simulated per-client training time between streaming arrivals")
    args = ap.parse_args(argv)
    torch.cuda.set_device(0)
    for name in args.configs.split(","):
        print(json.dumps(run(name, args.reps, cpu_aggregate, cpu_distances, args.train_ms)), flush=True)


if __name__ == "__main__":
    sys.exit("run as: python bench.py --e2e [--configs ...] [--reps N] [--train-ms MS]")
