"""FPF2 bookkeeping per round at the reference's size (fedavg_trainer.py:209-210, 271-278, 314-327).

    python bench.py --fpf [--n 1000] [--p 7850] [--k 100] [--rounds 20]

The reference's FPF2 state is active for models under THRESHOLD_WEIGHT_SIZE
(config.py:83) -- MNIST-LR, P = 7850 -- with one row per vehicle
(client_num_in_total = 1000 in the channel traces) and client_num_per_round
= 100 (config.py:20).  One JSON line per leg, the per-round cost of
:165's last_w upload + :210 for the round's K clients + :272-278 + :314-327:

* hip       : ``mfl_amd.FPFTracker`` -- the :210 rows come from the client
              rows the aggregate already placed in HBM (``record_round``);
* torch_gpu : the reference's own torch expressions with the state on the GPU,
              as the reference keeps it (``self.device``), including its
              per-client ``cat(...).to(device)`` uploads at :210 / :316;
* torch_cpu : the same expressions on the host (CPU baseline).

The aggregate itself is outside the timed region (bench.py measures it).
Algorithmic HBM bytes per round (hip leg): K*P*8 (:210 read row + write
diff) + N*P*4 (:272 read) + N_unselected*P*8 (:317 read+write) + O(P).
The torch legs come from bench.py (its baseline leg; oracle/fpf_oracle.py).
"""
from __future__ import annotations

import argparse
import copy
import json
import sys
import time
from collections import OrderedDict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

import mfl_amd


def _rounds(n, p, k, rounds, seed=0):
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    init = OrderedDict(weight=torch.randn(10, p // 10 - 1, generator=g) * 0.01, bias=torch.zeros(10))
    plan = []
    for t in range(rounds):
        idx = rng.choice(n, size=k, replace=False).tolist()
        states = [OrderedDict((key, v + 0.01 * torch.randn(v.shape, generator=g)) for key, v in init.items())
                  for _ in range(k)]
        plan.append((idx, 1 + t % 3, rng.integers(50, 600, size=k).tolist(), states))
    return init, plan


def _run(leg, init, plan, n, warmup, make_oracle, dev):
    comm = len(plan)
    agg = mfl_amd.DeviceAggregator(dev)
    if leg == "hip":
        tr = mfl_amd.FPFTracker(n, init, comm, device=dev, aggregator=agg)
    else:
        orc = make_oracle(n, sum(v.numel() for v in init.values()), comm,
                          device=dev if leg == "torch_gpu" else "cpu")
    model = OrderedDict((k, v.clone()) for k, v in init.items())
    times, rows = [], []
    for t, (idx, itr, counts, states) in enumerate(plan):
        last_w = copy.deepcopy(model)
        w_locals = [(c, OrderedDict((k, v.clone()) for k, v in sd.items())) for c, sd in zip(counts, states)]
        torch.cuda.synchronize(dev)
        if leg == "hip":
            w_glob = agg.aggregate(w_locals)  # client rows land in HBM (not timed here)
            t0 = time.perf_counter()
            tr.begin_round(last_w)
            tr.record_round(idx, w_locals, w_glob)
            fpf = tr.fpf_index()
            tr.end_round(t, idx, itr, w_glob)
            dt = time.perf_counter() - t0
        else:
            t0 = time.perf_counter()
            for c, (_, w) in zip(idx, w_locals):
                orc.record_client(c, w, last_w)  # :210, before the aggregate as in the reference
            if leg == "torch_gpu":
                torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            w_glob = agg.aggregate(w_locals)
            t0 = time.perf_counter()
            fpf = orc.fpf_index()
            orc.end_round(t, idx, itr, w_glob, last_w)
            if leg == "torch_gpu":
                torch.cuda.synchronize(dev)
            dt += time.perf_counter() - t0
        for k in model:
            model[k].copy_(w_glob[k])
        rows.append(np.asarray(fpf, dtype=np.float64))
        if t >= warmup:
            times.append(dt)
    return times, rows


def main(make_oracle, argv=None):
    ap = argparse.ArgumentParser(prog="bench.py --fpf")
    ap.add_argument("--n", type=int, default=1000, help="client_num_in_total (vehicles)")
    ap.add_argument("--p", type=int, default=7850, help="model elements (MNIST-LR)")
    ap.add_argument("--k", type=int, default=100, help="clients per round")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--legs", default="hip,torch_gpu,torch_cpu")
    args = ap.parse_args(argv)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    init, plan = _rounds(args.n, args.p, args.k, args.rounds + args.warmup)
    P = sum(v.numel() for v in init.values())
    results = {}
    for leg in args.legs.split(","):
        times, rows = _run(leg, init, plan, args.n, args.warmup, make_oracle, dev)
        results[leg] = rows
        unsel = args.n - args.k
        alg = args.k * P * 8 + args.n * P * 4 + unsel * P * 8 + 6 * P * 4
        line = {"bench": "fpf_round", "leg": leg, "n": args.n, "P": P, "k": args.k, "rounds": len(times),
                "ms_per_round_median": round(float(np.median(times)) * 1e3, 3),
                "ms_per_round_min": round(float(np.min(times)) * 1e3, 3),
                "alg_bytes_per_round": alg,
                "cpu_threads": torch.get_num_threads() if leg == "torch_cpu" else None}
        ref = results.get("torch_cpu")
        if ref is not None and leg != "torch_cpu":
            pass
        print(json.dumps(line), flush=True)
    if "torch_cpu" in results:
        ref = np.stack(results["torch_cpu"])
        for leg in results:
            if leg == "torch_cpu":
                continue
            got = np.stack(results[leg])
            nz = ref != 0
            rel = float(np.max(np.abs(got[nz] - ref[nz]) / np.abs(ref[nz]))) if nz.any() else 0.0
            print(json.dumps({"bench": "fpf_round_parity", "leg": leg, "vs": "torch_cpu",
                              "zero_positions_equal": bool(np.array_equal(got == 0, ref == 0)),
                              "max_rel": rel}), flush=True)


if __name__ == "__main__":
    sys.exit("run as: python bench.py --fpf [--n 1000] [--p 7850] [--k 100] [--rounds 20]")
