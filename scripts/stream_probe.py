"""Timeline probe of a streaming round's finish (RoundSession) at the target size.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o stream \
        -- python scripts/stream_probe.py [--K 100] [--P 25000000] [--train-ms 5] [--rounds 3]

Prints, per round, the host time of the last add and of finish; with the
rocprof traces the copies and kernels of the last round can be lined up
against them (host perf_counter_ns is printed next to each phase).
"""
from __future__ import annotations

import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--train-ms", type=float, default=5.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--keep-results", action="store_true",
                    help="keep every round's result alive (each round then copies into a never-used pinned buffer)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator().manual_seed(0)
    base = torch.randn(args.P, generator=g) * 0.05
    dicts = [OrderedDict(w=base + 1e-3 * torch.randn(args.P, generator=g)) for _ in range(args.K)]
    counts = list(np.random.default_rng(1).integers(1, 1000, size=args.K))
    agg = mfl_amd.DeviceAggregator(dev)
    kept = []
    for r in range(args.rounds):
        wl = [(int(n), OrderedDict(d)) for n, d in zip(counts, dicts)]
        torch.cuda.synchronize()
        sess = agg.begin_round(wl[0][1], args.K)
        add_ns = []
        for n, sd in wl:
            time.sleep(args.train_ms / 1e3)
            t0 = time.perf_counter_ns()
            sess.add(n, sd)
            add_ns.append((t0, time.perf_counter_ns()))
        t0 = time.perf_counter_ns()
        out = sess.finish(wl)
        t1 = time.perf_counter_ns()
        if args.keep_results:
            kept.append(out)
        print(json.dumps({"round": r, "last_add_start_ns": add_ns[-1][0], "last_add_end_ns": add_ns[-1][1],
                          "last_add_ms": (add_ns[-1][1] - add_ns[-1][0]) / 1e6,
                          "finish_start_ns": t0, "finish_end_ns": t1, "finish_ms": (t1 - t0) / 1e6,
                          "finish_phases_ms": {k: round(v, 3) for k, v in sess.finish_profile.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
