"""How the bench's per-launch kernel time compares with rocprofv3's for short
launches (the per-rank chunk kernel of an N-GPU plan, e.g. 4 x 781K columns
at N = 8: ~47 us per launch).  Rank 0's shard of the plan is built as
``bench.py --shard-of N --chunks C`` builds it, and the chunk reduce is timed
in phases, each exactly ``--calls`` chunk launches, in this order:

  attached   launch-attached HIP events (fedavg_reduce_f32_timed), back to back
  isolated   launch-attached events, the stream drained before every launch
  batched    one event pair around all calls of the phase, back to back
  bracketed  hipEventRecord pairs (torch events) around every call

Run it under ``rocprofv3 --kernel-trace --stats``; the kernel trace's
dispatches of the reduce kernel, in order, split into the same phases give
each phase's true kernel time beside what the events said.

    python scripts/launch_timing_probe.py [--shard-of 8 --chunks 4 --calls 200]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np
import torch

import mfl_amd
from mfl_amd import synthetic
from mfl_amd.distributed import ShardedReducer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--shard-of", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--calls", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load()
    counts = synthetic.sample_counts(args.K)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(counts), torch.float32, dev)
    red = ShardedReducer(args.K, args.P, chunks=args.chunks, device=dev, gather=False,
                         as_rank=(args.shard_of, 0))
    synthetic.fill_rows(red.clients, red.plan.local_segments())
    S = red.plan.block
    rows = red.clients
    ld = rows.stride(0)
    chunks = [(c * S, S) for c in range(red.plan.chunks)]
    out = torch.empty(red.plan.local_cols, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()
    sched = mfl_amd._lib.f32_schedule(args.K, S, ld)

    def launch(i, ev=None):
        c0, n = chunks[i % len(chunks)]
        src = rows[:, c0:c0 + n]
        if ev is None:
            rc = lib.fedavg_reduce_f32(src.data_ptr(), args.K, n, ld, w.data_ptr(), out[c0:].data_ptr(),
                                       stream.cuda_stream)
        else:
            rc = lib.fedavg_reduce_f32_timed(src.data_ptr(), args.K, n, ld, w.data_ptr(), out[c0:].data_ptr(),
                                             stream.cuda_stream, ev[0].cuda_event, ev[1].cuda_event)
        mfl_amd._lib.check(rc, "reduce")

    for i in range(20):  # warm
        launch(i)
    torch.cuda.synchronize()
    n = args.calls
    res = {}
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record()
        b.record()
    torch.cuda.synchronize()
    for i in range(n):
        launch(i, evs[i])
    torch.cuda.synchronize()
    res["attached"] = [a.elapsed_time(b) for a, b in evs]
    for i in range(n):
        torch.cuda.synchronize()
        launch(i, evs[i])
    torch.cuda.synchronize()
    res["isolated"] = [a.elapsed_time(b) for a, b in evs]
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(n):
        launch(i)
    b.record()
    torch.cuda.synchronize()
    res["batched"] = [a.elapsed_time(b) / n]
    for i in range(n):
        evs[i][0].record()
        launch(i)
        evs[i][1].record()
    torch.cuda.synchronize()
    res["bracketed"] = [a.elapsed_time(b) for a, b in evs]
    alg = 4 * args.K * S + 4 * S + 4 * args.K
    print(json.dumps({"shard_of": args.shard_of, "chunks": args.chunks, "chunk_cols": S, "calls_per_phase": n,
                      "schedule": sched, "algorithmic_bytes_per_launch": alg,
                      "phases_in_order": list(res),
                      "ms": {k: {"mean": round(float(np.mean(v)), 5), "median": round(float(np.median(v)), 5)}
                             for k, v in res.items()},
                      "frac_of_8TBps": {k: round(alg / (float(np.mean(v)) * 1e-3) / 8e12, 4) for k, v in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
