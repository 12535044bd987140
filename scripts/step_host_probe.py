"""Host cost of one reduce call for a cache-resident model (cfg2 FEMNIST x 10).

    python scripts/step_host_probe.py [--K 10] [--P 1206590] [--calls 2000]

bench.py's step for a small model is bound by the host's launch path, not the
kernel (~14 us per step for a ~7.5 us kernel).  This probe times N back-to-back
calls (wall clock / N, the GPU synchronised once at the end) of:
  raw      : the ctypes entry fedavg_reduce_f32 with prepared arguments;
  prepared : reduce.PreparedReduce.__call__ (the bench's per-chunk call);
  timed    : the same with launch-attached events (fedavg_reduce_f32_timed);
  step     : ShardedReducer.step at one rank, one chunk (bench.py's red_step
             without timing);
  step_timed : the same with the attached events bench.py passes.
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
from mfl_amd import _lib
from mfl_amd.distributed import ShardedReducer
from mfl_amd.reduce import PreparedReduce


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--P", type=int, default=1_206_590)
    ap.add_argument("--calls", type=int, default=2000)
    args = ap.parse_args()
    K, P, n = args.K, args.P, args.calls
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    red = ShardedReducer(K, P, device=dev, as_rank=(1, 0))
    red.clients.normal_()
    w = torch.full((K,), 1.0 / K, device=dev)
    ld = red.clients.stride(0)
    out = torch.empty(P, device=dev)
    prep = PreparedReduce(red.clients, w, P, out)
    s = int(torch.cuda.current_stream(dev).cuda_stream)
    args_raw = (red.clients.data_ptr(), K, P, ld, w.data_ptr(), out.data_ptr(), s)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record()
    ev[1].record()

    def raw():
        lib.fedavg_reduce_f32(*args_raw)

    legs = {
        "raw": raw,
        "prepared": lambda: prep(),
        "timed": lambda: prep(events=ev),
        "step": lambda: red.step(w),
        "step_timed": lambda: red.step(w, timing=lambda c: ev),
    }
    rec = {"K": K, "P": P, "calls": n}
    for name, fn in legs.items():
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        g0.record()
        for _ in range(n):
            fn()
        t_host = time.perf_counter() - t0
        g1.record()
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        rec[name] = {"host_us_per_call": round(t_host / n * 1e6, 2), "wall_us_per_call": round(t_all / n * 1e6, 2),
                     "gpu_us_per_call": round(g0.elapsed_time(g1) / n * 1e3, 2)}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
