"""Benchmark: device-resident FedAvg weighted reduction on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
    python bench.py --e2e [...]   # host state_dicts in/out vs the CPU loop (scripts/bench_e2e.py)
    python bench.py --fpf [...]   # FPF2 bookkeeping per round (scripts/bench_fpf.py)

Metric (BASELINE.json): "aggregated GB/s device-resident, K-client x P-param
fp32 weighted reduce".  A step is one pass of the hot path
(fedavg_trainer.py:441-458) over one batch of synthetic client updates
already resident in HBM: the exact sequential HIP kernel over this rank's
P-shard and, for N > 1, the RCCL all-gather that reassembles the averaged
model on every rank (overlapped chunk by chunk).

Default workload = the north-star target, K = 100 clients x P = 25M fp32
params per GPU (weak scaling: P grows with N; each rank owns a 25M-column
shard).  Algorithmic bytes per step = 4*K*P + 4*P + 4*K (reads of every
client row, the averaged-model write, the weights).

Rank 0 prints ONE JSON line.  Besides the contract keys it carries:
  roofline      : the reduce kernel's algorithmic HBM bytes / its average
                  launch time (HIP events on the launch stream), vs 8 TB/s;
  cpu_baseline  : the reference's torch CPU loop (oracle restatement, the
                  same expression as fedavg_trainer.py:450-457) on a bounded
                  sample, rank 0, N = 1 only;
  parity        : sampled columns compared bit for bit with the oracle.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np
import torch
import torch.distributed as dist

import mfl_amd
from mfl_amd.distributed import ShardedReducer

METRIC = "aggregated GB/s device-resident, K-client × P-param fp32 weighted reduce"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # name: (K, P per GPU, description)
    "target": (100, 25_000_000, "north-star target: 100 clients x 25M fp32 params per GPU"),
    "femnist_cnn": (10, 1_206_590, "cfg2 FEMNIST + CNN_DropOut, 10 clients (fits the 256 MiB MALL)"),
    "resnet56": (100, 600_372, "cfg3 CIFAR10 + resnet56, 100 clients (fits the 256 MiB MALL)"),
    "resnet18_gn": (500, 11_227_812, "cfg4 fed_cifar100 + resnet18_gn, 500 clients"),
    "synthetic_1000x100m_slice": (1000, 12_500_000, "cfg5 1000 clients, 12.5M-param P-slice per GPU"),
}


def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def algorithmic_bytes(K: int, P: int) -> int:
    return 4 * K * P + 4 * P + 4 * K


def sample_counts(K: int):
    return [int(v) for v in np.random.default_rng(1234).integers(1, 1001, size=K)]


def fill_synthetic(clients: torch.Tensor, rank: int):
    """client k = base + N(0, 1e-3^2), base ~ N(0, 0.05^2) (BASELINE.md inputs)."""
    K, cols = clients.shape
    g = torch.Generator(device=clients.device).manual_seed(rank * 7919)
    base = torch.randn(cols, generator=g, device=clients.device) * 0.05
    for k in range(K):
        gk = torch.Generator(device=clients.device).manual_seed(1000 + k + rank * 100_003)
        torch.randn(cols, generator=gk, device=clients.device, out=clients[k])
        clients[k].mul_(1e-3).add_(base)
    del base


def cpu_baseline(P: int, target_seconds: float = 12.0):
    """The reference's torch CPU loop (fedavg_trainer.py:444-458, restated in
    oracle/fedavg_oracle.py) on a bounded sample of the bench workload: a
    K-slice -- 10 clients with the workload's full P-element key (1 GB at
    P = 25M), so every tensor has the workload's size and the same cache
    behaviour (a P-slice of 10 MB tensors can sit in a large host L3 and
    overstate the CPU); repeated until ~target_seconds."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import fedavg_oracle as O

    threads = torch.get_num_threads()
    K = 10
    g = torch.Generator().manual_seed(0)
    base = torch.randn(P, generator=g) * 0.05
    clients = [base + torch.randn(P, generator=g) * 1e-3 for _ in range(K)]
    counts = sample_counts(K)
    times = []
    t_end = time.perf_counter() + target_seconds
    while time.perf_counter() < t_end or len(times) < 2:
        w_locals = [(counts[i], {"w": clients[i]}) for i in range(K)]  # fresh dicts: the loop mutates dict 0
        t0 = time.perf_counter()
        O.aggregate_torch(w_locals)
        times.append(time.perf_counter() - t0)
        if len(times) >= 50:
            break
    best = min(times[1:]) if len(times) > 1 else times[0]
    return {
        "value": round(algorithmic_bytes(K, P) / best / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"K-slice: K={K} x P={P} fp32 (the workload's key size), one flat key; reference torch CPU loop restated "
                  f"(oracle/fedavg_oracle.py aggregate_torch); best of {len(times) - 1} reps "
                  f"after 1 warm-up, {best * 1e3:.1f} ms/reduce, torch threads={threads}",
    }


def sampled_parity(red: ShardedReducer, weights, n_windows=6, width=2048):
    """Bit-compare sampled local columns of the device result with the oracle."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import fedavg_oracle as O

    segs = red.plan.local_segments()
    rng = np.random.default_rng(7)
    checked = 0
    for _ in range(n_windows):
        lstart, gstart, n = segs[int(rng.integers(0, len(segs)))]
        w = min(width, n)
        s = lstart + int(rng.integers(0, n - w + 1))
        exp = O.reduce_f32(red.clients[:, s:s + w].cpu().numpy(), weights)
        got = red.local_out[s:s + w].cpu().numpy()
        if red.host_out is not None:  # the copy the host consumer reads
            g = gstart + (s - lstart)
            if red.host_out[g:g + w].numpy().tobytes() != got.tobytes():
                return {"ok": False, "columns_checked": checked, "bar": "host_out == device shard"}
        if got.tobytes() != exp.tobytes():
            return {"ok": False, "columns_checked": checked, "bar": "bit-exact vs oracle"}
        checked += w
    return {"ok": True, "columns_checked": checked, "bar": "bit-exact vs oracle (sampled windows)"}


def overlap_diagnostics(red: ShardedReducer, w_dev, steps: int, step_elapsed: float, reps: int = 5) -> dict:
    """N > 1, after the timed region (not part of `value`): the reduce alone
    and the all-gather alone, each timed like a step (barrier + sync on both
    sides, max over ranks), so the JSON line shows how much of the exchange
    the chunked pipeline hides.  overlap = (reduce + gather - step) /
    min(reduce, gather): 1 = fully hidden, 0 = serialised."""
    def timed(fn):
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=red.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()) * 1e3

    gather = red.gather
    red.gather = False
    try:
        reduce_ms = timed(lambda: red.step(w_dev))
    finally:
        red.gather = gather
    gather_ms = timed(red.gather_only)
    step_ms = step_elapsed / steps * 1e3
    return {"reduce_only_ms": round(reduce_ms, 4), "gather_only_ms": round(gather_ms, 4), "step_ms": round(step_ms, 4),
            "overlap": round((reduce_ms + gather_ms - step_ms) / max(min(reduce_ms, gather_ms), 1e-9), 3),
            "gather_bytes_in_per_rank": int(red.plan.padded_P - red.plan.local_cols) * 4,
            "note": "after the timed region; not part of value"}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="target", choices=sorted(WORKLOADS))
    ap.add_argument("--chunks", type=int, default=0, help="all-gather pipeline chunks (0 = auto)")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the all-gather (reduce only)")
    ap.add_argument("--unroll", type=int, default=0, help="kernel variant: loads in flight per thread")
    ap.add_argument("--nt", type=int, default=-1, help="kernel variant: 1 = nontemporal loads")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true", help="N=1: replay each step from a captured hipGraph")
    ap.add_argument("--traffic-json", default="", help="PMC traffic summary (profiles/*.json) to attach")
    ap.add_argument("--host-out", action="store_true",
                    help="host consumer (SURVEY 8e): D2H each rank's shard into pinned host memory, no collective")
    args = ap.parse_args()

    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local_rank = env_int("LOCAL_RANK", 0)
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus > 1 needs torch.distributed.run (one process per GPU)")
        raise SystemExit(f"--gpus {args.gpus} does not match WORLD_SIZE={world} (one process per GPU)")
    # Rehearsal knobs (a 1-GPU box): FEDAVG_DIST_BACKEND=gloo and
    # FEDAVG_SAME_DEVICE=1 run N ranks on cuda:0.  The driver's runs use the
    # defaults: RCCL ("nccl") with one GPU per rank.
    backend = os.environ.get("FEDAVG_DIST_BACKEND", "nccl")
    dev_index = 0 if os.environ.get("FEDAVG_SAME_DEVICE") == "1" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    mfl_amd._lib.load()

    K, P_local, desc = WORKLOADS[args.workload]
    # N > 1: 8 chunks.  scripts/overlap_probe.py: with a
    # stand-in for RCCL's kernel that stays resident like an xGMI-bound
    # all-gather, 8 chunks hide 82-87 % of the shorter leg (4 chunks: 52-70 %)
    # for gathers of 1.0-3.0 ms per step
    chunks = args.chunks or (1 if world == 1 and not args.host_out else 4 if args.host_out else 8)
    P_total = P_local * world
    host_out = torch.empty(P_total, dtype=torch.float32, pin_memory=True) if args.host_out else None
    # Each rank owns exactly P_local valid columns: plan over the global P.
    red = ShardedReducer(K, P_total, chunks=chunks, device=dev, gather=not args.no_gather, host_out=host_out)
    fill_synthetic(red.clients, rank)
    counts = sample_counts(K)
    weights = mfl_amd.sample_weights(counts)
    w_dev = mfl_amd.weights_tensor(weights, torch.float32, dev)

    tuned = None
    if args.unroll or args.nt >= 0:
        tuned = (args.unroll or 8, max(args.nt, 0))

    S = red.plan.block
    sched = mfl_amd._lib.f32_schedule(K, S, red.plan.local_cols) if tuned is None else None
    launches_per_call = sched["launches"] if sched else 1
    ev_pairs = []

    def local_reduce(clients, w, P, out):
        mfl_amd.reduce_packed(clients, w, P, out, tuned=tuned)

    def timed_local_reduce(clients, w, P, out):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        mfl_amd.reduce_packed(clients, w, P, out, tuned=tuned)
        e.record()
        ev_pairs.append((s, e))

    red.local_reduce = local_reduce
    for _ in range(args.warmup):
        red.step(w_dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    step = lambda: red.step(w_dev)  # noqa: E731
    if args.graph:
        # one step captured into a hipGraph and replayed: removes the per-step
        # host launch path (Python + ctypes + hipLaunchKernel) that dominates
        # small, cache-resident workloads
        if world > 1:
            raise SystemExit("--graph is single-GPU only (RCCL capture is not used)")
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            red.step(w_dev)  # warm the capture stream
            torch.cuda.synchronize()
            with torch.cuda.graph(graph, stream=s):
                red.step(w_dev)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

        def step():
            st = torch.cuda.Event(enable_timing=True)
            en = torch.cuda.Event(enable_timing=True)
            st.record()
            graph.replay()
            en.record()
            ev_pairs.append((st, en))

        for _ in range(args.warmup):
            graph.replay()
        torch.cuda.synchronize()
        ev_pairs.clear()
    else:
        red.local_reduce = timed_local_reduce
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    kernel_ms = [s.elapsed_time(e) for s, e in ev_pairs]
    t = torch.tensor([elapsed, float(np.mean(kernel_ms))], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max, kernel_ms_max = float(t[0]), float(t[1])

    diagnostics = None
    if world > 1 and red.gather:
        diagnostics = overlap_diagnostics(red, w_dev, args.steps, elapsed_max)

    parity = sampled_parity(red, weights)
    if world > 1:
        ok = torch.tensor([1.0 if parity["ok"] else 0.0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        parity["ok"] = bool(ok.item() == 1.0)
        parity["ranks"] = world

    if rank == 0:
        bytes_step = algorithmic_bytes(K, P_total)
        value = bytes_step * args.steps / elapsed_max / 1e9
        # one reduce call = one chunk of one rank's shard = `launches_per_call`
        # round-split kernel launches of equal size
        bytes_call = algorithmic_bytes(K, S)
        achieved = bytes_call / (kernel_ms_max * 1e-3) / 1e9
        if sched:
            kern = "reduce_f32x4_buf_kernel" if sched["cols"] == 16 else "reduce_f32x4_var_kernel"
            kname = (f"{kern}<U={sched['unroll']},C={sched['cols']},nt={sched['nontemporal']}> "
                     f"(exact, sequential client order; round-split x{launches_per_call})")
        else:
            kname = f"tuned variant {tuned}"
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": kname,
            "bytes_per_launch": bytes_call // launches_per_call,
            "avg_launch_ms": round(kernel_ms_max / launches_per_call, 4),
            "launches": len(kernel_ms) * launches_per_call,
        }
        tj = args.traffic_json or str(ROOT / "profiles" / f"traffic_{args.workload}.json")
        if Path(tj).exists():
            try:
                tr = json.loads(Path(tj).read_text())
                src = os.path.relpath(tj, ROOT)
                if tr.get("algorithmic_bytes_per_launch") == roofline["bytes_per_launch"]:
                    roofline["traffic"] = tr.get("hbm_bytes_per_launch")
                    roofline["traffic_source"] = src
                elif tr.get("traffic_over_algorithmic"):
                    # other launch geometry (e.g. N > 1: 8 chunks per rank): the PMC
                    # traffic/algorithmic ratio of the same kernel, applied to this launch
                    ratio = float(tr["traffic_over_algorithmic"])
                    roofline["traffic"] = int(round(ratio * roofline["bytes_per_launch"]))
                    roofline["traffic_source"] = f"{src} (PMC ratio {ratio} x this launch's algorithmic bytes)"
            except (ValueError, OSError, KeyError):
                pass
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-generated: base~N(0,0.05^2) + per-client N(0,1e-3^2); counts U{1..1000})",
            "config": {
                "workload": desc,
                "K": K,
                "P_per_gpu": P_local,
                "P_total": P_total,
                "chunks": chunks,
                "exchange": ("rccl all_gather_into_tensor, overlapped per chunk" if red.gather else
                             "none: each rank D2Hs its shard chunks into pinned host memory (host consumer)"
                             if host_out is not None else "none (single GPU or --no-gather)"),
                "parallelism": f"p-shard{world}",
                "kernel_variant": {"unroll": tuned[0], "nt": tuned[1]} if tuned else "default",
                "launch": "hipGraph replay" if args.graph else "eager (stream-ordered)",
            },
            "roofline": roofline,
            # the whole step against the node's HBM-read roofline (N x 8 TB/s):
            # north_star's "fraction of the HBM-read roofline" at N GPUs
            "step_frac_of_node_hbm": round(value / (world * HBM_PEAK_GBS), 4),
            "parity": parity,
        }
        if diagnostics is not None:
            out["diagnostics"] = diagnostics
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(P_local)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def side_bench(argv) -> bool:
    """``bench.py --e2e ...`` / ``bench.py --fpf ...``: the host-in/host-out
    rate of the drop-in (scripts/bench_e2e.py) and the FPF2 bookkeeping per
    round (scripts/bench_fpf.py), each beside its CPU baseline -- the
    reference's torch expressions (oracle/), handed in from here."""
    if not argv or argv[0] not in ("--e2e", "--fpf"):
        return False
    sys.path.insert(0, str(ROOT / "scripts"))
    sys.path.insert(0, str(ROOT / "oracle"))
    if argv[0] == "--e2e":
        import bench_e2e
        import fedavg_oracle as O

        bench_e2e.main(O.aggregate_torch, O.client_distances_torch, argv[1:])
    else:
        import bench_fpf
        import fpf_oracle

        bench_fpf.main(fpf_oracle.FPFOracle, argv[1:])
    return True


if __name__ == "__main__":
    if not side_bench(sys.argv[1:]):
        main()
