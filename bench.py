"""Benchmark: device-resident FedAvg weighted reduction on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--scaling strong|weak]
    python bench.py --e2e [...]   # host state_dicts in/out vs the CPU loop (scripts/bench_e2e.py)
    python bench.py --fpf [...]   # FPF2 bookkeeping per round (scripts/bench_fpf.py)

Metric (BASELINE.json): "aggregated GB/s device-resident, K-client x P-param
fp32 weighted reduce".  A step is one pass of the hot path
(fedavg_trainer.py:441-458) over one batch of synthetic client updates
already resident in HBM: the exact sequential HIP kernel over this rank's
P-shard and, for N > 1, the RCCL all-gather that reassembles the averaged
model on every rank (overlapped chunk by chunk).

Multi-GPU: one process per GPU.  Under torch.distributed.run the ranks come
from the environment; ``python bench.py --gpus N`` without it starts
``torch.distributed.run`` itself as a child process (this process never
touches the GPU) and exits with its status.

Scaling (``--scaling``):
  strong (default): the workload's P is the GLOBAL model, split over the N
          ranks -- the BASELINE configurations: the target is 100 clients x
          25M params in total (3.125M columns per rank at N = 8),
          cfg4 500 x 11.2M, cfg5 1000 x 100M (12.5M per rank at N = 8);
  weak:   every rank owns P columns (the model has N x P params).
Algorithmic bytes per step = 4*K*P + 4*P + 4*K for the global P (reads of
every client row, the averaged-model write, the weights).

Inputs: ``mfl_amd.synthetic`` -- every value a pure function of (client,
global column), so the model does not depend on N and any window of the
gathered model is re-derived on the host by numpy + the oracle.

Rank 0 prints ONE JSON line.  Besides the contract keys it carries:
  roofline      : the reduce kernel's algorithmic HBM bytes / its average
                  launch time (HIP events on the launch stream), vs 8 TB/s;
  cpu_baseline  : the reference's torch CPU loop (oracle restatement, the
                  same expression as fedavg_trainer.py:450-457) on bounded
                  samples, rank 0, N = 1 only: one flat key and the
                  model-shaped resnet56 state_dict (350 keys);
  parity        : sampled windows bit for bit vs the oracle on host-derived
                  inputs (at N > 1: windows of the gathered model owned by
                  any rank, plus per-rank checksums of the reassembly).
"""
from __future__ import annotations

import argparse
import datetime
import json
import math
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent

METRIC = "aggregated GB/s device-resident, K-client × P-param fp32 weighted reduce"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # name: (K, P, description); P is the global model under strong scaling
    # and the per-rank shard under weak scaling
    "target": (100, 25_000_000, "north-star target: 100 clients x 25M fp32 params"),
    "femnist_cnn": (10, 1_206_590, "cfg2 FEMNIST + CNN_DropOut, 10 clients (fits the 256 MiB MALL)"),
    "resnet56": (100, 600_372, "cfg3 CIFAR10 + resnet56, 100 clients (fits the 256 MiB MALL)"),
    "resnet18_gn": (500, 11_227_812, "cfg4 fed_cifar100 + resnet18_gn, 500 clients"),
    "synthetic_1000x100m": (1000, 100_000_000, "cfg5 synthetic 1000 clients x 100M fp32 params"),
    "synthetic_1000x100m_slice": (1000, 12_500_000, "cfg5's per-GPU slice at N = 8 (1000 x 12.5M)"),
    "rehearsal_small": (8, 200_003, "CPU rehearsal of the multi-rank machinery (8 x 200,003; --cpu-rehearsal)"),
}

# chunked passes: every SPAN_EVERY-th pass of the timed region is bracketed by
# an event pair for the per-launch kernel time (the markers' own cost, above)
SPAN_EVERY = 8

# One rank's client rows may take this much HBM (MI355X: 288 GB); a larger
# single-GPU workload (cfg5 at N = 1: 400 GB) runs as P-chunked passes over
# one resident buffer ("each pass device-resident; time = sum").
ROW_BUDGET_BYTES = int(float(os.environ.get("FEDAVG_BENCH_ROW_BUDGET_GB", "230")) * 1e9)

# N > 1 pipeline: chunk count so that every chunk keeps enough columns for a
# full-chip launch of the short-row schedule (see auto_chunks)
MIN_CHUNK_COLS = 700_000
MAX_CHUNKS = 8
# ... and at N > 1 the warm-up times these depths (plus the rule's pick) and
# keeps the fastest whole step; a candidate needs >= SWEEP_MIN_BLOCK columns
# per chunk
SWEEP_CHUNKS = (1, 2, 4, 8)
SWEEP_MIN_BLOCK = 1024


def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def algorithmic_bytes(K: int, P: int) -> int:
    return 4 * K * P + 4 * P + 4 * K


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(argv) -> "int | None":
    """``--gpus N`` (N > 1) outside torch.distributed.run: start the N ranks
    with torch.distributed.run as a CHILD process -- nothing here has touched
    the GPU -- relay its output (rank 0 prints the JSON line) and return its
    exit status (non-zero if any rank failed).  None: run in this process."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    known, _ = ap.parse_known_args(argv)
    if known.gpus <= 1 or os.environ.get("WORLD_SIZE") not in (None, ""):
        return None
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # the box supports dmabuf IPC only
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={known.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()), *argv]
    return subprocess.call(cmd, env=env)


def one_group_per_cu(K: int, cols: int, cus: int = 256) -> bool:
    """Does the production fp32 schedule give (nearly) one column group per
    CU on a chunk of ``cols`` columns?  The bands of choose_f32_schedule
    (fedavg_reduce.hip): 6 slices per thread (1,536 float4 per group) for
    K >= 64, 3 slices for K >= 256, at 0.9 to 1 group per CU.  Those are the
    chunk shapes the kernel streams best: K = 100 x 1.56M (254 groups) at
    85-86 % of peak against 81.5-82 % for 781K / 1.04M chunks and 83.5 % for
    1.25M (0.8 groups per CU) (profiles/r03/shard8/, profiles/r03/chunk_schedules/)."""
    nvec = -(-cols // 4)
    if K >= 64 and cus * 9 // 10 * 256 * 6 <= nvec <= cus * 256 * 6:
        return True
    return K >= 256 and cus * 9 // 10 * 256 * 3 <= nvec <= cus * 256 * 3


def auto_chunks(K: int, shard_cols: int, world: int, host_out: bool) -> int:
    """All-gather pipeline depth.  One chunk at N = 1 (no exchange; the
    host-out consumer overlaps 4 D2H chunks).  At N > 1 the most chunks (up
    to 8) whose width lands in a one-group-per-CU band of the kernel (the
    gather of chunk c overlaps the reduce of chunk c + 1); failing that the
    deepest of 8/4/2/1 whose chunks keep >= MIN_CHUNK_COLS columns, so each
    chunk launch still fills the chip."""
    if host_out:
        return 4
    if world == 1:
        return 1
    for c in range(MAX_CHUNKS, 0, -1):
        width = -(-shard_cols // c)
        if one_group_per_cu(K, -(-width // 64) * 64):
            return c
    c = MAX_CHUNKS
    while c > 1 and shard_cols // c < MIN_CHUNK_COLS:
        c //= 2
    return c


def _thread_count():
    """Host threads for the CPU baseline: BASELINE.md's plan times the
    reference loop with torch.set_num_threads(len(os.sched_getaffinity(0)));
    the GPU box also sets OMP_NUM_THREADS (its 1-GPU job share of a larger
    machine), timed as a second, labelled entry.  Returns (affinity CPUs,
    OMP-capped count or None when there is no cap below the affinity)."""
    n_aff = len(os.sched_getaffinity(0))
    omp = env_int("OMP_NUM_THREADS", 0)
    return n_aff, (omp if 0 < omp < n_aff else None)


def cpu_baseline(K: int, P: int, flat_seconds: float = 6.0, model_seconds: float = 4.0, rep_budget_s: float = 2.5,
                 model: str = "resnet56"):
    """The reference's torch CPU loop (fedavg_trainer.py:444-458, restated in
    oracle/fedavg_oracle.py) on the GPU box's host cores, per BASELINE.md's
    CPU-baseline plan:

    * flat: the workload's own K x P (100 x 25M = 10 GB of host tensors at
      the target) with ``torch.set_num_threads(len(os.sched_getaffinity(0)))``
      -- ``value`` -- and again at the OMP_NUM_THREADS cap the box sets (a
      second, labelled entry).  When one full-K reduce at a thread count would
      take longer than ``rep_budget_s`` (estimated from a timed 10-client
      slice: the affinity count of a shared box can be many times its CPU
      share), that entry times the 10-client K-slice instead and says so.
    * model-shaped: cfg3's resnet56 state_dicts (350 keys, 58 int64
      num_batches_tracked buffers), all 100 clients -- the per-key dispatch
      cost the reference pays on real models (slowest layout) -- at
      the box's own thread share.
    Progress goes to stderr (a long silent CPU phase looks like a hang)."""
    import torch

    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "scripts"))
    import fedavg_oracle as O
    from model_shapes import CONFIGS, numel

    def note(msg):
        print(f"[cpu_baseline] {msg}", file=sys.stderr, flush=True)

    n_aff, n_omp = _thread_count()
    torch.set_num_threads(n_omp or n_aff)  # generation at the box's own share

    def timed(w_locals_factory, seconds, max_reps=50):
        times = []
        t_end = time.perf_counter() + seconds
        while time.perf_counter() < t_end or len(times) < 3:
            w_locals = w_locals_factory()  # fresh dicts: the loop mutates dict 0
            t0 = time.perf_counter()
            O.aggregate_torch(w_locals)
            times.append(time.perf_counter() - t0)
            if len(times) >= max_reps:
                break
        return min(times[1:]), len(times) - 1

    from mfl_amd.synthetic import sample_counts

    g = torch.Generator().manual_seed(0)
    base = torch.randn(P, generator=g) * 0.05
    shift = 7919
    noise = torch.randn(P + K * shift, generator=g) * 1e-3
    rows = torch.empty((K, P))  # client i = base + a shifted window of one noise vector (timing data)
    for i in range(K):
        torch.add(base, noise[i * shift:i * shift + P], out=rows[i])
    del noise, base
    counts = sample_counts(K)
    note(f"flat rows ready: K={K} x P={P} ({4 * K * P / 1e9:.1f} GB); affinity {n_aff} CPUs, OMP cap {n_omp}")
    layouts = []
    k_slice = min(K, 10)
    for label, n in (("affinity", n_aff), ("OMP_NUM_THREADS", n_omp)):
        if n is None:
            continue
        torch.set_num_threads(n)
        t0 = time.perf_counter()
        O.aggregate_torch([(counts[i], {"w": rows[i]}) for i in range(k_slice)])  # warm-up + estimate
        est_full = (time.perf_counter() - t0) * K / k_slice
        Kt = K if est_full <= rep_budget_s else k_slice
        best, reps = timed(lambda: [(counts[i], {"w": rows[i]}) for i in range(Kt)], flat_seconds)
        why = ("the workload" if Kt == K else
               f"K-slice of the workload: one full K={K} reduce at {n} threads would take ~{est_full:.1f} s")
        layouts.append({"layout": "flat", "threads": n, "threads_from": label, "K": Kt,
                        "value": round(algorithmic_bytes(Kt, P) / best / 1e9, 3), "unit": "GB/s",
                        "sample": f"{why}: K={Kt} x P={P} fp32, one flat key per client; best of {reps} reps after "
                                  f"1 warm-up, {best * 1e3:.1f} ms/reduce, {n} torch threads"})
        note(f"flat at {n} threads ({label}): {layouts[-1]['value']} GB/s (K={Kt})")
    del rows
    torch.set_num_threads(n_omp or n_aff)
    Km, shapes = CONFIGS[model]
    Pm = numel(shapes)
    mbase = {k: torch.randn(s, generator=g) * 0.05 for k, s in shapes}
    dicts = []
    for i in range(Km):
        sd = {}
        for k, s in shapes:
            sd[k] = (torch.tensor(1000 + i, dtype=torch.int64) if k.endswith("num_batches_tracked")
                     else mbase[k] + torch.randn(s, generator=g) * 1e-3)
        dicts.append(sd)
    mcounts = sample_counts(Km)
    # 35,000 small ops per reduce: at the box's own share of threads (an
    # oversubscribed team per op would time the scheduler, not the loop)
    n_m = n_omp or n_aff
    torch.set_num_threads(n_m)
    best_m, reps_m = timed(lambda: [(mcounts[0], dict(dicts[0]))] + list(zip(mcounts[1:], dicts[1:])), model_seconds,
                           max_reps=20)
    layouts.append({"layout": f"model-shaped ({model})", "threads": n_m,
                    "threads_from": "OMP_NUM_THREADS" if n_omp else "affinity",
                    "value": round(algorithmic_bytes(Km, Pm) / best_m / 1e9, 3), "unit": "GB/s",
                    "sample": f"{model} state_dicts: K={Km} x P={Pm}, {len(shapes)} keys; best of {reps_m} "
                              f"reps after 1 warm-up, {best_m * 1e3:.1f} ms/reduce, {n_m} torch threads"})
    note(f"model-shaped: {layouts[-1]['value']} GB/s")
    torch.set_num_threads(n_omp or n_aff)
    flat = layouts[0]
    out = {
        "value": flat["value"],
        "unit": "GB/s",
        "cores": n_aff,
        "kind": "port",
        "sample": flat["sample"] + " (value; torch.set_num_threads(len(os.sched_getaffinity(0))), BASELINE.md; "
                                   "threads_from: affinity); reference torch CPU loop restated "
                                   "(oracle/fedavg_oracle.py aggregate_torch)"
                  + (f". NOTE: {n_aff} affinity threads oversubscribe this job's {n_omp}-CPU share "
                     f"(OMP_NUM_THREADS) {n_aff // n_omp}x, so `value` times the scheduler as much as the "
                     f"reference loop; `value_at_share` ({n_omp} threads) is the reference's speed on this box"
                     if n_omp else ""),
        "affinity_cpus": n_aff,
        "layouts": layouts,
    }
    # the figure at the job's own CPU share (OMP_NUM_THREADS on the GPU box):
    # on a shared box the affinity count oversubscribes the share many times
    # over, so `value` times the scheduler as much as the loop
    share = [lay for lay in layouts if lay["layout"] == "flat" and lay["threads_from"] == "OMP_NUM_THREADS"]
    src = share[0] if share else flat
    out["value_at_share"] = src["value"]
    out["value_at_share_threads"] = src["threads"]
    out["value_at_share_K"] = src["K"]
    out["value_at_share_note"] = (f"flat layout at {src['threads']} torch threads "
                                  f"({src['threads_from']}), K={src['K']} x P={P}")
    return out


# ---------------------------------------------------------------------------
# parity: device results vs the oracle on host-derived inputs
# ---------------------------------------------------------------------------
def _oracle_window(K, weights, g0, n):
    sys.path.insert(0, str(ROOT / "oracle"))
    import fedavg_oracle as O
    from mfl_amd.synthetic import client_columns_numpy

    return O.reduce_f32(client_columns_numpy(K, g0, n), weights)


def _bits_equal(a, b) -> bool:
    return a.tobytes() == b.tobytes()


def sampled_parity(red, weights, *, passes=1, pass_cols=0, n_windows=6, width=2048):
    """Windows of this rank's result, bit for bit against the oracle applied to
    the same (client, column) inputs regenerated on the host:

    * local: windows of ``local_out`` (the rank's own columns), including the
      first and last valid column; the host copy too when there is one;
    * gathered (N > 1 or a forced gather): windows of ``full[:P]`` at random
      GLOBAL positions (any rank's columns), and ``full`` == ``local_out`` on
      every column this rank owns;
    * passes > 1 (single-GPU P-chunked passes over one resident buffer):
      windows of every pass's output slice against pass 0's columns."""
    import numpy as np
    import torch

    K = red.K
    plan = red.plan
    segs = plan.local_segments()
    rng = np.random.default_rng(7 + plan.rank)
    checked = 0
    picks = [(segs[0][0], segs[0][1], min(width, segs[0][2])),  # first valid column
             (segs[-1][0] + segs[-1][2] - min(width, segs[-1][2]), segs[-1][1] + segs[-1][2] - min(width, segs[-1][2]),
              min(width, segs[-1][2]))]  # last valid column
    for _ in range(n_windows):
        lstart, gstart, n = segs[int(rng.integers(0, len(segs)))]
        w = min(width, n)
        off = int(rng.integers(0, n - w + 1))
        picks.append((lstart + off, gstart + off, w))
    for l, g, w in picks:
        exp = _oracle_window(K, weights, g, w)
        got = red.local_out[l:l + w].cpu().numpy()
        if not _bits_equal(got, exp):
            return {"ok": False, "columns_checked": checked, "failed": f"local window at global column {g}"}
        if red.host_out is not None and not _bits_equal(red.host_out[g:g + w].numpy(), exp):
            return {"ok": False, "columns_checked": checked, "failed": f"host_out window at {g}"}
        checked += w
    if passes > 1:
        for p in range(1, passes):
            for l, g, w in picks[:3]:
                got = red.pass_out[p * pass_cols + l:p * pass_cols + l + w].cpu().numpy()
                if not _bits_equal(got, _oracle_window(K, weights, g, w)):
                    return {"ok": False, "columns_checked": checked, "failed": f"pass {p} window at {g}"}
                checked += w
    out = {"ok": True, "columns_checked": checked}
    if red.gather:
        P = plan.P
        for _ in range(n_windows):
            w = min(width, P)
            g = int(rng.integers(0, P - w + 1))
            if not _bits_equal(red.full[g:g + w].cpu().numpy(), _oracle_window(K, weights, g, w)):
                return {"ok": False, "columns_checked": checked, "failed": f"gathered window at {g}"}
            checked += w
        for l, g, n in segs:  # the reassembled model holds this rank's columns unchanged
            if not torch.equal(red.full[g:g + n].view(torch.int32), red.local_out[l:l + n].view(torch.int32)):
                return {"ok": False, "columns_checked": checked, "failed": f"full != local_out at {g}"}
        out["gathered_checked"] = True
    out["columns_checked"] = checked
    out["bar"] = "bit-exact vs oracle on host-regenerated inputs (sampled windows, first and last column)"
    return out


def reassembly_checksums(red, dist, dev):
    """Checksum of checksums: every rank sums the int32 bit patterns of its own
    valid columns (int64, exact); all ranks exchange them; each rank then
    recomputes every rank's sum from ITS gathered model at that rank's global
    positions.  A layout or stream-ordering error anywhere in the exchange
    shows up on every rank."""
    import torch

    from mfl_amd.distributed import plan_shards

    plan = red.plan
    ws = plan.world_size

    def csum(t):
        return t.view(torch.int32).to(torch.int64).sum()

    own = torch.zeros(1, dtype=torch.int64, device=dev)
    for l, _, n in plan.local_segments():
        own += csum(red.local_out[l:l + n])
    allsums = torch.zeros(ws, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allsums, own)
    mine = torch.zeros(ws, dtype=torch.int64, device=dev)
    for r in range(ws):
        for _, g, n in plan_shards(plan.P, ws, r, plan.chunks).local_segments():
            mine[r] += csum(red.full[g:g + n])
    return bool(torch.equal(allsums, mine))


def overlap_diagnostics(red, w_dev, steps: int, step_elapsed: float, reps: int = 5) -> dict:
    """N > 1, after the timed region (not part of `value`): the reduce alone
    and the all-gather alone, each timed like a step (barrier + sync on both
    sides, max over ranks), so the JSON line shows how much of the exchange
    the chunked pipeline hides.  overlap = (reduce + gather - step) /
    min(reduce, gather): 1 = fully hidden, 0 = serialised."""
    import torch
    import torch.distributed as dist

    def timed(fn):
        return timed_steps(fn, reps, red.device, True) / reps * 1e3

    gather = red.gather
    red.gather = False
    try:
        reduce_ms = timed(lambda: red.step(w_dev))
    finally:
        red.gather = gather
    gather_ms = timed(red.gather_only)
    step_ms = step_elapsed / steps * 1e3
    recv = (red.plan.padded_P - red.plan.local_cols) * 4
    return {"reduce_only_ms": round(reduce_ms, 4), "gather_only_ms": round(gather_ms, 4), "step_ms": round(step_ms, 4),
            "overlap": round((reduce_ms + gather_ms - step_ms) / max(min(reduce_ms, gather_ms), 1e-9), 3),
            "gather_bytes_in_per_rank": int(recv),
            "gather_GBps_in_per_rank": round(recv / (gather_ms * 1e-3) / 1e9, 1),
            "note": "after the timed region; not part of value"}


def shader_clock_mhz(fn, lead: int = 3, calls: int = 30, window_ms: float = 0.0) -> dict:
    """The shader clock the chip holds while ``fn`` (one launch sequence on the
    current stream) runs back to back: ``lead`` calls, then the clock probe
    (libfedavg_amd_probe's fedavg_probe_clock: 8 one-wave workgroups stamping
    s_memtime / s_memrealtime) on a side stream, then ``calls`` more calls
    covering the probe's window.  MHz = d(memtime) / d(realtime) x 100 per
    workgroup (MI355X_MICROARCH.md 'DVFS give-back' item 6); the median over
    workgroups is reported.  Diagnostic only: after the timed region."""
    import numpy as np
    import torch

    import mfl_amd

    lib = mfl_amd._lib.load_probe()
    cur = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    call_ms = max(a.elapsed_time(b), 1e-3)
    if not window_ms:
        window_ms = 0.6 * calls * call_ms  # inside the calls that follow the probe's launch
    samples = 16
    interval_us = max(1, int(window_ms * 1e3 / samples))
    blocks = 8
    out = torch.zeros(blocks * (samples + 1) * 2, dtype=torch.int64, device=cur.device)
    side = torch.cuda.Stream()
    side.wait_stream(cur)
    for _ in range(lead):
        fn()
    mfl_amd._lib.check(lib.fedavg_probe_clock(out.data_ptr(), blocks, samples, interval_us, side.cuda_stream),
                       "fedavg_probe_clock", lib)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record()
    for _ in range(calls):
        fn()
    c1.record()
    torch.cuda.synchronize()
    st = out.view(blocks, samples + 1, 2).cpu().numpy().astype(np.float64)
    dc, dr = st[:, -1, 0] - st[:, 0, 0], st[:, -1, 1] - st[:, 0, 1]
    mhz = dc / np.maximum(dr, 1) * 100.0
    return {"clock_mhz": round(float(np.median(mhz)), 1), "min": round(float(mhz.min()), 1),
            "max": round(float(mhz.max()), 1), "window_ms": round(float(np.median(dr)) / 1e5, 3),
            "call_ms": round(call_ms, 4), "calls_after_probe": calls,
            # the same calls' own time: clock and time from one window (cycles = ms x MHz)
            "ms_per_call_in_window": round(c0.elapsed_time(c1) / calls, 4),
            "method": "d(s_memtime)/d(s_memrealtime) x 100 MHz, 8 one-wave probe workgroups on a side stream "
                      "beside back-to-back calls; median over workgroups"}


def fused_round(red, w_dev, reps: int = 10) -> dict:
    """N = 1 side measurement of the round's second read: the aggregate plus
    the :291 sums of squares (fedavg_trainer.py:217 then :291) as two passes
    over the rows (fedavg_reduce_f32 + fedavg_client_sqdist_f32) against the
    fused pass (fedavg_reduce_sqdist_f32), interleaved, HIP events around
    each call; the averaged model must keep its bits."""
    import numpy as np
    import torch

    import mfl_amd

    K, P = red.clients.shape[0], red.plan.valid_local_cols()
    rows = red.clients
    o2, o1 = torch.empty(P, device=rows.device), torch.empty(P, device=rows.device)
    runs = {"two_pass": lambda: mfl_amd.client_sqdist(rows, mfl_amd.reduce_packed(rows, w_dev, P, o2), P),
            "fused": lambda: mfl_amd.reduce_with_sqdist(rows, w_dev, P, o1)[1]}
    sums = {n: fn() for n, fn in runs.items()}
    times = {n: [] for n in runs}
    for _ in range(reps):
        for n, fn in runs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            times[n].append((a, b))
    torch.cuda.synchronize()
    ms = {n: float(np.median([a.elapsed_time(b) for a, b in v])) for n, v in times.items()}
    alg = algorithmic_bytes(K, P)
    rel = float(((sums["fused"] - sums["two_pass"]).abs() / sums["two_pass"].abs().clamp_min(1e-300)).max())
    plan = int(mfl_amd._lib.load().fedavg_fused_plan_of(K, P))
    kind, tile, slots = plan // 1000000, (plan // 100) % 10000, plan % 100
    pf = 0 if os.environ.get("FEDAVG_SPLIT_PREFETCH", "") == "0" else 8  # csrc/common.hpp split_prefetch_rows
    kernel = {0: "two passes", 1: f"reduce_sqdist_f32_kernel<S={tile}> (LDS-DMA tiles)",
              2: f"reduce_sqdist_rs_kernel<S={tile},SLOTS={slots}> (register-staged tiles)",
              3: f"reduce_sqdist_win_kernel<KMAX={tile},VEC={slots}> (wave-owned windows)",
              4: f"reduce_sqdist_winn_kernel<KH={tile},VEC=1,NSMAX={slots},PF={pf}> (split-row windows)"}.get(kind, str(plan))
    return {"what": "aggregate + :291 sums of squares over the same resident rows (fedavg_trainer.py:217, :291)",
            "two_pass_ms": round(ms["two_pass"], 4), "fused_ms": round(ms["fused"], 4),
            "speedup": round(ms["two_pass"] / ms["fused"], 3),
            "fused_kernel": kernel,
            "fused_GBps_of_round_bytes": round(alg / ms["fused"] / 1e6, 1),
            "fused_frac_of_hbm_peak": round(alg / ms["fused"] / 1e6 / HBM_PEAK_GBS, 4),
            "out_bits_equal": bool(torch.equal(o1.view(torch.int32), o2.view(torch.int32))),
            "sums_max_rel_vs_two_pass": rel,
            "timing": f"median of {reps} interleaved calls, HIP events around each call",
            **_clock_entry(runs["fused"])}


def _clock_entry(fn) -> dict:
    try:  # a diagnostic: never the reason a measurement is missing
        c = shader_clock_mhz(fn)
        return {"clock_mhz": c["clock_mhz"], "clock": c}
    except Exception as e:  # noqa: BLE001
        return {"clock_mhz": None, "clock": {"error": f"{type(e).__name__}: {e}"}}


def launch_check(args):
    """``--launch-check``: the multi-rank launch path alone, on CPU (gloo) --
    every rank joins the group and all-reduces its rank; rank 0 prints one
    JSON line.  ``--fail-rank R`` makes rank R exit with status 3 (the parent
    must relay a failing rank as a non-zero exit)."""
    import torch
    import torch.distributed as dist

    world, rank = env_int("WORLD_SIZE", 1), env_int("RANK", 0)
    if world > 1:
        dist.init_process_group("gloo")
    if rank == args.fail_rank:
        raise SystemExit(3)
    t = torch.tensor([rank + 1], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "world": world, "rank_sum": int(t.item()),
                          "expected": world * (world + 1) // 2}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _sync(dev) -> None:
    import torch

    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _rehearsal_reduce(clients, weights, P, out):
    """``--cpu-rehearsal`` only: a torch stand-in for the HIP kernel (client 0
    first, mul then add) so the multi-rank bench machinery -- chunk sweep,
    exchange, parity checks, the CPU baseline at N > 1 -- runs on CPU with
    gloo.  Its numbers are not a measurement and the line says so."""
    acc = clients[0, :P] * weights[0]
    for i in range(1, clients.shape[0]):
        acc = acc + clients[i, :P] * weights[i]
    out[:P].copy_(acc)


def timed_steps(step, n: int, dev, use_pg: bool, region=None) -> float:
    """``n`` steps bracketed by barrier + synchronize on both sides; the
    MAX over ranks of the wall time (seconds).  ``region`` (optional): a
    (start, stop) event pair recorded on the current stream right after the
    opening synchronize and right after the last step's launches."""
    import torch
    import torch.distributed as dist

    _sync(dev)
    if use_pg:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    if region is not None:
        region[0].record()
    for _ in range(n):
        step()
    if region is not None:
        region[1].record()
    _sync(dev)
    if use_pg:
        dist.barrier()
    _sync(dev)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if use_pg:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def chunk_candidates(P_global: int, world: int, auto: int) -> list:
    """Pipeline depths the N > 1 warm-up times: 1/2/4/8 chunks and the kernel-
    band rule's pick, each while its chunks keep >= SWEEP_MIN_BLOCK columns."""
    from mfl_amd.distributed import plan_shards

    return [c for c in sorted({auto, *SWEEP_CHUNKS})
            if c == auto or plan_shards(P_global, world, 0, c).block >= SWEEP_MIN_BLOCK]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS), help="default: target")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the workload's P is the global model split over the ranks (BASELINE configs); "
                         "weak: every rank owns P columns")
    ap.add_argument("--chunks", type=int, default=0,
                    help="all-gather pipeline chunks (0 = auto: at N > 1 the fastest step of a warm-up sweep)")
    ap.add_argument("--no-chunk-sweep", action="store_true", help="N>1: take the kernel-band rule's chunk count")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the all-gather (reduce only)")
    ap.add_argument("--force-gather", action="store_true",
                    help="run the RCCL all-gather even at N=1 (world-size-1 nccl group)")
    ap.add_argument("--unroll", type=int, default=0, help="kernel variant: loads in flight per thread")
    ap.add_argument("--nt", type=int, default=-1, help="kernel variant: 1 = nontemporal loads")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true", help="N=1: replay each step from a captured hipGraph")
    ap.add_argument("--traffic-json", default="", help="PMC traffic summary (profiles/*.json) to attach")
    ap.add_argument("--host-out", action="store_true",
                    help="host consumer (SURVEY 8e): D2H each rank's shard into pinned host memory, no collective")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no HIP events in the timed region (no roofline): the events' own cost on the step")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="N=1 only: reduce rank 0's shard of an N-GPU strong-scaled plan (its chunks, no exchange) "
                         "-- the per-rank kernel at the N-GPU geometry, measured on one GPU")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="CPU + gloo, a torch stand-in for the kernel: exercises the multi-rank machinery "
                         "(chunk sweep, exchange, parity, CPU baseline); prints no value")
    ap.add_argument("--launch-check", action="store_true", help="CPU-only: check the multi-rank launch path")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    if args.launch_check:
        return launch_check(args)
    rehearsal = args.cpu_rehearsal
    if args.workload is None:
        args.workload = "rehearsal_small" if rehearsal else "target"
    if rehearsal and (args.graph or args.host_out or args.unroll or args.nt >= 0):
        raise SystemExit("--cpu-rehearsal runs the plain step only")

    import numpy as np
    import torch
    import torch.distributed as dist

    sys.path.insert(0, str(ROOT))
    import mfl_amd
    from mfl_amd import synthetic
    from mfl_amd.distributed import ShardedReducer

    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local_rank = env_int("LOCAL_RANK", 0)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} does not match WORLD_SIZE={world} (one process per GPU)")
    # Rehearsal knobs (a 1-GPU box): FEDAVG_DIST_BACKEND=gloo and
    # FEDAVG_SAME_DEVICE=1 run N ranks on cuda:0.  The driver's runs use the
    # defaults: RCCL ("nccl") with one GPU per rank.
    backend = "gloo" if rehearsal else os.environ.get("FEDAVG_DIST_BACKEND", "nccl")
    if rehearsal:
        dev = torch.device("cpu")
    else:
        dev_index = 0 if os.environ.get("FEDAVG_SAME_DEVICE") == "1" else local_rank
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    use_pg = world > 1 or args.force_gather
    cpu_group = None
    if use_pg:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
            if world > 1:
                # the other ranks wait on a host-side (gloo) barrier while rank 0
                # times the CPU baseline after the timed region: no collective
                # kernel spins on the GPUs meanwhile
                try:
                    cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(minutes=30))
                except Exception as e:  # noqa: BLE001 -- the default group's barrier still works
                    print(f"[bench] gloo side group unavailable ({type(e).__name__}: {e}); "
                          f"the CPU-baseline wait uses the RCCL barrier", file=sys.stderr, flush=True)
        else:
            dist.init_process_group(backend, timeout=datetime.timedelta(minutes=30))
    if not rehearsal:
        mfl_amd._lib.load()

    K, P_w, desc = WORKLOADS[args.workload]
    P_global = P_w if args.scaling == "strong" else P_w * world
    plan_world = world
    if args.shard_of > 1:
        if world != 1 or args.host_out or args.force_gather:
            raise SystemExit("--shard-of is a single-GPU rehearsal without exchange")
        plan_world = args.shard_of
    shard_cols = -(-P_global // plan_world)
    rule_chunks = auto_chunks(K, shard_cols, plan_world, args.host_out)

    # single-GPU workloads larger than the row budget: P-chunked passes
    passes = 1
    if 4 * K * shard_cols > ROW_BUDGET_BYTES:
        if world > 1:
            raise SystemExit(f"{args.workload} needs {4 * K * shard_cols / 1e9:.0f} GB of rows per rank; "
                             f"use more GPUs")
        passes = math.ceil(4 * K * shard_cols / ROW_BUDGET_BYTES)
    P_pass = -(-P_global // passes) if passes > 1 else P_global
    P_pass = (P_pass + 63) // 64 * 64 if passes > 1 else P_pass

    host_out = torch.empty(P_pass, dtype=torch.float32, pin_memory=True) if args.host_out else None
    gather = False if args.no_gather else (True if args.force_gather else None)
    counts = synthetic.sample_counts(K)
    weights = mfl_amd.sample_weights(counts)
    w_dev = (torch.tensor(np.array(weights, np.float64).astype(np.float32)) if rehearsal
             else mfl_amd.weights_tensor(weights, torch.float32, dev))

    def make_reducer(chunks):
        red = ShardedReducer(K, P_pass, chunks=chunks, device=dev, gather=gather, host_out=host_out,
                             as_rank=(plan_world, 0) if plan_world != world else None,
                             local_reduce=_rehearsal_reduce if rehearsal else None)
        synthetic.fill_rows(red.clients, red.plan.local_segments())
        return red

    # N > 1 with the exchange: the pipeline depth is the one whose whole step
    # (reduce + overlapped all-gather) is fastest, timed here in the warm-up on
    # this node (the kernel-band rule optimises the reduce alone, and the
    # strong-scaled N = 8 step is bound by the gather)
    chunk_sweep = None
    sweeping = (world > 1 and args.chunks == 0 and not args.no_chunk_sweep and not args.no_gather
                and not args.host_out and passes == 1)
    if sweeping:
        cands = chunk_candidates(P_global, world, rule_chunks)
        sweep_steps = max(5, min(args.steps, 20))
        ms = {}
        for c in cands:
            red = make_reducer(c)
            for _ in range(max(2, args.warmup)):
                red.step(w_dev)
            ms[c] = timed_steps(lambda: red.step(w_dev), sweep_steps, dev, use_pg) / sweep_steps * 1e3
            del red
            if dev.type == "cuda":
                torch.cuda.empty_cache()
        chunks = min(ms, key=ms.get)
        chunk_sweep = {"step_ms": {str(c): round(v, 4) for c, v in ms.items()}, "chosen": chunks,
                       "rule_choice": rule_chunks, "steps_per_candidate": sweep_steps,
                       "timing": "warm-up, per candidate: barrier + sync, then the steps, max over ranks"}
    else:
        chunks = args.chunks or rule_chunks
    red = make_reducer(chunks)

    tuned = None
    if args.unroll or args.nt >= 0:
        tuned = (args.unroll or 8, max(args.nt, 0))

    S = red.plan.block
    ld = red.clients.stride(0)
    sched = mfl_amd._lib.f32_schedule(K, S, ld) if tuned is None and not rehearsal else None
    launches_per_call = sched["launches"] if sched else 1
    ev_pairs = []

    # Kernel timing, checked against rocprofv3's kernel trace
    # (scripts/launch_timing_probe.py, profiles/r05/launch_timing/ and
    # r05/g3-g4):
    # * one call per pass (N = 1): ONE event pair on the launch stream around
    #   the whole timed region, divided by its launches -- per-launch kernel
    #   time including the back-to-back launch boundaries (~1.7 us each).
    #   Events attached to every launch (fedavg_reduce_f32_timed,
    #   hipExtLaunchKernel: round 5's first form, 704.2 vs rocprofv3's 702.9
    #   us) cost ~4.7 us of GPU time per launch (scripts/step_host_probe.py:
    #   FEMNIST x 10 12.2 vs 7.5 us per call), i.e. ~10 us of every target
    #   step and half of a cache-resident model's; a hipEventRecord marker
    #   before each launch cost ~20 us of step time (r05/g3).
    # * chunked passes (the per-rank kernel of an N-GPU plan, ~46-90 us per
    #   chunk): a hipEventRecord pair on the launch stream around the pass's
    #   chunk launches, which run back to back there (the all-gathers are
    #   issued after the last one, from a side stream), span / chunks --
    #   47.1 vs 46.6 us at 4 x 781K; attached events read ~4 us long PER
    #   CALL (49.9 vs 45.8 us), and a pass spanned by attached events on its
    #   first and last calls picked up the host's issue gaps between chunks.
    # The pool is created and recorded once before the timed region (torch
    # creates HIP events lazily).
    n_spans = args.steps * passes
    pool = []
    if not rehearsal:
        pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(n_spans)]
        for a, b in pool:
            a.record()
            b.record()
    _sync(dev)
    timing_on = [False]
    # one pair around the timed region: only where the region holds nothing but the reduce launches
    # (no exchange, no D2H) -- otherwise the sampled per-pass spans below
    whole = (red.plan.chunks == 1 and tuned is None and not rehearsal and world == 1 and not red.gather
             and host_out is None)

    def timing(c):  # per-launch attached events: not used in the timed region (their cost, above)
        return None

    # chunked passes (and tuning variants): a hipEventRecord pair around the
    # chunk launches of every SPAN_EVERY-th pass (the last one when fewer):
    # a marked pass costs ~8 us of step at the N = 8 rank shape (0.190 vs
    # 0.182 ms, profiles/r05/span_cost/), so the timed region carries few
    n_passes = args.steps * passes
    span_seen = [0]

    def span():
        if not timing_on[0] or rehearsal or whole or args.no_kernel_timing:
            return None
        i = span_seen[0]
        span_seen[0] += 1
        if i % SPAN_EVERY != SPAN_EVERY - 1 and not (i == n_passes - 1 and not ev_pairs):
            return None
        pair = pool[len(ev_pairs)]
        ev_pairs.append(pair)
        return pair

    if tuned is not None:
        def local_reduce(clients, w, P, out):
            mfl_amd.reduce_packed(clients, w, P, out, tuned=tuned)
        red.local_reduce = local_reduce

    if passes > 1:
        # every pass reduces the resident [K, P_pass] rows into its own slice
        # of the [passes * P_pass] model (the pass's columns; the data of
        # pass p is pass 0's buffer -- 400 GB of distinct rows do not fit)
        red.pass_out = torch.empty(passes * red.plan.local_cols, dtype=torch.float32, device=dev)

        def red_step(w):
            for p in range(passes):
                red.local_out = red.pass_out[p * red.plan.local_cols:(p + 1) * red.plan.local_cols]
                red.step(w, timing=timing, span=span())
    else:
        def red_step(w):
            red.step(w, timing=timing, span=span())

    for _ in range(args.warmup):
        red_step(w_dev)
    _sync(dev)

    step = lambda: red_step(w_dev)  # noqa: E731
    if args.graph:
        # one step captured into a hipGraph and replayed: removes the per-step
        # host launch path (Python + ctypes + hipLaunchKernel) that dominates
        # small, cache-resident workloads
        if use_pg:
            raise SystemExit("--graph is single-GPU only (RCCL capture is not used)")
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            red_step(w_dev)  # warm the capture stream
            torch.cuda.synchronize()
            with torch.cuda.graph(graph, stream=s):
                red_step(w_dev)
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
        calls_per_event = red.plan.chunks * passes
        region = None
    else:
        timing_on[0] = True
        calls_per_event = red.plan.chunks  # one span per reduce pass: its chunk calls
        region = None
        if whole and not args.no_kernel_timing:
            region = pool[0]
            ev_pairs.append(region)
            calls_per_event = args.steps * passes  # every reduce call of the timed region
    elapsed_max = timed_steps(step, args.steps, dev, use_pg, region=region)
    timing_on[0] = False

    kernel_ms = [s.elapsed_time(e) / calls_per_event for s, e in ev_pairs]
    kernel_ms_max = float("nan")
    if kernel_ms:
        t = torch.tensor([float(np.mean(kernel_ms))], dtype=torch.float64, device=dev)
        if use_pg:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        kernel_ms_max = float(t[0])

    diagnostics = None
    if world > 1 and red.gather:
        diagnostics = overlap_diagnostics(red, w_dev, args.steps, elapsed_max)
        if chunk_sweep is not None:
            diagnostics["chunk_sweep"] = chunk_sweep

    parity = sampled_parity(red, weights, passes=passes, pass_cols=red.plan.local_cols if passes > 1 else 0)
    if red.gather:
        parity["reassembly_checksums_ok"] = reassembly_checksums(red, dist, dev)
        parity["ok"] = parity["ok"] and parity["reassembly_checksums_ok"]
    if use_pg:
        ok = torch.tensor([1.0 if parity["ok"] else 0.0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        parity["ok"] = bool(ok.item() == 1.0)
        parity["ranks"] = world

    if rank == 0:
        P_done = P_pass * passes if passes > 1 else P_global
        if plan_world != world:
            P_done = red.plan.valid_local_cols()  # the one shard this GPU reduced
        bytes_step = algorithmic_bytes(K, P_done)
        value = bytes_step * args.steps / elapsed_max / 1e9
        roofline = None
        if not rehearsal and not args.no_kernel_timing:
            timing_desc = ("one HIP event pair on the launch stream around the whole timed region (recorded "
                           "after the opening barrier + synchronize and after the last step's launches), divided "
                           "by the region's reduce launches: kernel time incl. the back-to-back launch boundaries"
                           if whole else
                           f"hipEventRecord pair on the launch stream around a reduce pass's back-to-back chunk "
                           f"launches, every {SPAN_EVERY}th pass of the timed region ({len(ev_pairs)} of "
                           f"{args.steps * passes}), span / chunks")
            roofline = roofline_entry(args, K, S, kernel_ms_max, launches_per_call, sched, tuned, timing_desc,
                                      len(kernel_ms) * calls_per_event * launches_per_call, world)
        if red.gather:
            exchange = ("rccl" if backend == "nccl" else backend) + " all_gather_into_tensor, overlapped per chunk"
        elif host_out is not None:
            exchange = "none: each rank D2Hs its shard chunks into pinned host memory (host consumer)"
        else:
            exchange = "none (single GPU or --no-gather)"
        config = {
            "workload": desc,
            "K": K,
            "P_total": P_done,
            "P_per_gpu": red.plan.valid_local_cols() * passes,
            "scaling_mode": args.scaling,
            "chunks": red.plan.chunks,
            "chunks_from": ("warm-up step sweep (diagnostics.chunk_sweep)" if chunk_sweep is not None else
                            ("--chunks" if args.chunks else "kernel-band rule (bench.auto_chunks)")),
            "chunk_cols": S,
            "exchange": exchange,
            "parallelism": f"p-shard{world}",
            "kernel_variant": {"unroll": tuned[0], "nt": tuned[1]} if tuned else "default",
            "launch": "hipGraph replay" if args.graph else "eager (stream-ordered)",
        }
        if plan_world != world:
            config["rehearsal"] = (f"rank 0's shard of the {plan_world}-GPU strong-scaled plan of {K} x {P_global}, "
                                   f"reduced on one GPU in its {red.plan.chunks} chunks, no exchange; value counts "
                                   f"this shard only")
        if passes > 1:
            config["passes"] = passes
            config["pass_note"] = (f"{K} x {P_done} fp32 = {4 * K * P_done / 1e9:.0f} GB of rows exceeds one GPU; "
                                   f"{passes} P-chunked passes over one resident {K} x {P_pass} buffer "
                                   f"(each pass streams it from HBM; time = sum of passes)")
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-generated counter-hash uniform, base std 0.05 + per-client std 1e-3, "
                    "reproducible on the host; counts U{1..1000})",
            "config": config,
            "roofline": roofline,
            # the whole step against the node's HBM-read roofline (N x 8 TB/s):
            # north_star's "fraction of the HBM-read roofline" at N GPUs
            "step_frac_of_node_hbm": round(value / (world * HBM_PEAK_GBS), 4),
            "parity": parity,
        }
        if rehearsal:
            out["rehearsal"] = ("CPU + gloo with a torch stand-in for the HIP kernel: exercises the multi-rank "
                                "machinery only; NOT a measurement")
            out["rehearsal_value"] = out["value"]
            out["value"] = None
            out["dtype"] = "f32"
        if diagnostics is not None:
            out["diagnostics"] = diagnostics
        if world > 1 or plan_world > 1:
            out["north_star"] = north_star_block(args.workload, plan_world, roofline, out["step_frac_of_node_hbm"],
                                                 args.scaling, measured_world=world)
        if not rehearsal and world == 1 and passes == 1:
            # the shader clock the chip held under the timed kernel's load (same launches, after
            # the timed region): box-to-box spread in GB/s vs DVFS, by measurement
            clk = _clock_entry(lambda: red_step(w_dev))
            out["clock_mhz"] = clk["clock_mhz"]
            if roofline is not None:
                roofline["clock"] = clk["clock"]
        if (not rehearsal and world == 1 and passes == 1 and plan_world == 1 and K <= 1024
                and red.plan.chunks == 1):
            try:  # a side measurement: never the reason the bench line is missing
                out["round_with_distances"] = fused_round(red, w_dev)
            except Exception as e:  # noqa: BLE001
                out["round_with_distances"] = {"error": f"{type(e).__name__}: {e}"}
        if not args.no_cpu_baseline and world > 1:
            # the bench contract times the CPU baseline on rank 0 at N = 1 only:
            # an N-GPU line points at that run instead of spending 10-30 s of
            # the job's host time on the same number again
            out["cpu_baseline"] = {"value": None, "n_gpus_in_run": world,
                                   "note": "timed at N = 1 only (rank 0 of the 1-GPU run's line)"}
        elif not args.no_cpu_baseline:
            # on rank 0 after the timed region and the parity checks: the
            # workload's own K x P while its rows fit a bounded host sample
            # (<= 10 GB: the target); cfg5's 400 GB is timed on a P-slice
            try:
                if rehearsal:
                    out["cpu_baseline"] = cpu_baseline(K, P_global, flat_seconds=0.2, model_seconds=0.2,
                                                       model="mnist_lr")
                else:
                    out["cpu_baseline"] = cpu_baseline(K, min(P_global, 10_000_000_000 // (4 * K)))
                out["cpu_baseline"]["n_gpus_in_run"] = world
            except Exception as e:  # noqa: BLE001 -- never the reason the bench line is missing
                out["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
        print(json.dumps(out), flush=True)
    if use_pg:
        # the ranks leave together once rank 0 has printed (a host-side barrier
        # when the gloo side group exists: rank 0's CPU baseline runs 10-30 s)
        dist.barrier(group=cpu_group)
        dist.destroy_process_group()


NORTH_STAR_BAR = 0.70  # BASELINE.json north_star: >= 70 % of per-GPU HBM-read roofline at 1 and 8 GPUs
PREDICTION = ROOT / "profiles" / "r06" / "scale_prediction.json"  # scripts/predict_scale.py


def north_star_block(workload: str, n: int, roofline, step_frac: float, scaling: str, measured_world: int) -> dict:
    """north_star's bar against this line: the per-rank kernel fraction (each
    GPU's reduce launch against its own 8 TB/s -- the quantity the bar is
    met on) and the whole step against the node's N x 8 TB/s (which a
    strong-scaled step cannot reach once the RCCL all-gather over xGMI is
    longer than the per-rank reduce), next to the written prediction for this
    workload and N (profiles/r06/scale_prediction.json)."""
    kfrac = roofline.get("frac") if roofline else None
    block = {
        "bar": NORTH_STAR_BAR,
        "met_on": "per_rank_kernel_frac",
        "per_rank_kernel_frac": kfrac,
        "per_rank_kernel_meets_bar": None if kfrac is None else bool(kfrac >= NORTH_STAR_BAR),
        "step_frac_of_node_hbm": step_frac,
        "step_meets_bar": bool(step_frac >= NORTH_STAR_BAR) if step_frac is not None else None,
        "why_step_differs": ("strong scaling: every rank reduces P/N columns (HBM-bound, the per-rank kernel) and "
                             "receives (N-1)/N x 4P bytes in the RCCL all-gather over xGMI; at the target's N = 8 "
                             "that exchange (87.5 MB in per rank) is longer than the 0.18 ms reduce, so the step is "
                             "exchange-bound and its node-HBM fraction is not the bar's quantity"),
    }
    if scaling == "strong" and PREDICTION.exists():
        try:
            pred = json.loads(PREDICTION.read_text())["workloads"].get(workload, {}).get(str(n))
        except (ValueError, OSError):
            pred = None
        if pred is not None:
            block["prediction"] = {"per_rank_kernel_frac": pred["per_rank_kernel_frac"],
                                   "bound": pred["bound"],
                                   "step_ms": [pred["predicted"]["high"]["step_ms"], pred["predicted"]["low"]["step_ms"]],
                                   "value_GBps": [pred["predicted"]["low"]["value_GBps"],
                                                  pred["predicted"]["high"]["value_GBps"]],
                                   "step_frac_of_node_hbm": [pred["predicted"]["low"]["step_frac_of_node_hbm"],
                                                             pred["predicted"]["high"]["step_frac_of_node_hbm"]],
                                   "source": "profiles/r06/scale_prediction.json (xGMI in-rate 153 GB/s .. "
                                             "0.75 x (N-1) x 153 GB/s per rank; DESIGN.md section 7)"}
    if measured_world != n:
        block["note"] = f"--shard-of {n} rehearsal on {measured_world} GPU: no exchange, so the step fraction is the reduce's"
    return block


def roofline_entry(args, K, S, kernel_ms_max, launches_per_call, sched, tuned, timing_desc, launches, world):
    """The dominant kernel's algorithmic bytes per launch over its average
    launch time (HIP events on the launch stream, ``timing_desc``), with the
    PMC traffic of the same launch shape when profiles/ holds it."""
    bytes_call = algorithmic_bytes(K, S)
    achieved = bytes_call / (kernel_ms_max * 1e-3) / 1e9
    if sched:
        kname = f"{sched['kernel']}<U={sched['unroll']},C={sched['cols']},nt={min(1, sched['nontemporal'])}"
        if sched.get("block", 256) != 256:
            kname += f",B={sched['block']}"
        kname += f"> (exact, sequential client order; round-split x{launches_per_call})"
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
        "launches": launches,
        "timing": "hipGraph replay bracketed by events" if args.graph else timing_desc,
    }
    attach_traffic(roofline, args, world)
    return roofline


def attach_traffic(roofline: dict, args, world: int) -> None:
    """PMC traffic for this launch shape: the summaries under profiles/ hold
    per-launch HBM bytes for the launch geometries they were collected on
    (``traffic_<workload>.json`` at N = 1, ``traffic_<workload>_shard<N>.json``
    for one rank of an N-GPU plan, optionally a ``launches`` list).  An exact
    geometry match gives the measured bytes; otherwise the same kernel's PMC
    traffic/algorithmic ratio is applied to this launch and labelled so."""
    n = args.shard_of if args.shard_of > 1 else world
    cands = [args.traffic_json] if args.traffic_json else []
    if n > 1:
        cands.append(str(ROOT / "profiles" / f"traffic_{args.workload}_shard{n}.json"))
    cands.append(str(ROOT / "profiles" / f"traffic_{args.workload}.json"))
    entries = []
    for tj in cands:
        if not Path(tj).exists():
            continue
        try:
            tr = json.loads(Path(tj).read_text())
        except (ValueError, OSError):
            continue
        src = os.path.relpath(tj, ROOT)
        for e in [tr, *tr.get("launches", [])]:
            if "algorithmic_bytes_per_launch" in e:
                entries.append((src, e))
    for src, e in entries:
        if e.get("algorithmic_bytes_per_launch") == roofline["bytes_per_launch"] and e.get("hbm_bytes_per_launch"):
            roofline["traffic"] = int(e["hbm_bytes_per_launch"])
            roofline["traffic_source"] = f"{src} (PMC, this launch shape)"
            return
    for src, e in entries:
        if e.get("traffic_over_algorithmic"):
            ratio = float(e["traffic_over_algorithmic"])
            roofline["traffic"] = int(round(ratio * roofline["bytes_per_launch"]))
            roofline["traffic_source"] = (f"{src} (PMC ratio {ratio} of a {e['algorithmic_bytes_per_launch']}-B launch "
                                          f"x this launch's algorithmic bytes; not this geometry)")
            return


def side_bench(argv) -> bool:
    """``bench.py --e2e ...`` / ``bench.py --fpf ...``: the host-in/host-out
    rate of the drop-in (scripts/bench_e2e.py) and the FPF2 bookkeeping per
    round (scripts/bench_fpf.py), each beside its CPU baseline -- the
    reference's torch expressions (oracle/), handed in from here."""
    if not argv or argv[0] not in ("--e2e", "--fpf"):
        return False
    sys.path.insert(0, str(ROOT))
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
    _argv = sys.argv[1:]
    _rc = self_launch(_argv)
    if _rc is not None:
        sys.exit(_rc)
    if not side_bench(_argv):
        main(_argv)
