"""Zero-copy (segments) reduce vs the row reduce, on the same bytes.

    python scripts/segments_probe.py [--K 100 --P 25000000] [--rounds 4] [--reps 8] [--sweep]

Three variants, interleaved in one process, all bit-identical:
  rows         production reduce on one [K, ld] buffer (fedavg_reduce_f32),
  seg-rows     fedavg_reduce_segments_f32 with the pointers set to the rows of
               that same buffer (one key of P elements per client),
  seg-tensors  fedavg_reduce_segments_f32 on K separately allocated client
               tensors (the device-resident drop-in's case),
  *-pow2-pitch the first two on rows at a power-of-two pitch (128 MiB),
  ptrs-*       fedavg_reduce_ptrs_f32 (device pointer array) on the rows and
               on the separate tensors,
  seg-skewed-tensors  K separate allocations whose client starts are skewed
               by k * 37 mod 64 x 256 B (the allocator's 2 MiB-congruent
               starts broken, the allocations -- and their translations -- kept),
  seg-2mib-pitch  one buffer, rows at a 2 MiB-multiple pitch (congruent
               starts, one allocation); with --names pick a subset.
Separates the kernel's own cost from where the clients' memory lies.  One
JSON line per variant: median ms per call (HIP events) and GB/s.
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


def model_mode(args, dev, lib):
    """Multi-key models (scripts/bench_e2e.py shapes) as K separately allocated
    device state_dicts: production zero-copy reduce vs (U, C, blocks/CU)
    schedules of fedavg_reduce_segments_f32_variant, interleaved, bits checked."""
    sys.path.insert(0, str(ROOT / "scripts"))
    from bench_e2e import CONFIGS
    K, shapes = CONFIGS[args.model]
    g = torch.Generator(device=dev).manual_seed(4)
    clients = []
    for _ in range(K):
        sd = []
        for name, shp in shapes:
            if name.endswith("num_batches_tracked"):
                sd.append(torch.randint(0, 1000, shp, generator=g, device=dev))
            else:
                sd.append(torch.randn(shp, generator=g, device=dev) * 0.05)
        clients.append(sd)
    numel = np.array([t.numel() for t in clients[0]], dtype=np.int64)
    offset = np.concatenate([[0], np.cumsum(numel)[:-1]]).astype(np.int64)
    kind = np.array([1 if t.dtype == torch.int64 else 0 for t in clients[0]], dtype=np.int64)
    ptrs = np.array([[t.data_ptr() for t in sd] for sd in clients], dtype=np.int64)
    P = int(numel.sum())
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    nk = len(numel)
    need = lib.fedavg_segments_workspace(K, nk)
    stream = torch.cuda.current_stream(dev)
    sched = [None] + ([tuple(int(t) for t in v.split(",")) for v in args.sched] if args.sched else
                      [(4, 8, 3), (2, 16, 3), (4, 4, 3), (1, 16, 3), (8, 4, 3), (2, 8, 3)])
    names = ["production" if v is None else f"U{v[0]}C{v[1]}b{v[2]}" for v in sched]
    ws = {n: (torch.empty(need, dtype=torch.uint8, pin_memory=True), torch.empty(need, dtype=torch.uint8, device=dev))
          for n in names}
    outs = {n: torch.empty(P, device=dev) for n in names}
    a = (ptrs.ctypes.data, numel.ctypes.data, offset.ctypes.data, kind.ctypes.data, nk, K, w.data_ptr())

    def run(n, v):
        h, d = ws[n]
        if v is None:
            rc = lib.fedavg_reduce_segments_f32(*a, outs[n].data_ptr(), h.data_ptr(), d.data_ptr(), need,
                                                stream.cuda_stream)
        else:
            rc = lib.fedavg_reduce_segments_f32_variant(*a, outs[n].data_ptr(), h.data_ptr(), d.data_ptr(), need,
                                                        v[0], v[1], v[2], stream.cuda_stream)
        mfl_amd._lib.check(rc, n)

    for n, v in zip(names, sched):
        run(n, v)
    torch.cuda.synchronize()
    same = {n: bool(torch.equal(outs[n].view(torch.int32), outs["production"].view(torch.int32))) for n in names}
    times = {n: [] for n in names}
    for _ in range(args.rounds):
        for n, v in zip(names, sched):
            for _ in range(args.reps):
                s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                run(n, v)
                e0.record()
                times[n].append((s0, e0))
            torch.cuda.synchronize()  # the pinned table of the next call
    alg = 4 * K * P + 4 * P + 4 * K
    for n in names:
        ms = float(np.median([s0.elapsed_time(e0) for s0, e0 in times[n]]))
        print(json.dumps({"model": args.model, "variant": n, "K": K, "P": P, "keys": nk, "ms_median": round(ms, 4),
                          "GBps": round(alg / ms / 1e6, 1), "bit_identical": same[n]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--sweep", action="store_true",
                    help="also time fedavg_reduce_segments_f32_variant schedules (U, C, blocks per CU) on the "
                         "separate tensors and on the rows")
    ap.add_argument("--model", default="", help="multi-key mode: a scripts/bench_e2e.py config name")
    ap.add_argument("--sched", nargs="*", default=[], help="multi-key mode: U,C,blocks_per_cu variants to time")
    ap.add_argument("--only", default="", help="time only 'rows' and this variant (for per-kernel PMC passes)")
    ap.add_argument("--names", nargs="*", default=[], help="time only these variants ('rows' is always timed)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    if args.model:
        model_mode(args, dev, lib)
        return
    K, P = args.K, args.P
    ld = (P + 63) // 64 * 64
    rows = torch.empty((K, ld), device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    tensors = []
    for k in range(K):
        t = torch.randn(P, generator=g, device=dev) * 0.05
        rows[k, :P].copy_(t)
        tensors.append(t)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    # rows of one buffer at a power-of-two pitch (128 MiB for P=25M): do
    # congruent client starts alone cost the separate tensors their rate?
    ld2 = 1 << max(0, (P - 1).bit_length())
    rows2 = torch.empty((K, ld2), device=dev)
    rows2[:, :P].copy_(rows[:, :P])
    # separate allocations with skewed starts (each padded by up to 16 KiB)
    skew = [(k * 37 % 64) * 64 for k in range(K)]  # floats: multiples of 256 B
    skewed = []
    for k in range(K):
        buf = torch.empty(P + 64 * 64, device=dev)
        buf[skew[k]:skew[k] + P].copy_(tensors[k])
        skewed.append(buf[skew[k]:skew[k] + P])
    # one buffer, pitch rounded up to 2 MiB (every row start congruent mod 2 MiB)
    ld3 = (P * 4 + (2 << 20) - 1) // (2 << 20) * (2 << 20) // 4
    rows3 = torch.empty((K, ld3), device=dev)
    rows3[:, :P].copy_(rows[:, :P])
    names = ["rows", "rows-pow2-pitch", "seg-rows", "seg-pow2-pitch", "seg-tensors", "ptrs-rows", "ptrs-tensors",
             "seg-skewed-tensors", "seg-2mib-pitch"]
    sched = [(4, 8, 3), (4, 8, 0), (4, 8, 2), (4, 8, 4), (4, 8, 6), (8, 4, 3), (8, 4, 6), (2, 8, 3), (2, 8, 6),
             (4, 4, 3), (4, 4, 6), (8, 2, 6), (16, 2, 3), (2, 16, 3), (1, 16, 3), (1, 16, 6)]
    if args.sweep:
        names += [f"var-{src}-U{u}C{c}b{b}" for src in ("tensors", "rows", "skewed") for u, c, b in sched]
    if args.only:
        names = ["rows", args.only]
    if args.names:
        names = ["rows"] + [n for n in args.names if n != "rows"]
    outs = {n: torch.empty(P, device=dev) for n in names}
    meta = [np.array([v], dtype=np.int64) for v in (P, 0, 0)]
    ptr_rows = np.array([[rows[k].data_ptr()] for k in range(K)], dtype=np.int64)
    ptr_tens = np.array([[t.data_ptr()] for t in tensors], dtype=np.int64)
    ptr_pow2 = np.array([[rows2[k].data_ptr()] for k in range(K)], dtype=np.int64)
    ptr_skew = np.array([[t.data_ptr()] for t in skewed], dtype=np.int64)
    ptr_2mib = np.array([[rows3[k].data_ptr()] for k in range(K)], dtype=np.int64)
    starts = [int(t.data_ptr()) for t in tensors]
    print(json.dumps({"tensor_start_alignment_log2": [min(31, (a & -a).bit_length() - 1) for a in starts[:8]],
                      "skewed_start_mod_2mib": [int(t.data_ptr()) % (2 << 20) for t in skewed[:8]],
                      "pitch_bytes_rows": ld * 4, "pitch_bytes_pow2": ld2 * 4, "pitch_bytes_2mib": ld3 * 4}),
          flush=True)
    dptrs = {"ptrs-rows": torch.from_numpy(ptr_rows[:, 0].copy()).to(dev),
             "ptrs-tensors": torch.from_numpy(ptr_tens[:, 0].copy()).to(dev)}
    need = lib.fedavg_segments_workspace(K, 1)
    ws = {n: (torch.empty(need, dtype=torch.uint8, pin_memory=True), torch.empty(need, dtype=torch.uint8, device=dev))
          for n in names if n.startswith(("seg-", "var-"))}
    stream = torch.cuda.current_stream(dev)

    def run(n):
        if n == "rows":
            mfl_amd.reduce_packed(rows, w, P, outs[n])
            return
        if n == "rows-pow2-pitch":
            mfl_amd.reduce_packed(rows2, w, P, outs[n])
            return
        if n in dptrs:  # fedavg_reduce_ptrs_f32: device pointer array, no table staging
            mfl_amd._lib.check(lib.fedavg_reduce_ptrs_f32(dptrs[n].data_ptr(), K, P, w.data_ptr(), outs[n].data_ptr(),
                                                          stream.cuda_stream), n)
            return
        h, d = ws[n]
        if n.startswith("var-"):
            _, src, uc = n.split("-")
            u, rest = uc[1:].split("C")
            c, b = rest.split("b")
            ptrs = {"tensors": ptr_tens, "rows": ptr_rows, "skewed": ptr_skew}[src]
            mfl_amd._lib.check(lib.fedavg_reduce_segments_f32_variant(
                ptrs.ctypes.data, meta[0].ctypes.data, meta[1].ctypes.data, meta[2].ctypes.data, 1, K, w.data_ptr(),
                outs[n].data_ptr(), h.data_ptr(), d.data_ptr(), need, int(u), int(c), int(b), stream.cuda_stream), n)
            return
        ptrs = {"seg-rows": ptr_rows, "seg-pow2-pitch": ptr_pow2, "seg-tensors": ptr_tens,
                "seg-skewed-tensors": ptr_skew, "seg-2mib-pitch": ptr_2mib}[n]
        mfl_amd._lib.check(lib.fedavg_reduce_segments_f32(ptrs.ctypes.data, meta[0].ctypes.data, meta[1].ctypes.data,
                                                          meta[2].ctypes.data, 1, K, w.data_ptr(), outs[n].data_ptr(),
                                                          h.data_ptr(), d.data_ptr(), need, stream.cuda_stream), n)

    for n in outs:
        run(n)
    torch.cuda.synchronize()
    same = {n: bool(torch.equal(outs[n].view(torch.int32), outs["rows"].view(torch.int32))) for n in outs}
    times = {n: [] for n in outs}
    for _ in range(args.rounds):
        for n in outs:
            for _ in range(args.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run(n)
                e.record()
                times[n].append((s, e))
            torch.cuda.synchronize()  # the pinned table of the next call
    alg = 4 * K * P + 4 * P + 4 * K
    for n in outs:
        ms = float(np.median([s.elapsed_time(e) for s, e in times[n]]))
        print(json.dumps({"variant": n, "K": K, "P": P, "ms_median": round(ms, 4), "GBps": round(alg / ms / 1e6, 1),
                          "bit_identical": same[n]}), flush=True)


if __name__ == "__main__":
    main()
