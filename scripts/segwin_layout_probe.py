"""Does the device clients' memory layout set the zero-copy fused kernel's time?

    python scripts/segwin_layout_probe.py --layout separate|arena|shuffled [--config resnet56] [--calls 30]

The same device round (fedavg_device_round_f32, fused) on the same values,
with the clients' tensors placed three ways:
  separate : one torch allocation per tensor (the caching allocator packs the
             small ones into 2 MB segments), as KeyTable.collect sees real
             device-resident clients;
  arena    : one allocation for the whole round, client after client, each
             key 256-B aligned (not the packed [K, ld] layout the row
             kernel's arena check accepts);
  shuffled : the same arena, the (client, key) tensors at shuffled slots;
  packed   : the [K, ld] rows layout (client i's key j at i * ld + offset_j),
             so the same bytes also run the row kernel (fedavg_reduce_sqdist_f32,
             `rows_gpu_us_*`) -- the host rows' fused pass the device round is
             held against.
Run under rocprofv3 --kernel-trace --stats: the kernels' average durations
per layout answer whether address translation (many 2 MB segments per
window) or the kernel's own structure costs the time against the packed
rows' fused pass.  Prints one JSON line with the layout and an event-timed
median per call (the tables' H2D, the integer-key pass, the fused kernel
and the sums' finalize).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd
from host_cost_probe import device_clients


def relayout(dicts, layout, dev):
    if layout == "separate":
        return dicts, None
    if layout == "packed":
        table = mfl_amd.KeyTable(dicts[0])
        g = table.groups[torch.float32]
        K, ld = len(dicts), g.ld
        rows = torch.empty((K, ld), device=dev)
        out = []
        for i, sd in enumerate(dicts):
            nd = type(sd)()
            for e in table.entries:
                t = sd[e.name]
                if t.dtype == torch.float32:
                    v = rows[i, e.offset:e.offset + e.numel].view(t.shape)
                    v.copy_(t)
                    nd[e.name] = v
                else:
                    nd[e.name] = t
            out.append(nd)
        return out, rows
    slots = [(i, k) for i, sd in enumerate(dicts) for k in sd]
    sizes = {(i, k): (dicts[i][k].numel() * dicts[i][k].element_size() + 255) // 256 * 256 for i, k in slots}
    order = list(slots)
    if layout == "shuffled":
        rng = np.random.default_rng(7)
        order = [order[j] for j in rng.permutation(len(order))]
    total = sum(sizes.values())
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    off, where = 0, {}
    for s in order:
        where[s] = off
        off += sizes[s]
    out = []
    for i, sd in enumerate(dicts):
        nd = type(sd)()
        for k, t in sd.items():
            o = where[(i, k)]
            v = arena[o:o + t.numel() * t.element_size()].view(t.dtype).view(t.shape)
            v.copy_(t)
            nd[k] = v
        out.append(nd)
    return out, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="separate", choices=["separate", "arena", "shuffled", "packed"])
    ap.add_argument("--config", default="resnet56")
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--clients", type=int, default=0, help="the config's first N clients (0: all)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load()
    counts, dicts = device_clients(args.config, dev)
    if args.clients:
        counts, dicts = counts[:args.clients], dicts[:args.clients]
    dicts, rows = relayout(dicts, args.layout, dev)
    torch.cuda.synchronize()
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
    partials = torch.empty(max(1, lib.fedavg_reduce_sqdist_segments_partials(K)), dtype=torch.float64, device=dev)
    sumsq = torch.empty(K, dtype=torch.float64, device=dev)
    n_s = lib.fedavg_device_round_scratch(numel.ctypes.data, kind.ctypes.data, n, K)
    scr = torch.empty(max(1, n_s), device=dev)
    need = lib.fedavg_device_round_workspace(K, n)
    ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    ws_d = torch.empty(need, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    ts = []
    for _ in range(args.calls):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        rc = lib.fedavg_device_round_f32(ptrs.ctypes.data, n_cols, ki.ctypes.data, numel.ctypes.data,
                                         offset.ctypes.data, kind.ctypes.data, n, K, w64.ctypes.data, out.data_ptr(),
                                         partials.data_ptr(), partials.numel(), sumsq.data_ptr(), scr.data_ptr(),
                                         scr.numel(), ws_h.data_ptr(), ws_d.data_ptr(), need, stream.cuda_stream)
        e1.record(stream)
        assert rc in (0, 1), rc  # 1: a source not 16-B aligned (packed keys), the reduce alone ran
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    rec = {"layout": args.layout, "config": args.config, "K": K, "keys": n, "fused": rc == 0,
           "round_gpu_us_median": round(float(np.median(ts)), 2), "round_gpu_us_min": round(float(np.min(ts)), 2),
           "out_checksum": float(out.double().sum()), "sums_checksum": float(sumsq.sum())}
    if rows is not None:  # the row kernel on the same bytes (int keys are not in these rows: fp32 keys only)
        w_dev = torch.tensor(w64, dtype=torch.float32, device=dev)
        out_r = torch.empty(g.P, device=dev)
        tr = []
        for _ in range(args.calls):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            mfl_amd.reduce_with_sqdist(rows, w_dev, g.P, out_r)
            e1.record(stream)
            torch.cuda.synchronize()
            tr.append(e0.elapsed_time(e1) * 1e3)
        rec["rows_gpu_us_median"] = round(float(np.median(tr)), 2)
        rec["rows_gpu_us_min"] = round(float(np.min(tr)), 2)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
