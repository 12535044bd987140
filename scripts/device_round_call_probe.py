"""Host cost of one fedavg_device_round_f32 call at a model's shape.

    python scripts/device_round_call_probe.py [--config resnet56] [--calls 50]

Device clients as scripts/host_cost_probe.py builds them; the walk's address
table from KeyTable.collect; then the native call alone, timed per call
(each followed by a stream synchronize outside the timed region), in its
forms: fused with the integer keys' scratch (production), the reduce alone
(no conversion), fused right after a fresh walk (the address table just
written by the walker threads, as in a round), the walk itself
(KeyTable.collect) at 1, 2, 4, 8 and all intra-op threads, the call's host
phases after a walk (probe library build, fedavg_device_round_phases), and, for scale, hipPointerGetAttributes and an empty
hipMemcpyAsync-sized H2D of the table bytes through torch.  One JSON line
per form with the median and min call time in microseconds.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd
from host_cost_probe import device_clients


def timed(fn, calls, sync=True, setup=None):
    ts = []
    for _ in range(calls):
        if setup is not None:
            setup()
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
        if sync:
            torch.cuda.synchronize()
    return round(float(np.median(ts)), 2), round(float(np.min(ts)), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="resnet56")
    ap.add_argument("--calls", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load()
    counts, dicts = device_clients(args.config, dev)
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
    s = torch.cuda.current_stream(dev).cuda_stream

    cur = {"ptrs": ptrs}

    def walk():  # a fresh address table, written by the walker threads as in a round
        cur["ptrs"] = table.collect(dicts, dev)[0]

    def call(sums):
        rc = lib.fedavg_device_round_f32(cur["ptrs"].ctypes.data, n_cols, ki.ctypes.data, numel.ctypes.data,
                                         offset.ctypes.data, kind.ctypes.data, n, K, w64.ctypes.data, out.data_ptr(),
                                         partials.data_ptr(), partials.numel(), sumsq.data_ptr() if sums else None,
                                         scr.data_ptr(), scr.numel(), ws_h.data_ptr(), ws_d.data_ptr(), need, s)
        assert rc in (0, 1), rc

    recs = {"config": args.config, "K": K, "keys": n, "int_keys": int(np.count_nonzero(kind)),
            "ws_bytes": need}
    recs["fused_us"] = timed(lambda: call(True), args.calls)
    recs["reduce_only_us"] = timed(lambda: call(False), args.calls)
    recs["fused_after_walk_us"] = timed(lambda: call(True), args.calls, setup=walk)
    # the same call from the probe library, which records its host phases
    try:
        probe = mfl_amd._lib.load_probe()
    except Exception:  # noqa: BLE001 -- probe library not built
        probe = None
    if probe is not None:
        names = ["checks", "key_validation", "fill", "spot_check", "plan_keys_weights", "h2d_issue",
                 "int_launch", "reduce_launches"]
        buf = (ctypes.c_double * 10)()
        ph = {nm: [] for nm in names}
        for _ in range(args.calls):
            walk()
            rc = probe.fedavg_device_round_f32(cur["ptrs"].ctypes.data, n_cols, ki.ctypes.data, numel.ctypes.data,
                                               offset.ctypes.data, kind.ctypes.data, n, K, w64.ctypes.data,
                                               out.data_ptr(), partials.data_ptr(), partials.numel(),
                                               sumsq.data_ptr(), scr.data_ptr(), scr.numel(), ws_h.data_ptr(),
                                               ws_d.data_ptr(), need, s)
            assert rc == 0, rc
            m = probe.fedavg_device_round_phases(buf, 10)
            for i, nm in enumerate(names[: m - 1]):
                ph[nm].append(buf[i + 1] - buf[i])
            torch.cuda.synchronize()
        recs["phases_after_walk_us"] = {nm: round(float(np.median(v)), 2) for nm, v in ph.items() if v}
    nt = torch.get_num_threads()
    for t in sorted({1, 2, 4, 8, nt}):
        torch.set_num_threads(t)
        recs[f"walk_us_threads_{t}"] = timed(walk, args.calls, sync=False)
    torch.set_num_threads(nt)
    # the walk's fixed part: one client, and the [K, N] address table's allocation
    recs["walk_us_one_client"] = timed(lambda: table.collect(dicts[:1], dev), args.calls, sync=False)
    recs["alloc_table_us"] = timed(lambda: torch.empty((K, n_cols), dtype=torch.int64), args.calls, sync=False)
    hip = ctypes.CDLL("libamdhip64.so")
    attr = ctypes.create_string_buffer(256)
    p = ctypes.c_void_p(out.data_ptr())
    recs["hipPointerGetAttributes_us"] = timed(lambda: hip.hipPointerGetAttributes(attr, p), args.calls, sync=False)
    hp = ctypes.c_void_p(ws_h.data_ptr())
    recs["hipPointerGetAttributes_pinned_us"] = timed(lambda: hip.hipPointerGetAttributes(attr, hp), args.calls,
                                                      sync=False)
    src = ws_h[: need // 2]
    dst = ws_d[: need // 2]
    recs["h2d_copy_issue_us"] = timed(lambda: dst.copy_(src, non_blocking=True), args.calls)
    torch.cuda.synchronize()
    print(json.dumps(recs), flush=True)


if __name__ == "__main__":
    main()
