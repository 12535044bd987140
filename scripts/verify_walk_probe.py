"""Host walk of a streamed round's :217 check (fedavg_collect_ext.verify_rows)
and of the device round's state_dict walk (collect) at the resnet56 x 100
layout, timed at several torch thread counts (the walk splits the clients
over torch's intra-op threads).

    python scripts/verify_walk_probe.py [--threads 1,2,4,8,16] [--reps 30]
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
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np
import torch

import mfl_amd
from mfl_amd.layout import _PACK_KIND, KeyTable, _collect_ext
from model_shapes import CONFIGS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--expect-version", type=int, default=1, help="-1: skip the version-counter check")
    args = ap.parse_args()
    ext = _collect_ext()
    K, shapes = CONFIGS["resnet56"]
    g = torch.Generator().manual_seed(0)
    # every client's own key strings, as each net.cpu().state_dict() builds them (client.py:96)
    dicts = [OrderedDict(("".join(list(k)), torch.tensor(1000 + i, dtype=torch.int64)
                          if k.endswith("num_batches_tracked") else torch.randn(s, generator=g)) for k, s in shapes)
             for i in range(K)]
    assert dicts[1] is not dicts[0] and next(iter(dicts[1])) is not next(iter(dicts[0]))
    table = KeyTable(dicts[0])
    lib = mfl_amd._lib.load()
    stage = {dt: torch.zeros((K, grp.ld), dtype=dt) for dt, grp in table.groups.items()}
    ptrs, _ = table.collect(dicts)
    for dt, grp in table.groups.items():
        items = table.pack_items(grp, ptrs, 0, grp.ld)
        mfl_amd._lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], stage[dt].data_ptr(), 4, 8), "pack")
    w_locals = [(i + 1, copy.deepcopy(d)) for i, d in enumerate(dicts)]
    counts = [i + 1 for i in range(K)]
    gidx = {dt: j for j, dt in enumerate(table.groups)}
    names = [e.name for e in table.entries]
    templ = table.meta_template()
    group = [gidx[e.dtype] for e in table.entries]
    offset = [int(e.offset) for e in table.entries]
    kind = [0 if e.src_dtype == e.dtype else _PACK_KIND[e.src_dtype] for e in table.entries]
    st = [stage[dt] for dt in table.groups]
    sp, sld, ses = [t.data_ptr() for t in st], [int(t.stride(0)) for t in st], [t.element_size() for t in st]
    wdicts = [sd for _, sd in w_locals]
    for nt in [int(t) for t in args.threads.split(",")]:
        torch.set_num_threads(nt)
        tv, tc = [], []
        for r in range(args.reps + 2):
            t0 = time.perf_counter()
            res = ext.verify_rows(w_locals, counts, names, templ, group, offset, kind, sp, sld, ses, 4096, r, 1 << 20,
                                   args.expect_version)
            t1 = time.perf_counter()
            ext.collect(wdicts, names, templ, -1)
            t2 = time.perf_counter()
            tv.append(t1 - t0)
            tc.append(t2 - t1)
            assert res[0] == 0
        print(json.dumps({"threads": nt, "verify_ms_median": round(float(np.median(tv[2:])) * 1e3, 3),
                          "verify_ms_min": round(float(np.min(tv[2:])) * 1e3, 3),
                          "collect_ms_median": round(float(np.median(tc[2:])) * 1e3, 3),
                          "collect_ms_min": round(float(np.min(tc[2:])) * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
