"""Row reduce through buffer descriptors vs the production row reduce.

    python scripts/buf_probe.py [--K 100 --P 25000000] [--rounds 5] [--reps 6]

fedavg_reduce_f32_buf (tuning hook: one descriptor per client row and column
group, base in SGPRs, 32-bit lane offsets) against fedavg_reduce_f32 on the
same [K, ld] rows, interleaved in one process, bit-identity checked.  One JSON
line per variant: median ms per call (HIP events) and GB/s of algorithmic
bytes (4K+4 B per element + weights).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--buf", nargs="*", default=["4,8,0", "4,8,768", "8,4,0", "4,4,0", "2,8,0", "2,16,0", "1,16,0",
                                                 "8,8,0"], help="U,C,max_blocks[,block] of fedavg_reduce_f32_buf (block: 256 default, 128, 64)")
    ap.add_argument("--glob", nargs="*", default=[], help="U,C,max_blocks of the global-pointer variant kernel")
    ap.add_argument("--nt", nargs="*", default=[], help="U,C,max_blocks,nt of the global-pointer variant kernel")
    ap.add_argument("--chunks", type=int, default=1,
                    help="rows hold this many column chunks of P (ld = P x chunks, as a rank's shard at N > 1); "
                         "call i reduces chunk i %% chunks, so the data is not cache-resident between calls")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = mfl_amd._lib.load_probe()
    K, P = args.K, args.P
    C = max(1, args.chunks)
    if C > 1:
        P = (P + 63) // 64 * 64  # chunk starts stay 256-B aligned
    ld = (P * C + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(5)
    rows = torch.randn((K, ld), generator=g, device=dev) * 0.05
    calls = {"i": 0}
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ap_sched = [tuple(int(t) for t in v.split(",")) for v in args.buf]
    variants = {"production": None}
    for sch in ap_sched:
        u, c, b = sch[:3]
        bs = sch[3] if len(sch) > 3 else 256
        variants[f"buf-U{u}C{c}b{b}" + (f"B{bs}" if bs != 256 else "")] = (u, c, b, bs)
    for u, c, b in [tuple(int(t) for t in v.split(",")) for v in args.glob]:
        variants[f"global-U{u}C{c}b{b}"] = ("var", u, c, b)
    for u, c, b, nt in [tuple(int(t) for t in v.split(",")) for v in args.nt]:
        variants[f"global-U{u}C{c}b{b}nt{nt}"] = ("var", u, c, b, nt)
    outs = {n: torch.empty(P, device=dev) for n in variants}

    def run(n, check=False):
        v = variants[n]
        j = 0 if check else calls["i"] % C
        calls["i"] += 1
        x = rows[:, j * P:(j + 1) * P]
        if v is None:
            mfl_amd.reduce_packed(x, w, P, outs[n])
            return
        if v[0] == "var":  # the global-pointer kernel, round-split (pipelined mode 4), nt loads unless given
            mfl_amd.reduce_packed(x, w, P, outs[n], tuned=(v[1], v[4] if len(v) > 4 else 1, v[2], 4, v[3]))
            return
        mfl_amd._lib.check(lib.fedavg_reduce_f32_buf(x.data_ptr(), K, P, ld, w.data_ptr(), outs[n].data_ptr(),
                                                     v[0], v[1], v[3], v[2], stream), n, lib)

    for n in variants:
        run(n, check=True)
    torch.cuda.synchronize()
    same = {n: bool(torch.equal(outs[n].view(torch.int32), outs["production"].view(torch.int32))) for n in outs}
    times = {n: [] for n in variants}
    for _ in range(args.rounds):
        for n in variants:
            for _ in range(args.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run(n)
                e.record()
                times[n].append((s, e))
        torch.cuda.synchronize()
    alg = 4 * K * P + 4 * P + 4 * K
    for n in variants:
        ms = float(np.median([s.elapsed_time(e) for s, e in times[n]]))
        print(json.dumps({"variant": n, "K": K, "P": P, "chunks": C, "ms_median": round(ms, 4),
                          "GBps": round(alg / ms / 1e6, 1),
                          "bit_identical": same[n]}), flush=True)


if __name__ == "__main__":
    main()
