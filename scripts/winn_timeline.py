"""Per-wave timeline of the split-row window kernel (probe MODE 8).

    python scripts/winn_timeline.py [--shapes 1000x12500000 500x11227812] [--codes 88800008 88800016]

Lane 0 of every wave of the first 8 workgroups stores s_memtime (shader
clock) at five points of each of its first 48 windows
(reduce_sqdist_winn_kernel, fedavg_dist.hip):
  0 top       window loop entry
  1 arrived   after the wait for the wave's own rows of this window (PF > 0)
  2 turn      the wave's chain turn starts (after the hand-off barrier)
  3 handed    its partial is written to LDS for the next wave
  4 squared   its squares done and the next window's reloads issued
  5 released  past the end-of-window barrier
One JSON line per (shape, code): cycle budget per window (median over the
steady-state windows 4..47 of the 8 workgroups) and the kernel time.
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

MAGIC = 0x504D415453
BLOCKS, WINS, SLOTS = 8, 48, 8


def stamps_of(wv, K, G, nsmax, ns):
    """The stamp block after the K x G partials: [blocks, waves, windows, slots]."""
    st = wv[K * G + 1:K * G + 1 + BLOCKS * nsmax * WINS * SLOTS].reshape(BLOCKS, nsmax, WINS, SLOTS)
    return st[:, :ns].astype(np.float64)


def summarize(st, ns, wins):
    """Median cycles per window over the steady-state windows 4..wins-2."""
    sl = slice(4, wins - 1)
    top, arr, turn, hand, sq, rel = (st[..., i] for i in range(6))
    have = {n: bool((st[:, :, sl, i] != 0).all()) for i, n in enumerate(("top", "arr", "turn", "hand", "sq", "rel"))}
    med = lambda a: round(float(np.median(a)), 1)
    cyc = {"window_period": med((top[:, 0, 1:wins] - top[:, 0, :wins - 1])[:, 3:]),
           "chain": med(hand[:, ns - 1, sl] - turn[:, 0, sl]), "turn": med((hand - turn)[:, :, sl]),
           "squares_after_chain_mean": med((sq[:, :, sl] - hand[:, ns - 1, sl][:, None, :]).mean(axis=1)),
           "squares_after_chain_max": med((sq[:, :, sl] - hand[:, ns - 1, sl][:, None, :]).max(axis=1)),
           "top_to_turn_wave0": med(turn[:, 0, sl] - top[:, 0, sl]),
           # the chain's start against the block's previous window: how far it overlaps the reloads
           "turn0_after_last_squares_prev": med(turn[:, 0, 5:wins] - sq[:, :, 4:wins - 1].max(axis=1)),
           "turn0_after_first_squares_prev": med(turn[:, 0, 5:wins] - sq[:, :, 4:wins - 1].min(axis=1))}
    if ns > 1:
        cyc["handoff"] = med(turn[:, 1:, sl] - hand[:, :-1, sl])
    if have["arr"]:
        wait_rows = (arr - top)[:, :, sl]
        cyc.update(wait_own_rows=med(wait_rows), wait_own_rows_wave0=med(wait_rows[:, 0]),
                   wait_own_rows_last_wave=med(wait_rows[:, ns - 1]),
                   last_arrival_to_turn0=med(turn[:, 0, sl] - arr[:, :, sl].max(axis=1)))
    if have["rel"]:
        cyc.update(end_barrier=med(rel[:, :, sl] - sq[:, :, sl].max(axis=1)[:, None, :]),
                   release_to_next_top=med(top[:, :, 5:wins] - rel[:, :, 4:wins - 1]))
    return cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=["1000x12500000", "500x11227812"])
    ap.add_argument("--codes", nargs="*", type=int, default=[88800008])
    ap.add_argument("--nsmax", type=int, default=16)
    ap.add_argument("--out", default=None, help="npz of the raw stamps")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    probe = mfl_amd._lib.load_probe()
    raw = {}
    for shape in args.shapes:
        K, P = (int(v) for v in shape.split("x"))
        ld = (P + 63) // 64 * 64
        g = torch.Generator(device=dev).manual_seed(K + P)
        x = torch.randn((K, ld), generator=g, device=dev) * 0.05
        w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, dev)
        ns = (K + 63) // 64
        n_ws = K * 4096 + 1 + BLOCKS * args.nsmax * WINS * SLOTS
        work = torch.zeros(n_ws, dtype=torch.float64, device=dev)
        o = torch.empty(P, device=dev)
        s = torch.empty(K, dtype=torch.float64, device=dev)
        for code in args.codes:
            def run():
                mfl_amd._lib.check(probe.fedavg_reduce_sqdist_f32_variant(
                    x.data_ptr(), K, P, ld, w.data_ptr(), o.data_ptr(), work.data_ptr(), n_ws, s.data_ptr(), code, 0,
                    torch.cuda.current_stream(dev).cuda_stream), str(code), probe)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            ms = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run()
                b.record()
                b.synchronize()
                ms.append(a.elapsed_time(b))
            wv = work.view(torch.int64).cpu().numpy()
            G = next((g_ for g_ in range(1, 4097) if wv[K * g_] == MAGIC), None)
            if G is None:
                print(json.dumps({"K": K, "P": P, "code": code, "error": "no stamp header"}), flush=True)
                continue
            st = stamps_of(wv, K, G, args.nsmax, ns)
            raw[f"{K}x{P}_{code}"] = st
            rec = {"K": K, "P": P, "code": code, "grid": G, "windows_per_block": round(((P + 63) // 64) / G, 1),
                   "ms_median": round(float(np.median(ms)), 4),
                   "cycles_median": summarize(st, ns, min(WINS, ((P + 63) // 64) // G))}
            print(json.dumps(rec), flush=True)
        del x, work
        torch.cuda.empty_cache()
    if args.out:
        np.savez_compressed(args.out, **raw)


if __name__ == "__main__":
    main()
