"""Zero-edit streaming at scale: mfl_amd.install alone on the loop-replay
harness (tests/loop_replay.py: fedavg_trainer.py:172-219's order), K clients
x P fp32 parameters, host state_dicts.

    python scripts/stream_install_probe.py [--K 100 --P 25000000] [--rounds 4] [--delay-ms 20]

Per round, two times: ``aggregate_ms`` = the :217 call alone (the last
client has been trained, validated and deep-copied by the loop; what the
drop-in adds to the round after it), and ``last_train_to_model_ms`` = from the
last client's train() return to the model (includes the loop's own
deepcopy at :199).  Both legs (streaming on / plain drop-in) on the same
clients in one process; results compared bit for bit.  ``--delay-ms``: the
simulated training time of each client (client.py:58-90).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from collections import OrderedDict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "tests")):
    sys.path.insert(0, p)

import numpy as np
import torch

import mfl_amd
from loop_replay import fresh_classes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--delay-ms", type=float, default=20.0)
    ap.add_argument("--keys", type=int, default=1, help="split P over this many keys")
    ap.add_argument("--shards", default="1",
                    help="streaming legs over N column shards (install(devices=[0]*N): every shard on cuda:0 "
                         "here, one PCIe link -- a rehearsal of the N-GPU finish, not its link rates)")
    ap.add_argument("--no-plain", action="store_true", help="skip the plain (streaming off) leg")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, P = args.K, args.P
    t0 = time.perf_counter()
    base = torch.randn(P) * 0.05
    sizes = [P // args.keys] * args.keys
    sizes[-1] += P - sum(sizes)
    clients = []
    for i in range(K):
        flat = base + (i * 1e-3 - 0.05)
        sd, off = OrderedDict(), 0
        for j, n in enumerate(sizes):
            sd[f"layer{j}.weight"] = flat[off:off + n].clone()
            off += n
        clients.append(sd)
    counts = [int(c) for c in np.random.default_rng(1234).integers(1, 1000, size=K)]
    rounds = [[(counts[(i + r) % K], [clients[i]]) for i in range(K)] for r in range(args.rounds)]
    print(json.dumps({"setup_s": round(time.perf_counter() - t0, 1)}), flush=True)
    legs = {}
    leg_list = [(f"streaming_shards{n}" if n > 1 else "streaming", True, n)
                for n in (int(x) for x in args.shards.split(","))]
    if not args.no_plain:
        leg_list.append(("plain", False, 1))
    for leg, stream, n_sh in leg_list:
        T, C = fresh_classes()
        mfl_amd.install(T, device=dev, client_cls=C, stream_clients=stream,
                        devices=[0] * n_sh if n_sh > 1 else None)
        round_stats = []

        tr = T(OrderedDict((k, torch.zeros_like(v)) for k, v in clients[0].items()), rounds,
               train_delay_s=args.delay_ms / 1e3)
        orig_agg = T.aggregate

        def agg_and_snap(self, w_locals, _orig=orig_agg, _rs=round_stats):
            out = _orig(self, w_locals)
            f = self.__dict__.get("_mfl_feed")
            _rs.append(dict(f.stats["last_round"], verify=dict(f.stats.get("last_verify", {})))
                       if f is not None else None)
            return out

        T.aggregate = agg_and_snap
        tr.train()
        legs[leg] = tr
        feed = tr.__dict__.get("_mfl_feed")
        for r, tm in enumerate(tr.timings):
            if feed is not None and r < len(round_stats):
                tm = dict(tm, feed=round_stats[r])
            print(json.dumps({"leg": leg, "shards": n_sh, "K": K, "P": P, "keys": args.keys, "round": r,
                              "aggregate_ms": round(tm["aggregate_ms"], 3),
                              "last_train_to_model_ms": round(tm["last_train_to_model_ms"], 3),
                              "delay_ms": args.delay_ms, "feed": tm.get("feed")}), flush=True)
        if feed is not None:
            print(json.dumps({"leg": leg, "feed_stats": feed.stats}), flush=True)
    names = list(legs)
    same = all(torch.equal(a[k].view(-1).view(torch.int32), b[k].view(-1).view(torch.int32))
               for other in names[1:] for a, b in zip(legs[names[0]].results, legs[other].results) for k in a)
    agg = {leg: float(np.median([t["aggregate_ms"] for t in tr.timings[1:]])) for leg, tr in legs.items()}
    print(json.dumps({"summary": True, "K": K, "P": P, "bit_identical": same,
                      "median_aggregate_ms_after_round0": agg}), flush=True)


if __name__ == "__main__":
    main()
