"""Replay the FPF2 golden rounds (tests/golden/fpf, made by oracle/gen_golden_fpf.py).

``replay(case, impl)`` drives an implementation through the reference round
loop's FPF2 call order (fedavg_trainer.py:165 ``last_w`` snapshot, :210 per
client diff row, :217 aggregate, :219 ``load_state_dict``, :272 index,
:314-327 end-of-round updates) and returns the per-round FPF2 rows, to be
compared with the reference's own CSV rows (``case.fpf``).
"""
from __future__ import annotations

import copy
import hashlib
import json
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional

import numpy as np
import torch

FPF_DIR = Path(__file__).resolve().parent / "golden" / "fpf"


@dataclass
class FPFCase:
    meta: dict
    init: "OrderedDict[str, torch.Tensor]"
    client_states: Optional[List[List["OrderedDict[str, torch.Tensor]"]]]  # [round][j]; None: regenerated
    fpf: np.ndarray  # [rounds, client_num_in_total], the reference's CSV values
    stats: Optional[np.ndarray] = None  # [rounds, (rho, beta, delta)] after each round's :289-305 update

    def client_state(self, t: int, j: int, model_state) -> "OrderedDict[str, torch.Tensor]":
        """Client ``j``'s returned state in round ``t``: the stored one, or --
        for a scenario stored as digests (``meta["inputs"] == "sha256"``) --
        rebuilt from ``model_state`` (the model the round's clients start
        from) by the generator's stub ``Client.train`` recipe
        (oracle/gen_golden_fpf.py) and checked against the reference input's
        sha256."""
        if self.client_states is not None:
            return self.client_states[t][j]
        rd = self.meta["rounds"][t]
        ds = rd["client_indexes"][j]
        g = torch.Generator().manual_seed(1000 * t + ds)
        w = OrderedDict()
        for k, v in model_state.items():
            v = v.detach().cpu()
            if v.dtype == torch.int64:
                w[k] = v + rd["local_itr"]
            else:
                w[k] = v + (0.01 * (1 + ds) * torch.randn(v.shape, generator=g)).to(v.dtype)
        want = self.meta["client_sha256"][f"r{t}_i{j}"]
        assert _digest(w) == want, f"regenerated client r{t} i{j} differs from the reference's input"
        return w


def _digest(sd) -> str:
    h = hashlib.sha256()
    for v in sd.values():
        h.update(v.numpy().tobytes())
    return h.hexdigest()


# the digest-only scenarios' models (the generator's make_model): P = 1,001,000 and 25,005,000
_DIGEST_MODELS = {"big": (1000, 1000), "target": (5000, 5000)}


def big_init(kind: str = "big") -> "OrderedDict[str, torch.Tensor]":
    """A digest-only scenario's initial model: the generator's ``make_model(kind)``."""
    torch.manual_seed(1234)
    return OrderedDict((k, v.detach().clone()) for k, v in torch.nn.Linear(*_DIGEST_MODELS[kind]).state_dict().items())


def case_names(stats_only: bool = False, max_p: Optional[int] = None):
    """Scenario names; ``stats_only=False`` leaves out the regenerated
    (digest-only) scenarios, whose replay costs seconds per round;
    ``max_p`` leaves out scenarios with more parameters."""
    names = sorted(p.stem for p in FPF_DIR.glob("*.npz"))
    if not stats_only:
        names = [n for n in names if not n.startswith(("big", "target"))]
    if max_p is not None:
        names = [n for n in names if _weight_size(n) <= max_p]
    return names


def _weight_size(name: str) -> int:
    z = np.load(FPF_DIR / f"{name}.npz", allow_pickle=False)
    return int(json.loads(bytes(z["meta"]).decode())["weight_size"])


def load_case(name: str) -> FPFCase:
    z = np.load(FPF_DIR / f"{name}.npz", allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    stats = z["stats"] if "stats" in z.files else None
    if meta.get("inputs") == "sha256":
        init = big_init(meta["model"])
        assert _digest(init) == meta["init_sha256"], "the regenerated initial model differs from the reference's"
        return FPFCase(meta, init, None, z["fpf"], stats)
    keys = [k["name"] for k in meta["keys"]]
    bf16 = {k["name"] for k in meta["keys"] if k["dtype"] == "bfloat16"}  # stored as int16 bits

    def tensor(arr, k):
        t = torch.from_numpy(arr.copy())
        return t.view(torch.bfloat16) if k in bf16 else t

    init = OrderedDict((k, tensor(z[f"init__{k}"], k)) for k in keys)
    states = []
    for t, rd in enumerate(meta["rounds"]):
        states.append([OrderedDict((k, tensor(z[f"w__r{t}__i{j}__{k}"], k)) for k in keys)
                       for j in range(len(rd["client_indexes"]))])
    return FPFCase(meta, init, states, z["fpf"], stats)


def replay(case: FPFCase, impl, record_after_aggregate: bool = False) -> np.ndarray:
    """``impl`` provides begin_round(last_w), record_client(idx, w, last_w),
    record_round(idx_list, w_locals, w_glob) (used when
    ``record_after_aggregate``), aggregate(w_locals, model_state),
    fpf_index() and end_round(t, idx_list, local_itr, w_glob, last_w)."""
    model_state = OrderedDict((k, v.clone()) for k, v in case.init.items())
    rows = []
    for t, rd in enumerate(case.meta["rounds"]):
        idx, itr = rd["client_indexes"], rd["local_itr"]
        last_w = copy.deepcopy(model_state)  # :165
        impl.begin_round(last_w)
        w_locals = [(n, copy.deepcopy(case.client_state(t, j, model_state))) for j, n in enumerate(rd["sample_nums"])]
        if not record_after_aggregate:
            for c, (_, w) in zip(idx, w_locals):
                impl.record_client(c, w, last_w)  # :210, before aggregate aliases w_locals[0][1]
        w_glob = impl.aggregate(w_locals, model_state)  # :217
        if record_after_aggregate:
            impl.record_round(idx, w_locals, w_glob)
        for k in model_state:  # :219 load_state_dict (copy_ casts into the buffer's dtype)
            model_state[k].copy_(w_glob[k])
        # :272-278, in the index's own dtype: fp32, or fp64 once A_mat has
        # become fp64 (a model with an fp64 key, torch.cat's promotion at :319)
        rows.append(np.asarray(impl.fpf_index()))
        impl.end_round(t, idx, itr, w_glob, last_w)  # :314-327
    return np.stack(rows)


def replay_stats(case: FPFCase, aggregate, norms):
    """Drive the rounds through the loop's :217 aggregate and the :289-305
    statistics.  ``aggregate(w_locals, model_state)`` -> ``w_glob``;
    ``norms(w_locals, w_glob)`` -> the round's :291 distances.  Returns
    ``(stats, norms_per_round)``: ``stats`` [rounds, (rho, beta, delta)] after
    each round's update, comparable with ``case.stats`` (the reference's)."""
    import fedavg_oracle as O

    rho0, beta0, delta0 = case.meta["stats_init"]
    st = (delta0, rho0, beta0, True, True)  # :107
    lr = case.meta["lr"]
    model_state = OrderedDict((k, v.clone()) for k, v in case.init.items())
    out, all_norms = [], []
    for t, rd in enumerate(case.meta["rounds"]):
        w_locals = [(n, copy.deepcopy(case.client_state(t, j, model_state))) for j, n in enumerate(rd["sample_nums"])]
        w_glob = aggregate(w_locals, model_state)  # :217
        for k in model_state:  # :219
            model_state[k].copy_(w_glob[k])
        nrm = np.asarray(norms(w_locals, w_glob)) if w_locals else np.zeros(0)  # :291
        all_norms.append(nrm)
        st = O.round_stats_update(st, rd["sample_nums"], nrm, rd["rhos"], rd["betas"], lr,
                                  have_losses=bool(rd["losses"]))
        out.append((st[1], st[2], st[0]))
    return np.array(out, dtype=np.float64), all_norms
