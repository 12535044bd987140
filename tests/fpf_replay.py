"""Replay the FPF2 golden rounds (tests/golden/fpf, made by oracle/gen_golden_fpf.py).

``replay(case, impl)`` drives an implementation through the reference round
loop's FPF2 call order (fedavg_trainer.py:165 ``last_w`` snapshot, :210 per
client diff row, :217 aggregate, :219 ``load_state_dict``, :272 index,
:314-327 end-of-round updates) and returns the per-round FPF2 rows, to be
compared with the reference's own CSV rows (``case.fpf``).
"""
from __future__ import annotations

import copy
import json
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import List

import numpy as np
import torch

FPF_DIR = Path(__file__).resolve().parent / "golden" / "fpf"


@dataclass
class FPFCase:
    meta: dict
    init: "OrderedDict[str, torch.Tensor]"
    client_states: List[List["OrderedDict[str, torch.Tensor]"]]  # [round][j]
    fpf: np.ndarray  # [rounds, client_num_in_total], the reference's CSV values


def case_names():
    return sorted(p.stem for p in FPF_DIR.glob("*.npz"))


def load_case(name: str) -> FPFCase:
    z = np.load(FPF_DIR / f"{name}.npz", allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
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
    return FPFCase(meta, init, states, z["fpf"])


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
        w_locals = [(n, copy.deepcopy(sd)) for n, sd in zip(rd["sample_nums"], case.client_states[t])]
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
