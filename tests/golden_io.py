"""Load the golden vectors in tests/golden (made by oracle/gen_golden.py).

Each case is returned as (meta, w_locals, expected) where ``w_locals`` is a
list of (sample_num, OrderedDict[str, torch.Tensor]) exactly as the reference
``aggregate`` saw it, and ``expected`` maps key -> torch.Tensor result.
"""
from __future__ import annotations

import json
from collections import OrderedDict
from pathlib import Path

import numpy as np
import torch

GOLDEN_DIR = Path(__file__).resolve().parent / "golden"

_DT = {
    "float32": torch.float32,
    "float64": torch.float64,
    "float16": torch.float16,
    "bfloat16": torch.bfloat16,
    "int64": torch.int64,
    "int32": torch.int32,
    "uint8": torch.uint8,
    "bool": torch.bool,
}


def case_names():
    return sorted(p.stem for p in GOLDEN_DIR.glob("*.npz"))


def _tensor(arr: np.ndarray, dtype: str) -> torch.Tensor:
    t = torch.from_numpy(np.array(arr, copy=True))
    if dtype == "bfloat16":
        return t.view(torch.bfloat16)
    assert t.dtype == _DT[dtype], (t.dtype, dtype)
    return t


def _sample_num(v, tname):
    return float(v) if tname == "float" else int(v)


def load_case(name: str):
    z = np.load(GOLDEN_DIR / f"{name}.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    w_locals = []
    for i in range(meta["K"]):
        sd = OrderedDict()
        for k in meta["in_keys"]:
            sd[k["name"]] = _tensor(z[f"in__{i}__{k['name']}"], k["dtype"])
        w_locals.append((_sample_num(meta["sample_nums"][i], meta["sample_num_types"][i]), sd))
    expected = OrderedDict()
    for k in meta["out_keys"]:
        expected[k["name"]] = _tensor(z[f"out__{k['name']}"], k["dtype"])
    return meta, w_locals, expected


def bits_equal(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Bit-exact tensor equality (dtype, shape and every bit, NaN payloads included)."""
    if a.dtype != b.dtype or tuple(a.shape) != tuple(b.shape):
        return False
    a = a.detach().cpu().contiguous().reshape(-1)
    b = b.detach().cpu().contiguous().reshape(-1)
    if a.dtype == torch.bool:
        return torch.equal(a, b)
    return bytes(a.view(torch.uint8).numpy()) == bytes(b.view(torch.uint8).numpy())
