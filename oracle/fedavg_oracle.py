"""CPU oracle for the FedAvg server-side weighted reduction.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it, and only as the checker (or, for ``bench.py``, as
the timed CPU baseline).  The product path (``mobile-federated-learning_amd``)
never imports this module and fails loudly when its HIP library is missing.

What it restates
----------------
``FedAvgTrainer.aggregate`` in the reference,
``/root/reference/src/fedavg_trainer.py:441-458``:

* ``:442-443`` empty ``w_locals`` -> a deep copy of the global model's CPU
  state_dict (``empty_result``).
* ``:444-447`` ``training_num = sum(n_i)`` as a Python number
  (``sample_weights``).
* ``:449`` ``averaged_params`` *is* ``w_locals[0][1]`` (aliased, mutated).
* ``:450-457`` for every key of client 0, for ``i = 0..K-1`` in order:
  ``w = n_i / training_num`` (Python double, ``:453``), then
  ``i == 0: acc = p_0[k] * w`` (``:455``) else ``acc += p_i[k] * w`` (``:457``).
  For an fp32 tensor ATen rounds ``w`` to fp32 once and computes
  ``fl32(acc + fl32(p * fl32(w)))`` -- a multiply and an add, never fused.
  Integer/bool tensors are promoted to fp32 (the default dtype) before the
  multiply; fp64 tensors stay fp64 (``w`` kept as a double).

Parity pin
----------
The restatement is pinned bit-for-bit against golden vectors produced by
importing the reference ``aggregate`` itself in the build container
(``oracle/gen_golden.py`` -> ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.  The reference has no tests or fixtures of
its own, so those captured vectors are the pin.
"""
from __future__ import annotations

import copy
from collections import OrderedDict
from typing import Iterable, List, Sequence, Tuple

import numpy as np

__all__ = [
    "sample_weights",
    "reduce_f32",
    "reduce_f64",
    "reduce_half",
    "f32_to_bf16_bits",
    "bf16_bits_to_f32",
    "aggregate_torch",
    "aggregate_numpy",
    "empty_result",
    "client_distances_torch",
    "client_distances_exact",
    "delta_from_norms",
]


def sample_weights(sample_nums: Sequence) -> List[float]:
    """``w_i = n_i / sum(n)`` with Python semantics (fedavg_trainer.py:444-447, :453).

    Returns Python doubles exactly as the reference forms them; raises
    ``ZeroDivisionError`` when the sum is zero, as the reference does.
    """
    training_num = 0
    for n in sample_nums:
        training_num += n
    return [n / training_num for n in sample_nums]


def reduce_f32(clients: np.ndarray, weights: Sequence[float]) -> np.ndarray:
    """Sequential fp32 weighted sum over the client axis of ``clients[K, P]``.

    ``acc = x_0 * f32(w_0)``; ``acc = acc + x_i * f32(w_i)`` for i = 1..K-1
    (fedavg_trainer.py:451-457), each numpy op rounding to fp32, no fusion.
    """
    x = np.ascontiguousarray(clients, dtype=np.float32)
    if x.ndim != 2 or x.shape[0] == 0:
        raise ValueError("clients must be [K>0, P]")
    w32 = np.asarray(weights, dtype=np.float64).astype(np.float32)
    acc = x[0] * w32[0]
    for i in range(1, x.shape[0]):
        acc = acc + x[i] * w32[i]
    return acc.astype(np.float32, copy=False)


def reduce_f64(clients: np.ndarray, weights: Sequence[float]) -> np.ndarray:
    """fp64 variant: the weight stays a double (ATen opmath for double)."""
    x = np.ascontiguousarray(clients, dtype=np.float64)
    w64 = np.asarray(weights, dtype=np.float64)
    acc = x[0] * w64[0]
    for i in range(1, x.shape[0]):
        acc = acc + x[i] * w64[i]
    return acc


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 bit pattern, round-to-nearest-even, NaN -> 0x7FC0 (c10::BFloat16)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return np.where(np.isnan(x), np.uint16(0x7FC0), r).astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b).astype(np.uint16).astype(np.uint32) << 16).view(np.float32)


def reduce_half(clients: np.ndarray, weights: Sequence[float], kind: str) -> np.ndarray:
    """fp16 / bf16 keys keep their dtype (``tensor * float`` does not promote).

    ATen computes each op in fp32 (opmath) and rounds to the storage type:
    ``term = rh(f32(x) * f32(w))``, ``acc = rh(f32(acc) + f32(term))``.
    ``clients`` holds fp16 values (kind "float16") or bf16 bit patterns as
    uint16/int16 (kind "bfloat16"); the result uses the same representation.
    """
    if kind == "float16":
        to32 = lambda a: np.asarray(a, dtype=np.float16).astype(np.float32)
        toh = lambda a: a.astype(np.float16)
    elif kind == "bfloat16":
        to32 = bf16_bits_to_f32
        toh = f32_to_bf16_bits
    else:
        raise ValueError(kind)
    w32 = np.asarray(weights, dtype=np.float64).astype(np.float32)
    acc = toh(to32(clients[0]) * w32[0])
    for i in range(1, len(clients)):
        term = toh(to32(clients[i]) * w32[i])
        acc = toh(to32(acc) + to32(term))
    return acc


def aggregate_torch(w_locals):
    """The reference's torch CPU loop, restated (fedavg_trainer.py:444-458).

    Same operators in the same order on the same objects, so it is also the
    CPU baseline that ``bench.py`` times (``cpu_baseline.kind == "port"``).
    Mutates and returns ``w_locals[0][1]`` like the reference.
    """
    weights = sample_weights([n for n, _ in w_locals])
    acc_dict = w_locals[0][1]
    for key in list(acc_dict.keys()):
        for i, (_, params) in enumerate(w_locals):
            term = params[key] * weights[i]
            if i == 0:
                acc_dict[key] = term
            else:
                acc_dict[key] += term
    return acc_dict


def _half_kind(key, arr, bf16_keys):
    if key in bf16_keys:
        return "bfloat16"
    if arr.dtype == np.float16:
        return "float16"
    return None


def aggregate_numpy(w_locals, bf16_keys: Iterable[str] = ()) -> "OrderedDict[str, np.ndarray]":
    """Numpy restatement over state_dicts of numpy arrays (no aliasing).

    Per key: fp32 path for fp32/integer/bool arrays, fp64 path for fp64,
    half path for fp16 and for the keys named in ``bf16_keys`` (numpy has no
    bf16; those arrays carry bf16 bit patterns).
    """
    bf16_keys = set(bf16_keys)
    weights = sample_weights([n for n, _ in w_locals])
    out = OrderedDict()
    for key in w_locals[0][1].keys():
        arrs = [np.asarray(sd[key]) for _, sd in w_locals]
        shape = arrs[0].shape
        for a in arrs:
            if a.shape != shape:
                raise ValueError(f"shape mismatch for key {key!r}")
        if kind_hint := _half_kind(key, arrs[0], bf16_keys):
            flat = np.stack([a.reshape(-1) for a in arrs])
            out[key] = reduce_half(flat, weights, kind_hint).reshape(shape)
        elif arrs[0].dtype == np.float64:
            flat = np.stack([a.reshape(-1).astype(np.float64) for a in arrs])
            out[key] = reduce_f64(flat, weights).reshape(shape)
        elif arrs[0].dtype == np.float32 or arrs[0].dtype.kind in "iub":
            flat = np.stack([a.reshape(-1).astype(np.float32) for a in arrs])
            out[key] = reduce_f32(flat, weights).reshape(shape)
        else:
            raise TypeError(f"oracle has no rule for dtype {arrs[0].dtype}")
    return out


def empty_result(model_global):
    """fedavg_trainer.py:442-443: deep copy of the global model's CPU state."""
    return copy.deepcopy(model_global.cpu().state_dict())


def client_distances_torch(w_locals, w_glob, keys=None):
    """fedavg_trainer.py:291 restated: torch.norm(torch.cat([w[k] - w_glob[k]])).item().

    Uses ATen's CPU fp32 norm, which accumulates in fp32 SIMD lanes, so the
    value depends on the host's vector width; it approximates the exact norm
    to within its own rounding error.
    """
    import torch

    keys = list(w_glob.keys()) if keys is None else list(keys)
    return np.array([torch.norm(torch.cat([w[k].reshape((-1,)) - w_glob[k].reshape((-1,)) for k in keys])).item()
                     for _, w in w_locals])


def client_distances_exact(w_locals, w_glob, keys=None):
    """Accurate form of :291: the differences rounded exactly as the
    reference forms them (``w[k] - w_glob[k]`` in each key's promoted dtype:
    fp32, fp64, or fp32 opmath rounded to fp16/bf16), widened exactly by
    torch.cat, squares and sum in fp64, the root rounded to torch.cat's dtype
    (what ``torch.norm(...).item()`` returns, without its accumulation error)."""
    import torch

    keys = list(w_glob.keys()) if keys is None else list(keys)
    out = []
    for _, w in w_locals:
        d = torch.cat([w[k].reshape((-1,)) - w_glob[k].reshape((-1,)) for k in keys])
        s = np.sqrt(np.sum(np.square(d.double().numpy())))
        out.append(float(torch.tensor(s, dtype=torch.float64).to(d.dtype).double()))
    return np.array(out)


def delta_from_norms(sample_nums, norms, lr):
    """fedavg_trainer.py:293."""
    sample_nums = np.asarray(sample_nums)
    return np.sum(sample_nums * np.asarray(norms)) / np.sum(sample_nums) / lr


THRESHOLD_RHO = 1000  # config.py:85
THRESHOLD_BETA = 1000  # config.py:86


def round_stats_update(stats, sample_nums, norms, rho_locals, beta_locals, lr, have_losses=True):
    """fedavg_trainer.py:289-305: the loop's scheduler statistics after a round.

    ``stats`` = ``(delta, rho, beta, rho_flag, beta_flag)`` as they stood
    (:107 draws the first three, both flags True); ``norms`` = the round's
    :291 distances (one per ``w_locals`` entry).  Returns the updated tuple:
    ``delta`` replaced by :293 when finite; ``rho`` / ``beta`` by their
    sample-weighted means when larger (or on the first update) and finite
    and below THRESHOLD_RHO / THRESHOLD_BETA, which also clears the flag.
    Nothing changes for an empty round (:289)."""
    delta, rho, beta, rho_flag, beta_flag = stats
    if not (len(sample_nums) and have_losses):
        return stats
    sample_nums = np.array(sample_nums)
    delta_tmp = np.sum(sample_nums * np.asarray(norms)) / np.sum(sample_nums) / lr
    if not np.isnan(delta_tmp) and not np.isinf(delta_tmp):
        delta = delta_tmp
    rho_tmp = np.sum(sample_nums * np.array(rho_locals)) / np.sum(sample_nums)
    if rho_tmp > rho or rho_flag:
        if (not np.isnan(rho_tmp) and not np.isinf(rho_tmp)) and rho_tmp < THRESHOLD_RHO:
            rho, rho_flag = rho_tmp, False
    beta_tmp = np.sum(sample_nums * np.array(beta_locals)) / np.sum(sample_nums)
    if beta_tmp > beta or beta_flag:
        if (not np.isnan(beta_tmp) and not np.isinf(beta_tmp)) and beta_tmp < THRESHOLD_BETA:
            beta, beta_flag = beta_tmp, False
    return delta, rho, beta, rho_flag, beta_flag
