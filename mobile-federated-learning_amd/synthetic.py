"""Synthetic K-client x P-param inputs of the BASELINE measurement, generated
on the device and reproducible bit for bit in numpy.

BASELINE.md's inputs are ``base ~ N(0, 0.05^2)`` and client k =
``base + N(0, 1e-3^2)``.  Above a few GB they have to be generated on the GPU
("generate on device with a counter-based hash RNG
reproduced in numpy"), and at N > 1 every rank generates only its own
columns.  Here every value is a pure function of (client k, GLOBAL column g):

    u(s, g)  = uniform in (-1, 1) from the top 24 bits of mix64(g * A + s * B)
    base[g]  = fl32(fl32(u(0, g)) * (0.05 * sqrt 3))
    x[k][g]  = fl32(base[g] + fl32(u(1 + k, g) * (1e-3 * sqrt 3)))

(uniform with the BASELINE variances).  So

* the global model does not depend on how the columns are sharded (1, 2, 4
  or 8 ranks, any chunking), and
* any window of any rank's columns can be regenerated on the host with
  numpy, from nothing but (k, g), and reduced by the oracle -- the parity
  check of the gathered model at N > 1 needs no copy of another rank's
  device buffers.

``mix64`` is the splitmix64 finaliser over wrapping int64 arithmetic (torch's
and numpy's int64 ops both wrap; right shifts are masked to be logical), and
every float step is one IEEE fp32 multiply or add, so the torch (any device)
and numpy forms give identical bits (tests/test_host_logic.py pins it).
This module is measurement input, not product code: the aggregate never
calls it.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

__all__ = ["client_columns_torch", "client_columns_numpy", "fill_rows", "sample_counts", "BASE_SCALE", "NOISE_SCALE"]

_A = 0x9E3779B97F4A7C15 - (1 << 64)  # golden-ratio increment, as a signed int64
_B = 0x632BE59BD9B4E019 - (1 << 64)
_M1 = 0xBF58476D1CE4E5B9 - (1 << 64)
_M2 = 0x94D049BB133111EB - (1 << 64)
_LOW = {s: (1 << (64 - s)) - 1 for s in (27, 30, 31)}  # masks that make >> logical
_TWO24 = float(1 << 24)
BASE_SCALE = np.float32(0.05 * 3 ** 0.5)  # uniform(-1, 1) * s has std s / sqrt 3
NOISE_SCALE = np.float32(1e-3 * 3 ** 0.5)


def sample_counts(K: int) -> list:
    """n_k ~ U{1..1000} from numpy.random.default_rng(1234)."""
    return [int(v) for v in np.random.default_rng(1234).integers(1, 1001, size=K)]


# ---------------------------------------------------------------- torch form
def _mix_t(x: torch.Tensor) -> torch.Tensor:
    # logical right shifts: arithmetic shift, then mask off the sign copies
    x = x ^ ((x >> 30) & _LOW[30])
    x = x * _M1
    x = x ^ ((x >> 27) & _LOW[27])
    x = x * _M2
    return x ^ ((x >> 31) & _LOW[31])


def _wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= 1 << 63 else v


def _uniform_t(seed: int, g: torch.Tensor) -> torch.Tensor:
    h = _mix_t(g * _A + _wrap64(seed * _B))
    v = ((h >> 40) & 0xFFFFFF).to(torch.float32)  # exact: < 2^24
    return (v * 2.0 + (1.0 - _TWO24)) / _TWO24  # (2v + 1 - 2^24) / 2^24, every step exact in fp32


def _base_t(g: torch.Tensor) -> torch.Tensor:
    return _uniform_t(0, g) * float(BASE_SCALE)


def client_columns_torch(k: int, g: torch.Tensor, base: torch.Tensor = None) -> torch.Tensor:
    """x[k][g] for an int64 tensor of global columns (any device)."""
    if base is None:
        base = _base_t(g)
    return base + _uniform_t(1 + k, g) * float(NOISE_SCALE)


def fill_rows(rows: torch.Tensor, segments: Sequence, K: int = None) -> None:
    """Fill a device ``[K, cols]`` row buffer: for every ``(local_start,
    global_start, n)`` segment, ``rows[k, l:l+n] = x[k][g:g+n]``.  Columns
    no segment covers are zeroed (plan padding).  Works in column pieces so
    the int64 temporaries stay small."""
    K = rows.shape[0] if K is None else K
    rows.zero_()
    piece = 1 << 24
    for lstart, gstart, n in segments:
        for off in range(0, n, piece):
            m = min(piece, n - off)
            g = torch.arange(gstart + off, gstart + off + m, dtype=torch.int64, device=rows.device)
            base = _base_t(g)
            for k in range(K):
                rows[k, lstart + off:lstart + off + m] = client_columns_torch(k, g, base)
            del g, base


# ---------------------------------------------------------------- numpy form
def _mix_n(x: np.ndarray) -> np.ndarray:
    x = x ^ ((x >> np.int64(30)) & np.int64(_LOW[30]))
    x = x * np.int64(_M1)
    x = x ^ ((x >> np.int64(27)) & np.int64(_LOW[27]))
    x = x * np.int64(_M2)
    return x ^ ((x >> np.int64(31)) & np.int64(_LOW[31]))


def _uniform_n(seed: int, g: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = _mix_n(g * np.int64(_A) + np.int64(_wrap64(seed * _B)))
    v = ((h >> np.int64(40)) & np.int64(0xFFFFFF)).astype(np.float32)
    return (v * np.float32(2.0) + np.float32(1.0 - _TWO24)) / np.float32(_TWO24)


def client_columns_numpy(K: int, g0: int, n: int) -> np.ndarray:
    """``[K, n]`` fp32 host copy of clients 0..K-1 at global columns g0..g0+n-1."""
    g = np.arange(g0, g0 + n, dtype=np.int64)
    base = _uniform_n(0, g) * BASE_SCALE
    out = np.empty((K, n), dtype=np.float32)
    for k in range(K):
        out[k] = base + _uniform_n(1 + k, g) * NOISE_SCALE
    return out
