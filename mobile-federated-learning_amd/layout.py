"""state_dict <-> packed client-major buffers.

The reference hands the reduction a list of host state_dicts
(``w_locals``, fedavg_trainer.py:199; produced by ``net.cpu().state_dict()``
in client.py:96) and iterates over ``w_locals[0][1].keys()``
(fedavg_trainer.py:450).  On the device we want ONE contiguous buffer per
result dtype, client-major ``[K, ld]``, every row a client's parameters
flattened in key order, so the kernel streams rows with 16-B loads.

A ``KeyTable`` records, for every key of client 0 in order, its shape, source
dtype, the *result* dtype the reference produces for it and its offset inside
that result group:

* fp32 keys and integer/bool keys -> fp32 group (``int_tensor * float`` is
  promoted to the default dtype fp32 by ATen, so integer buffers such as
  ``num_batches_tracked`` come back as fp32, fedavg_trainer.py:455);
* fp64 keys -> fp64 group; fp16 -> fp16 group; bf16 -> bf16 group.

Each group's row stride ``ld`` is its element count rounded up to
``ALIGN_ELEMS`` (64), so every row starts 256-B aligned (fp32).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Sequence, Tuple

import torch

from .reduce import ALIGN_ELEMS

__all__ = ["KeyEntry", "Group", "KeyTable", "ShapeMismatchError", "result_dtype"]

_FLOAT_GROUPS = (torch.float32, torch.float64, torch.float16, torch.bfloat16)


class ShapeMismatchError(RuntimeError, ValueError):
    """A client's tensor for a key differs in shape from client 0's.

    The reference would broadcast compatible shapes silently or raise a
    RuntimeError from ``+=``; the drop-in always raises.
    """


def result_dtype(src: torch.dtype) -> torch.dtype:
    """dtype of ``tensor(src) * python_float`` under ATen type promotion."""
    if src in _FLOAT_GROUPS:
        return src
    if src.is_complex:
        raise TypeError(f"complex state_dict entries are not supported ({src})")
    if src.is_floating_point:  # float8 and other exotic float types
        raise TypeError(f"unsupported floating dtype {src}")
    return torch.get_default_dtype()  # integer / bool -> fp32


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


@dataclass
class KeyEntry:
    name: str
    shape: Tuple[int, ...]
    src_dtype: torch.dtype
    dtype: torch.dtype  # result dtype == group dtype
    offset: int  # element offset inside the group row
    numel: int


@dataclass
class Group:
    dtype: torch.dtype
    P: int = 0  # valid elements per client row
    keys: List[KeyEntry] = field(default_factory=list)

    @property
    def ld(self) -> int:
        return max(_round_up(self.P, ALIGN_ELEMS), ALIGN_ELEMS)


class KeyTable:
    """Key order, shapes and group offsets of client 0's state_dict."""

    def __init__(self, template: Mapping[str, torch.Tensor]):
        self.entries: List[KeyEntry] = []
        self.groups: Dict[torch.dtype, Group] = OrderedDict()
        for name, t in template.items():
            if not isinstance(t, torch.Tensor):
                raise TypeError(f"state_dict entry {name!r} is not a tensor")
            rdt = result_dtype(t.dtype)
            g = self.groups.setdefault(rdt, Group(rdt))
            e = KeyEntry(name, tuple(t.shape), t.dtype, rdt, g.P, t.numel())
            g.P += e.numel
            g.keys.append(e)
            self.entries.append(e)

    @property
    def total_elements(self) -> int:
        return sum(g.P for g in self.groups.values())

    def signature(self):
        return tuple((e.name, e.shape, e.src_dtype) for e in self.entries)

    def validate(self, state_dicts: Sequence[Mapping[str, torch.Tensor]]) -> None:
        """Every client must hold every key of client 0 with the same shape/dtype.

        A missing key raises ``KeyError`` like the reference's
        ``local_model_params[k]`` (fedavg_trainer.py:457); keys only present in
        later clients are ignored, as the reference iterates client 0's keys.
        """
        for i, sd in enumerate(state_dicts):
            for e in self.entries:
                t = sd[e.name]  # KeyError, as in the reference
                if tuple(t.shape) != e.shape:
                    raise ShapeMismatchError(
                        f"client {i} key {e.name!r}: shape {tuple(t.shape)} != client 0's {e.shape}")
                if t.dtype != e.src_dtype:
                    raise TypeError(f"client {i} key {e.name!r}: dtype {t.dtype} != client 0's {e.src_dtype}")

    def pack_into(self, group: Group, buf: torch.Tensor, state_dicts: Sequence[Mapping[str, torch.Tensor]]) -> None:
        """Copy every client's keys of ``group`` into rows of ``buf`` [K, >=ld]."""
        for i, sd in enumerate(state_dicts):
            row = buf[i]
            for e in group.keys:
                src = sd[e.name]
                dst = row[e.offset:e.offset + e.numel]
                if src.dtype == dst.dtype and src.is_contiguous():
                    dst.copy_(src.reshape(-1))
                else:
                    # integer/bool -> fp32 uses the same static_cast ATen's
                    # TensorIterator applies when it promotes `int * float`
                    dst.copy_(src.reshape(-1).to(dst.dtype))

    def unpack(self, group: Group, flat: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        """Views of ``flat`` [>=P] shaped as the group's keys (result dtype)."""
        out = OrderedDict()
        for e in group.keys:
            out[e.name] = flat[e.offset:e.offset + e.numel].view(e.shape)
        return out
