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

import os
from collections import OrderedDict
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
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
    key_index: "np.ndarray" = None  # positions of this group's keys in the table
    numel: "np.ndarray" = None
    offset: "np.ndarray" = None
    kind: "np.ndarray" = None  # fedavg_pack_item.kind per key

    @property
    def ld(self) -> int:
        return max(_round_up(self.P, ALIGN_ELEMS), ALIGN_ELEMS)


_COLLECT = []


def _collect_ext():
    """The native state_dict walk (csrc/fedavg_collect_ext.cpp), or None if it
    was not built -- it only speeds up host bookkeeping; the Python walk below
    computes the same pointers and raises the same errors."""
    if not _COLLECT:
        mod = None
        try:
            import importlib.util

            from .build import collect_ext_path

            # FEDAVG_COLLECT_EXT_PATH: a sanitizer build of the same source
            # (tests/test_native_sanitized.py); the in-tree build otherwise
            path = Path(os.environ.get("FEDAVG_COLLECT_EXT_PATH") or collect_ext_path())
            if path.exists():
                spec = importlib.util.spec_from_file_location("fedavg_collect_ext", path)
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
        except (ImportError, OSError):
            mod = None
        _COLLECT.append(mod)
    return _COLLECT[0]


_META_TEMPLATES: Dict[tuple, List[torch.Tensor]] = {}  # KeyTable.meta_template, by signature

# fedavg_pack_item.kind codes (include/fedavg_amd.h)
_PACK_KIND = {torch.int64: 1, torch.int32: 2, torch.int16: 3, torch.int8: 4, torch.uint8: 5, torch.bool: 6}


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
        self._names = [e.name for e in self.entries]
        self._template = [template[n] for n in self._names]
        self._shapes = [torch.Size(e.shape) for e in self.entries]
        self._dtypes = [e.src_dtype for e in self.entries]
        # per group: column indices into the entry list + pack metadata
        index = {id(e): i for i, e in enumerate(self.entries)}
        for g in self.groups.values():
            g.key_index = np.array([index[id(e)] for e in g.keys], dtype=np.int64)
            g.numel = np.array([e.numel for e in g.keys], dtype=np.int64)
            g.offset = np.array([e.offset for e in g.keys], dtype=np.int64)
            g.kind = np.array([0 if e.src_dtype == g.dtype else _PACK_KIND[e.src_dtype] for e in g.keys],
                              dtype=np.int64)

    def client_device(self, state_dicts: Sequence[Mapping[str, torch.Tensor]]) -> torch.device:
        """Where the clients' tensors live, read from client 0's first key:
        the host (client.py:96 returns ``net.cpu().state_dict()``) or one HIP
        device (clients left in HBM).  :meth:`collect` then requires every
        tensor of every client to be there."""
        if not state_dicts or not self._names:
            return torch.device("cpu")
        t = state_dicts[0][self._names[0]]  # KeyError, as in the reference
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"state_dict entry {self._names[0]!r} is not a tensor")
        if t.device.type not in ("cpu", "cuda"):
            raise TypeError(f"state_dict tensors on {t.device} are not supported (host or HIP device only)")
        return t.device

    def collect(self, state_dicts: Sequence[Mapping[str, torch.Tensor]], device: Optional[torch.device] = None):
        """Validate every client against client 0 and gather source addresses.

        Returns ``(ptrs, keepalive)``: ``ptrs`` is an int64 ``[K, n_keys]``
        array of data pointers in table order, all on ``device`` (default:
        :meth:`client_device`); ``keepalive`` holds contiguous copies made for
        non-contiguous sources.  Raises like :meth:`validate`, and
        ``TypeError`` for a tensor on another device.  One list comprehension
        per attribute per client keeps the per-key Python cost to a few
        hundred ns.
        """
        names, shapes, dtypes = self._names, self._shapes, self._dtypes
        if device is None:
            device = self.client_device(state_dicts)
        dev_index = -1 if device.type == "cpu" else device.index
        ext = _collect_ext()
        if ext is not None:
            got, bad_i, _bad_j = ext.collect(list(state_dicts), names, self._template, dev_index)
            if got is not None:
                return got.numpy(), []
            # something unusual at client bad_i (missing key, other shape/dtype,
            # non-contiguous tensor or one on another device): the general
            # path below raises the reference's exception or handles it
        ptrs = np.empty((len(state_dicts), len(names)), dtype=np.int64)
        keepalive = []
        for i, sd in enumerate(state_dicts):
            ts = [sd[n] for n in names]  # KeyError, as in the reference
            if [t.shape for t in ts] != shapes or [t.dtype for t in ts] != dtypes:
                self.validate([sd], first_index=i)
                raise AssertionError("unreachable")  # validate raised
            if not all([t.device == device for t in ts]):
                raise TypeError(f"client {i}: every state_dict tensor must be on {device}, like client 0's first "
                                "key (host tensors as client.py:96 returns them, or all on one HIP device)")
            if not all([t.is_contiguous() for t in ts]):
                ts = [t if t.is_contiguous() else t.contiguous() for t in ts]
                keepalive.append(ts)
            ptrs[i] = [t.data_ptr() for t in ts]
        return ptrs, keepalive

    def forget_tensors(self) -> "KeyTable":
        """Replace the template tensors (client 0's, kept for the native walk's
        shape/dtype checks) by meta tensors of the same shapes and dtypes, so a
        table retained across rounds does not keep a round's host tensors
        alive.  Idempotent; returns self."""
        if self._template and self._template[0].device.type != "meta":
            self._template = self.meta_template()
        return self

    def meta_template(self) -> List[torch.Tensor]:
        """Meta tensors with the keys' shapes and source dtypes, shared by every
        table of the same signature (350 meta tensors cost ~1 ms to make; a
        streamed round's finish needs them on its critical path)."""
        sig = self.signature()
        got = _META_TEMPLATES.get(sig)
        if got is None:
            got = [torch.empty(e.shape, dtype=e.src_dtype, device="meta") for e in self.entries]
            if len(_META_TEMPLATES) >= 16:
                _META_TEMPLATES.clear()
            _META_TEMPLATES[sig] = got
        return list(got)

    def try_collect(self, state_dicts: Sequence[Mapping[str, torch.Tensor]]):
        """:meth:`collect` for a table reused from an earlier round: the
        ``(ptrs, keepalive)`` pair when client 0 has exactly this table's keys
        in this order and every client holds them with the recorded shapes and
        dtypes as contiguous tensors on one device (checked by the native walk), else
        ``None`` -- never raises for a mismatch; the caller then builds a fresh
        table from client 0."""
        ext = _collect_ext()
        if ext is None or not state_dicts:
            return None
        try:
            device = self.client_device(state_dicts)
        except (KeyError, TypeError):  # client 0 without this table's first key: a fresh table decides
            return None
        # strict0: client 0's dict entries must be exactly this table's keys in order
        got, _, _ = ext.collect(list(state_dicts), self._names, self._template,
                                -1 if device.type == "cpu" else device.index, True)
        return None if got is None else (got.numpy(), [])

    def pack_items(self, group: "Group", ptrs: np.ndarray, row0: int, ld: int) -> np.ndarray:
        """fedavg_pack_item rows [(src, numel, dst_offset, kind)] for clients
        ``row0 .. row0+len(ptrs)-1`` of ``group`` (dst offsets in elements from
        the start of the [K, ld] staging buffer)."""
        nc, nk = ptrs.shape[0], len(group.keys)
        # the numel / offset / kind columns depend only on the table and the row
        # range: built once per (row0, rows, ld); only the addresses change per
        # call.  The array is reused by the next call with the same range, so
        # it must be consumed (the packer does, synchronously) before then.
        cache = group.__dict__.setdefault("_items_cache", {})
        items = cache.get((row0, nc, ld))
        if items is None:
            items = np.empty((nc, nk, 4), dtype=np.int64)
            items[:, :, 1] = group.numel
            items[:, :, 2] = (np.arange(row0, row0 + nc, dtype=np.int64) * ld)[:, None] + group.offset[None, :]
            items[:, :, 3] = group.kind
            if len(cache) >= 256:  # bounded: a session adds one row range per client
                cache.clear()
            cache[(row0, nc, ld)] = items
        np.take(ptrs, group.key_index, axis=1, out=items[:, :, 0])
        return items.reshape(nc * nk, 4)

    @property
    def total_elements(self) -> int:
        return sum(g.P for g in self.groups.values())

    def signature(self):
        sig = self.__dict__.get("_sig")
        if sig is None:
            sig = self._sig = tuple((e.name, e.shape, e.src_dtype) for e in self.entries)
        return sig

    def validate(self, state_dicts: Sequence[Mapping[str, torch.Tensor]], first_index: int = 0) -> None:
        """Every client must hold every key of client 0 with the same shape/dtype.

        A missing key raises ``KeyError`` like the reference's
        ``local_model_params[k]`` (fedavg_trainer.py:457); keys only present in
        later clients are ignored, as the reference iterates client 0's keys.
        """
        for i, sd in enumerate(state_dicts, start=first_index):
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

    def unpack_into(self, target, group: Group, flat: torch.Tensor) -> None:
        """``target[name] = `` the view of ``flat`` for every key of ``group``
        (existing keys keep their place: fedavg_trainer.py:455 assigns into
        client 0's dict) -- one native call, no intermediate dict."""
        ext = _collect_ext()
        if ext is not None and hasattr(ext, "unpack_into") and flat.dim() == 1 and flat.is_contiguous():
            names, offsets, shapes = self._unpack_meta_of(group)
            ext.unpack_into(target, flat, names, offsets, shapes)
            return
        for name, t in self.unpack(group, flat).items():
            target[name] = t

    @staticmethod
    def _unpack_meta_of(group: Group):
        meta = group.__dict__.get("_unpack_meta")
        if meta is None:
            meta = ([e.name for e in group.keys], [int(e.offset) for e in group.keys],
                    [tuple(int(d) for d in e.shape) for e in group.keys])
            group._unpack_meta = meta
        return meta

    def unpack(self, group: Group, flat: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        """Views of ``flat`` [>=P] shaped as the group's keys (result dtype)."""
        ext = _collect_ext()
        if ext is not None and hasattr(ext, "unpack") and flat.dim() == 1 and flat.is_contiguous():
            meta = group.__dict__.get("_unpack_meta")
            if meta is None:
                meta = ([e.name for e in group.keys], [int(e.offset) for e in group.keys],
                        [tuple(int(d) for d in e.shape) for e in group.keys])
                group._unpack_meta = meta
            names, offsets, shapes = meta
            return OrderedDict(zip(names, ext.unpack(flat, offsets, shapes)))
        out = OrderedDict()
        for e in group.keys:
            out[e.name] = flat[e.offset:e.offset + e.numel].view(e.shape)
        return out
