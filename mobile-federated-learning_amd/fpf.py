"""FPF2 bookkeeping on the GPU (fedavg_trainer.py:108-119, :209-210, :271-278, :314-327).

The reference keeps, per vehicle (``client_num_in_total`` rows), the
difference between its last trained model and the global model it started
from (``local_w_diffs``), a per-parameter EMA ``A_mat``, an EMA of recorded
local iterations ``G_mat``, and derives the FPF2 index the ``sch_pn``
scheduler consumes: ``norm(local_w_diffs * A_mat, dim=1) / G_mat``.  When the
model has ``THRESHOLD_WEIGHT_SIZE`` (config.py:83) or more elements it
switches to the LRU form ``LRU_itr_lst / G_mat``.

``FPFTracker`` keeps that state resident in HBM and updates it with the HIP
kernels of ``csrc/fedavg_fpf.hip``.  The round's client rows do not have to be
uploaded again: ``record_round`` forms the :210 differences from the rows the
aggregate (or a ``RoundSession``) already placed in HBM.  Call order, as in
the reference loop::

    fpf = FPFTracker(client_num_in_total, model.state_dict(), comm_round)
    for round_idx ...:
        last_w = copy.deepcopy(model.cpu().state_dict())        # :165
        fpf.begin_round(last_w)
        ...train clients; w_locals.append(...)                  # :199
        #   either fpf.record_client(client_idx, w) here (:210), or after :217:
        w_glob = aggregate(w_locals)                            # :217
        fpf.record_round(client_indexes, w_locals, w_glob)      # :210, rows already in HBM
        model.load_state_dict(w_glob)                           # :219
        FPF2_idx_lst = fpf.fpf_index()                          # :271-278
        ...
        fpf.end_round(round_idx, client_indexes, local_itr, w_glob)  # :314-327

Results: ``local_w_diffs``, ``G_mat``, ``local_itr_lst`` and ``LRU_itr_lst``
are bit-identical to the reference's; ``A_mat`` and the index go through one
fp64-accumulated reduction each (``mean`` at :319, ``norm`` at :272) and agree
with the reference to its own fp32 rounding error (tests/test_gpu_parity.py,
pinned by the reference's own round loop: tests/golden/fpf).

Models with fp64 / fp16 / bf16 keys follow ``torch.cat``'s promotion at
:210/:316: each key's difference is formed in its own dtype and the
concatenation has the promoted dtype T of all keys.  ``local_w_diffs`` stays
fp32 (it receives fl32 of the T values), :317 runs in promote(fp32, T), and
:319 in T: ``A_mat`` becomes fp64 after the first ``end_round`` of a model
with an fp64 key (and the FPF2 index fp64 with it), while a pure fp16/bf16
model forms ``g / G2 / g.mean()`` in 16-bit arithmetic before adding it to
the fp32 ``A_mat``.  These run the per-key kernels of the promoted path
(``fedavg_fpf_cat_diff`` / ``fedavg_fpf_end_round_promoted`` /
``fedavg_fpf_index_f64``) over the aggregate's per-dtype group rows.

Error behaviour kept: a client index outside ``[-N, N)`` raises
``IndexError`` where the reference's tensor indexing does (:210 in full mode,
:322 when iterations are recorded); ``round_idx`` outside
``[-comm_round, comm_round)`` raises ``IndexError`` (:322/:327); a bool key
raises ``RuntimeError`` at :210 (torch refuses ``bool - bool``).
"""
from __future__ import annotations

import ctypes
from typing import Mapping, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .layout import KeyTable
from .reduce import ALIGN_ELEMS

__all__ = ["FPFTracker", "G1", "G2", "THRESHOLD_WEIGHT_SIZE"]

G1 = 2  # config.py:74
G2 = 2  # config.py:75
THRESHOLD_WEIGHT_SIZE = 100000  # config.py:83

_KIND = {torch.float32: 0, torch.float64: 1, torch.float16: 2, torch.bfloat16: 3}  # fedavg_fpf_groups.kind
_KIND_F64_FROM_F32 = 4  # fedavg_fpf_end_round_promoted: the first fp64 round (A_mat still fp32)


class FPFTracker:
    """Device-resident FPF2 state for ``client_num_in_total`` vehicles."""

    def __init__(self, client_num_in_total: int, model_state: Mapping[str, torch.Tensor], comm_round: int, *,
                 device: Optional[torch.device] = None, g1: float = G1, g2: float = G2,
                 threshold: int = THRESHOLD_WEIGHT_SIZE, aggregator=None):
        if device is None:
            if not torch.cuda.is_available():
                raise _lib.FedAvgLibraryError("no HIP device visible: FPFTracker has no CPU fallback")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("FPFTracker needs a cuda (HIP) device")
        self._lib = _lib.load()
        self.n = int(client_num_in_total)
        if self.n < 1:
            raise ValueError("client_num_in_total must be >= 1")
        self.comm_round = int(comm_round)
        self.g1, self.g2 = float(g1), float(g2)
        self.weight_size = sum(int(t.numel()) for t in model_state.values())  # :112
        self.full = self.weight_size < threshold  # :113
        self._agg = aggregator
        dev = self.device
        self._itr = torch.zeros((self.comm_round, self.n), dtype=torch.float32, device=dev)  # :109
        self._g = torch.zeros(self.n, dtype=torch.float32, device=dev)  # :110
        self._out = torch.empty(self.n, dtype=torch.float32, device=dev)
        self._out_host = torch.empty(self.n, dtype=torch.float32, pin_memory=True)
        self._mixed = False
        self._a_is64 = False
        if self.full:
            self.table = KeyTable(model_state)
            self._has_bool = any(e.src_dtype == torch.bool for e in self.table.entries)
            if set(self.table.groups) != {torch.float32}:
                self._init_promoted(dev)
        if self.full and not self._mixed:
            self.P = self.table.groups[torch.float32].P
            self.ld = self.table.groups[torch.float32].ld
            self._has_bool = any(e.src_dtype == torch.bool for e in self.table.entries)
            self._diffs = torch.zeros((self.n, self.ld), dtype=torch.float32, device=dev)  # :115
            self._a = torch.ones(self.ld, dtype=torch.float32, device=dev)  # :114
            self._last_w = torch.zeros(self.ld, dtype=torch.float32, device=dev)
            self._w_glob = torch.zeros(self.ld, dtype=torch.float32, device=dev)
            self._row = torch.zeros((1, self.ld), dtype=torch.float32, device=dev)
            self._host = torch.zeros((1, self.ld), dtype=torch.float32, pin_memory=True)
            self._ws = torch.empty(max(1, self._lib.fedavg_fpf_workspace(self.P)), dtype=torch.float64, device=dev)
            self._lru = None
        elif not self.full:
            self.P = self.weight_size
            self._lru = torch.zeros(self.n, dtype=torch.float32, device=dev)  # :118
        self._have_last_w = False

    def _init_promoted(self, dev) -> None:
        """State for a model with fp64/fp16/bf16 keys: local_w_diffs / A_mat in
        torch.cat's column order over every key, per-dtype group rows for
        last_w, one client and w_glob, and the device key table."""
        self._mixed = True
        T = None
        for e in self.table.entries:
            T = e.src_dtype if T is None else torch.promote_types(T, e.src_dtype)
        self.T = T  # torch.cat's result dtype at :210/:316
        self.P = self.weight_size
        self.ld = max((self.P + ALIGN_ELEMS - 1) // ALIGN_ELEMS * ALIGN_ELEMS, ALIGN_ELEMS)
        gidx = {dt: i for i, dt in enumerate(self.table.groups)}
        # an integer key's difference (held as fp32 in the fp32 group) is cast to a 16-bit T by the cat
        rnd = _KIND[T] if T in (torch.float16, torch.bfloat16) else 0
        keys, cat = [], 0
        for e in self.table.entries:
            keys.append([e.numel, cat, gidx[e.dtype], e.offset, 0 if e.src_dtype.is_floating_point else rnd])
            cat += e.numel
        self._keys = torch.tensor(keys, dtype=torch.int64).to(dev)
        groups = self.table.groups
        self._gl = {dt: torch.zeros(g.ld, dtype=dt, device=dev) for dt, g in groups.items()}  # last_w (:165)
        self._gr = {dt: torch.zeros((1, g.ld), dtype=dt, device=dev) for dt, g in groups.items()}  # one client
        self._gg = {dt: torch.zeros(g.ld, dtype=dt, device=dev) for dt, g in groups.items()}  # w_glob
        self._gh = {dt: torch.zeros((1, g.ld), dtype=dt, pin_memory=True) for dt, g in groups.items()}
        self._diffs = torch.zeros((self.n, self.ld), dtype=torch.float32, device=dev)  # :115
        self._a = torch.ones(self.ld, dtype=torch.float32, device=dev)  # :114
        self._a64 = torch.ones(self.ld, dtype=torch.float64, device=dev) if T == torch.float64 else None
        self._gd = torch.zeros(self.ld, dtype=torch.float64, device=dev)  # global_w_diff (:316), T values
        self._ws = torch.empty(max(1, self._lib.fedavg_fpf_workspace(self.P)), dtype=torch.float64, device=dev)
        self._out64 = torch.empty(self.n, dtype=torch.float64, device=dev)
        self._out64_host = torch.empty(self.n, dtype=torch.float64, pin_memory=True)
        self._lru = None

    # -- state views (the reference's tensors) ---------------------------
    @property
    def local_w_diffs(self) -> torch.Tensor:
        return self._diffs[:, :self.P]

    @property
    def A_mat(self) -> torch.Tensor:
        return (self._a64 if self._a_is64 else self._a)[:self.P]

    @property
    def G_mat(self) -> torch.Tensor:
        return self._g

    @property
    def local_itr_lst(self) -> torch.Tensor:
        return self._itr

    @property
    def LRU_itr_lst(self) -> torch.Tensor:
        return self._lru

    # -- helpers ---------------------------------------------------------
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _row_index(self, c) -> int:
        r = int(c)
        if not -self.n <= r < self.n:
            raise IndexError(f"index {r} is out of bounds for dimension 0 with size {self.n}")
        return r + self.n if r < 0 else r

    def _aggregator(self):
        if self._agg is not None:
            return self._agg
        from .aggregate import default_aggregator

        return default_aggregator(self.device)

    def _upload(self, table: KeyTable, sd: Mapping[str, torch.Tensor], dst: torch.Tensor) -> None:
        """Pack one state_dict into the pinned row and copy it to ``dst`` [ld]
        (a state_dict already on this GPU is packed in HBM by one kernel)."""
        agg = self._aggregator()
        where = agg._client_device(table, [sd])  # ValueError for another GPU
        ptrs, keep = table.collect([sd], where)
        g = table.groups[torch.float32]
        if where.type == "cuda":
            with torch.cuda.device(self.device):
                agg._pack_on_device(table, g, ptrs, 0, dst, torch.cuda.current_stream(self.device))
            del keep
            return
        items = table.pack_items(g, ptrs, 0, self.ld)
        with torch.cuda.device(self.device):
            torch.cuda.current_stream(self.device).synchronize()  # the pinned row is free again
            _lib.check(self._lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], self._host.data_ptr(), 4,
                                                  max(1, torch.get_num_threads())), "fedavg_pack_rows")
            dst.copy_(self._host[0], non_blocking=True)
        del keep

    def _check_glob_table(self, w_glob) -> KeyTable:
        gt = KeyTable(w_glob)
        if (set(gt.groups) != set(self.table.groups)
                or [(e.name, e.numel, e.dtype) for e in gt.entries]
                != [(e.name, e.numel, e.dtype) for e in self.table.entries]):
            raise ValueError("w_glob does not hold the tracked model's keys/shapes/dtypes")
        return gt

    def _same_round_table(self, table: KeyTable) -> bool:
        return ([(e.name, e.numel, e.dtype) for e in table.entries]
                == [(e.name, e.numel, e.dtype) for e in self.table.entries])

    # -- promoted (fp64 / fp16 / bf16 keys) path ---------------------------
    def _upload_groups(self, table: KeyTable, sd: Mapping[str, torch.Tensor], dsts) -> None:
        """Pack one state_dict's dtype groups into ``dsts[dtype]`` (device,
        row 0): on the device from device tensors, else through the pinned rows."""
        agg = self._aggregator()
        where = agg._client_device(table, [sd])  # ValueError for another GPU
        ptrs, keep = table.collect([sd], where)
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device)
            if where.type == "cuda":
                for dt, g in table.groups.items():
                    agg._pack_on_device(table, g, ptrs, 0, dsts[dt], stream)
            else:
                stream.synchronize()  # the pinned rows are free again
                for dt, g in table.groups.items():
                    host = self._gh[dt]
                    items = table.pack_items(g, ptrs, 0, g.ld)
                    _lib.check(self._lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], host.data_ptr(),
                                                          host.element_size(), max(1, torch.get_num_threads())),
                               "fedavg_pack_rows")
                    dsts[dt].reshape(-1)[:g.ld].copy_(host[0], non_blocking=True)
        del keep

    def _groups(self, rows) -> "_lib.FpfGroups":
        """fedavg_fpf_groups from {dtype: (device tensor whose first element is
        row 0, row stride in elements)}; unused groups stay kind 0."""
        s = _lib.FpfGroups()
        for i, dt in enumerate(self.table.groups):
            t, ld = rows[dt]
            s.base[i] = t.data_ptr()
            s.ld[i] = int(ld)
            s.kind[i] = _KIND[dt]
        return s

    def _cat_rows(self, rows, idx: Sequence[int]) -> None:
        """:210 for client rows ``rows[dtype]`` [K, ld_g] -> local_w_diffs[idx]
        (duplicates: the reference's sequential writes leave the last one)."""
        last = {}
        for k, r in enumerate(idx):
            last[r] = k
        ks = sorted(last.values())
        groups = [(0, list(idx))] if len(ks) == len(idx) else [(k, [idx[k]]) for k in ks]
        lastg = self._groups({dt: (self._gl[dt], self.table.groups[dt].ld) for dt in self.table.groups})
        with torch.cuda.device(self.device):
            for k0, rs in groups:
                cur = self._groups({dt: (t[k0], t.stride(0)) for dt, t in rows.items()})
                ridx = torch.tensor(rs, dtype=torch.int64).to(self.device, non_blocking=True)
                _lib.check(self._lib.fedavg_fpf_cat_diff(
                    self._keys.data_ptr(), self._keys.shape[0], self.P, ctypes.addressof(cur), len(rs),
                    ctypes.addressof(lastg), ridx.data_ptr(), self.n, self._diffs.data_ptr(), self.ld, 0,
                    self._stream()), "fedavg_fpf_cat_diff")

    def _glob_groups(self, w_glob):
        """w_glob's dtype groups on the device: the averaged groups the
        aggregate left in HBM, else uploaded."""
        last = self._aggregator()._last
        acc = last.get("acc")
        if (acc is not None and acc() is w_glob and set(last.get("dev", {})) == set(self.table.groups)
                and self._same_round_table(last["table"])):
            return {dt: (last["dev"][dt][1], self.table.groups[dt].ld) for dt in self.table.groups}
        gt = self._check_glob_table(w_glob)
        self._upload_groups(gt, w_glob, self._gg)
        return {dt: (self._gg[dt], self.table.groups[dt].ld) for dt in self.table.groups}

    def _end_round_promoted(self, w_glob, keep_dev, s) -> None:
        """:316-319 under torch.cat's promotion."""
        cur = self._groups(self._glob_groups(w_glob))
        lastg = self._groups({dt: (self._gl[dt], self.table.groups[dt].ld) for dt in self.table.groups})
        _lib.check(self._lib.fedavg_fpf_cat_diff(
            self._keys.data_ptr(), self._keys.shape[0], self.P, ctypes.addressof(cur), 1, ctypes.addressof(lastg),
            None, 1, self._gd.data_ptr(), self.ld, 1, s), "fedavg_fpf_cat_diff")
        a = self._a64 if self.T == torch.float64 else self._a
        kind = _KIND[self.T]
        if self.T == torch.float64 and not self._a_is64:
            # the reference's A_mat is still fp32 here (:114): its product with
            # (1 - 1/G2) is an fp32 one, the sum with the fp64 term promotes
            self._a64.copy_(self._a)  # exact widening, on the current stream (= s)
            kind = _KIND_F64_FROM_F32
        _lib.check(self._lib.fedavg_fpf_end_round_promoted(
            self._diffs.data_ptr(), self.n, self.ld, keep_dev.data_ptr(), a.data_ptr(), self._gd.data_ptr(), self.P,
            kind, self.g2, self._ws.data_ptr(), self._ws.numel(), s), "fedavg_fpf_end_round_promoted")
        if self.T == torch.float64:
            self._a_is64 = True  # fl32(A_mat * c2) + fp64 term -> fp64 from now on

    def _check_bool(self):
        if self._has_bool:
            raise RuntimeError("Subtraction, the `-` operator, with a bool tensor is not supported "
                               "(fedavg_trainer.py:210 on a state_dict with bool buffers)")

    def _set_rows(self, rows: torch.Tensor, ld_rows: int, idx: Sequence[int]) -> None:
        # duplicates: the reference's sequential row writes leave the last one
        last = {}
        for k, r in enumerate(idx):
            last[r] = k
        ks = sorted(last.values())
        with torch.cuda.device(self.device):
            if len(ks) == len(idx):
                groups = [(0, list(idx))]
            else:
                groups = [(k, [idx[k]]) for k in ks]
            for k0, rs in groups:
                ridx = torch.tensor(rs, dtype=torch.int64).to(self.device, non_blocking=True)
                _lib.check(self._lib.fedavg_fpf_set_rows_f32(
                    self._diffs.data_ptr(), self.n, self.ld, ridx.data_ptr(), len(rs), rows[k0].data_ptr(), ld_rows,
                    self._last_w.data_ptr(), self.P, self._stream()), "fedavg_fpf_set_rows_f32")

    def _need_last_w(self):
        if not self._have_last_w:
            raise RuntimeError("begin_round(last_w) must be called first (fedavg_trainer.py:165)")

    # -- the reference's steps -------------------------------------------
    def begin_round(self, last_w: Mapping[str, torch.Tensor]) -> None:
        """:165 -- the global model the round's clients start from."""
        if self.full and self._mixed:
            self._upload_groups(self.table, last_w, self._gl)
        elif self.full:
            self._upload(self.table, last_w, self._last_w)
        self._have_last_w = True

    def record_client(self, client_idx, w: Mapping[str, torch.Tensor]) -> None:
        """:209-210 -- ``local_w_diffs[client_idx] = cat(w - last_w)`` (uploads ``w``)."""
        if not self.full:
            return
        self._need_last_w()
        r = self._row_index(client_idx)
        self._check_bool()
        if self._mixed:
            self._upload_groups(self.table, w, {dt: t[0] for dt, t in self._gr.items()})
            self._cat_rows(self._gr, [r])
            return
        self._upload(self.table, w, self._row[0])
        self._set_rows(self._row, self.ld, [r])

    def record_round(self, client_indexes, w_locals, w_glob) -> None:
        """:209-210 for every client of the round, from the rows the last
        ``aggregate`` / ``RoundSession.finish`` left in HBM (``w_locals[j]``
        is ``client_indexes[j]``'s result).  After ``aggregate`` the dict of
        client 0 holds the average (:449), so the host copies cannot be used
        any more: without those device rows this raises ``ValueError`` --
        call ``record_client`` before ``aggregate`` instead."""
        if not self.full:
            return
        self._need_last_w()
        idx = [self._row_index(c) for c in list(client_indexes)]
        if len(idx) != len(w_locals):
            raise ValueError(f"{len(client_indexes)} client indexes for {len(w_locals)} w_locals")
        if not idx:
            return
        self._check_bool()
        last = self._aggregator()._last
        refs = last.get("refs")
        ok = (refs is not None and last["acc"]() is w_glob and len(refs) == len(w_locals)
              and all(r() is sd for r, (_, sd) in zip(refs, w_locals))
              and set(last.get("dev", {})) == set(self.table.groups)
              and self._same_round_table(last["table"]))
        if not ok:
            raise ValueError("record_round needs the device rows of the aggregate that produced w_glob; "
                             "call record_client(client_idx, w) before aggregate instead")
        has_f32 = torch.float32 in self.table.groups
        devbuf = self._aggregator().materialize_rows() if has_f32 else None  # packed on demand after zero-copy
        if devbuf is None and has_f32:
            raise ValueError("record_round: the round's client dicts are gone; call record_client before aggregate")
        if self._mixed:
            rows = {dt: (devbuf if dt == torch.float32 else last["dev"][dt][0]) for dt in self.table.groups}
            if any(v is None for v in rows.values()):
                raise ValueError("record_round: the round left no device rows for every dtype group; "
                                 "call record_client before aggregate")
            self._cat_rows(rows, idx)
            return
        self._set_rows(devbuf, devbuf.stride(0), idx)

    def fpf_index(self) -> np.ndarray:
        """:271-278 -- the FPF2 index per vehicle, NaN/inf replaced by 0 (float32)."""
        with torch.cuda.device(self.device):
            s = self._stream()
            if self._a_is64:  # A_mat is fp64 (a model with an fp64 key, after its first end_round)
                _lib.check(self._lib.fedavg_fpf_index_f64(self._diffs.data_ptr(), self.n, self.ld, self.P,
                                                          self._a64.data_ptr(), self._g.data_ptr(),
                                                          self._out64.data_ptr(), s), "fedavg_fpf_index_f64")
                self._out64_host.copy_(self._out64, non_blocking=True)
                torch.cuda.current_stream(self.device).synchronize()
                return self._out64_host.numpy().copy()
            if self.full:
                _lib.check(self._lib.fedavg_fpf_index_f32(self._diffs.data_ptr(), self.n, self.ld, self.P,
                                                          self._a.data_ptr(), self._g.data_ptr(),
                                                          self._out.data_ptr(), s), "fedavg_fpf_index_f32")
            else:
                _lib.check(self._lib.fedavg_fpf_index_lru(self._lru.data_ptr(), self._g.data_ptr(), self.n,
                                                          self._out.data_ptr(), s), "fedavg_fpf_index_lru")
            self._out_host.copy_(self._out, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
        return self._out_host.numpy().copy()

    def end_round(self, round_idx: int, client_indexes, local_itr, w_glob=None) -> None:
        """:314-327 -- unselected diffs ``-= global_w_diff``, ``A_mat`` EMA,
        ``local_itr_lst`` / ``LRU_itr_lst`` record and the ``G_mat`` EMA."""
        client_indexes = list(client_indexes)
        t = int(round_idx)
        if not -self.comm_round <= t < self.comm_round:
            raise IndexError(f"index {t} is out of bounds for dimension 0 with size {self.comm_round}")
        record = bool(client_indexes) and local_itr > 0  # :321
        with torch.cuda.device(self.device):
            s = self._stream()
            if self.full:
                self._need_last_w()
                if w_glob is None:
                    raise ValueError("full FPF2 mode needs w_glob (fedavg_trainer.py:316)")
                glob_dev = None if self._mixed else self._glob_on_device(w_glob)
                keep = np.ones(self.n, dtype=np.uint8)  # rows NOT in set(range(N)) - set(client_indexes)
                keep[list(set(range(self.n)) - set(client_indexes))] = 0
                keep_dev = torch.from_numpy(keep).to(self.device, non_blocking=True)
            if self.full and self._mixed:
                self._end_round_promoted(w_glob, keep_dev, s)
            elif self.full:
                _lib.check(self._lib.fedavg_fpf_end_round_f32(
                    self._diffs.data_ptr(), self.n, self.ld, keep_dev.data_ptr(), self._a.data_ptr(),
                    glob_dev.data_ptr(), self._last_w.data_ptr(), self.P, self.g2, self._ws.data_ptr(),
                    self._ws.numel(), s), "fedavg_fpf_end_round_f32")
            sel = np.zeros(self.n, dtype=np.uint8)
            sel[[self._row_index(c) for c in client_indexes] if record else []] = 1  # :322 IndexError
            sel_dev = torch.from_numpy(sel).to(self.device, non_blocking=True)
            itr_row = self._itr[t + self.comm_round if t < 0 else t]
            _lib.check(self._lib.fedavg_fpf_update_g(
                self._g.data_ptr(), itr_row.data_ptr(), self._lru.data_ptr() if self._lru is not None else None,
                sel_dev.data_ptr(), self.n, float(local_itr) if record else 0.0, 1 if record else 0, self.g1, s),
                "fedavg_fpf_update_g")
            torch.cuda.current_stream(self.device).synchronize()  # keep/sel host arrays may go now
        self._have_last_w = False

    def _glob_on_device(self, w_glob) -> torch.Tensor:
        last = self._aggregator()._last
        acc = last.get("acc")
        if (acc is not None and acc() is w_glob and set(last.get("dev", {})) == {torch.float32}
                and [(e.name, e.numel) for e in last["table"].entries]
                == [(e.name, e.numel) for e in self.table.entries]):
            return last["dev"][torch.float32][1]  # the averaged model the aggregate left in HBM
        self._upload(self._check_glob_table(w_glob), w_glob, self._w_glob)
        return self._w_glob
