"""Drop-in replacement for ``FedAvgTrainer.aggregate`` (fedavg_trainer.py:441-458).

Same signature, same return object, same dtypes and same fp32 bits as the
reference's torch CPU loop; the weighted sum itself runs in the gfx950 HIP
kernel (libfedavg_amd.so).  Host code stays Python on PyTorch-ROCm.

Use it in the reference's standalone loop without touching ``main_fedavg.py``::

    import mfl_amd
    from fedavg_trainer import FedAvgTrainer       # reference class
    mfl_amd.install(FedAvgTrainer)                 # patches .aggregate

or subclass: ``class Trainer(mfl_amd.FedAvgAggregateMixin, FedAvgTrainer)``.

Contract kept from the reference:
* ``w_locals`` is a list of ``(sample_num, state_dict)`` (fedavg_trainer.py:199);
* empty list -> ``deepcopy(self.model_global.cpu().state_dict())`` (:442-443);
* weights ``n_i / sum(n)`` are Python doubles (:444-447, :453), rounded to
  fp32 once (ATen's scalar cast) for fp32/fp16/bf16 keys, kept double for fp64;
* the returned object IS ``w_locals[0][1]`` (:449), its values replaced by new
  tensors of the key's shape in the reference's result dtype (integer keys come
  back fp32, :455); other clients' dicts are untouched;
* a key missing in a later client raises ``KeyError``; a zero sample total
  raises ``ZeroDivisionError``.
Deliberate tightening: differing shapes or dtypes for one key raise
(``ShapeMismatchError`` / ``TypeError``) instead of broadcasting.
Representation difference: the returned tensors of one dtype group are views
of one freshly allocated host buffer (values and shapes are the reference's;
``load_state_dict`` at fedavg_trainer.py:219 copies them out).

Device-resident clients: when the clients' tensors are all on this GPU (a
deployment that drops client.py:96's ``.cpu()``), the reference's device-
agnostic loop would compute on the GPU and return GPU tensors; so does the
drop-in: the fp32 keys are reduced straight from the clients' own tensors
(``fedavg_reduce_segments_f32``, a pointer-table kernel, no packing; other
dtype groups are packed into rows by ``fedavg_pack_rows_device`` first), and
the result comes back as views of a device buffer, ordered on the current
stream without a host synchronization.
Clients split between host and device raise ``TypeError``.
"""
from __future__ import annotations

import copy
import os
import threading
import time
import weakref
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from .layout import KeyTable
from .layout import _collect_ext as layout_collect_ext
from .reduce import client_sqdist, reduce_packed, reduce_with_sqdist

__all__ = [
    "sample_weights",
    "prepare",
    "client_distances",
    "estimate_delta",
    "DeviceAggregator",
    "aggregate",
    "FedAvgAggregateMixin",
    "install",
    "default_aggregator",
    "client_arena",
]


def sample_weights(sample_nums: Sequence) -> List[float]:
    """``n_i / sum(n)`` as Python numbers (fedavg_trainer.py:444-447, :453)."""
    training_num = 0
    for n in sample_nums:
        training_num += n
    return [n / training_num for n in sample_nums]


class _Prepared(tuple):
    """(acc_dict, KeyTable, state_dicts, weights, src_ptrs, keepalive) for a non-trivial call."""


class _Flats(list):
    """[(Group, flat result)] of a round: written into client 0's dict by
    KeyTable.unpack_into (one native call per dtype group)."""


def prepare(w_locals, model_global=None, table_hint: Optional[KeyTable] = None):
    """Host-side part of ``aggregate``: the reference's early returns and errors.

    Returns either the final answer (empty ``w_locals`` -> copy of the global
    model state, fedavg_trainer.py:442-443; state_dicts without keys -> the
    untouched ``w_locals[0][1]``) or a ``_Prepared`` tuple for the device.
    Raises what the reference raises (``ZeroDivisionError`` on a zero sample
    total, ``KeyError`` on a missing key) and refuses inputs it would have
    broadcast (``ShapeMismatchError``).  Touches no GPU.

    ``table_hint``: the key table of an earlier round, reused when client 0
    has exactly its keys and every client matches it (a round's model
    structure rarely changes); otherwise a fresh table is built from client 0.
    """
    if not w_locals:
        if model_global is None:
            raise ValueError("empty w_locals needs model_global (fedavg_trainer.py:442-443)")
        return copy.deepcopy(model_global.cpu().state_dict())
    sample_nums = [n for n, _ in w_locals]
    acc_dict = w_locals[0][1]
    if len(acc_dict) == 0:
        sum(sample_nums)  # the reference still forms training_num (:444-447)
        return acc_dict
    weights = sample_weights(sample_nums)  # ZeroDivisionError like the reference
    dicts = [sd for _, sd in w_locals]
    for i in range(1, len(dicts)):
        if dicts[i] is acc_dict:
            raise ValueError(
                f"w_locals[{i}][1] is the same dict object as w_locals[0][1]; the reference would read "
                "its own partial sums there (fedavg_trainer.py:199 deep-copies to avoid this)")
    got = table_hint.try_collect(dicts) if table_hint is not None else None
    if got is not None:
        table = table_hint
        ptrs, keepalive = got
    else:
        table = KeyTable(acc_dict)
        ptrs, keepalive = table.collect(dicts)  # validates every client (KeyError / ShapeMismatchError / TypeError)
    return _Prepared((acc_dict, table, dicts, weights, ptrs, keepalive))


def _trivial(w_locals, model_global=None):
    """The reference's early answers (fedavg_trainer.py:442-447) without
    building a key table: the empty list and state_dicts without keys.
    Returns ``(True, answer)`` or ``(False, None)``."""
    if not w_locals or len(w_locals[0][1]) == 0:
        return True, prepare(w_locals, model_global)
    return False, None


# D2H pipelining of the averaged model: the reduce runs in column chunks and
# chunk c's copy to pinned host memory overlaps the reduce of chunk c+1 (the
# copy, ~50 GB/s over PCIe, is the slower of the two).  Chunks of >= 2M
# columns keep every launch a full-chip one; all schedules give the same bits.
# (FEDAVG_D2H_MAX_CHUNKS / FEDAVG_D2H_CHUNK_MIN_COLS override them for measurements)
D2H_CHUNK_MIN_COLS = int(os.environ.get("FEDAVG_D2H_CHUNK_MIN_COLS", str(2 << 20)))
D2H_MAX_CHUNKS = int(os.environ.get("FEDAVG_D2H_MAX_CHUNKS", "8"))
# D2H engine of fedavg_copy_to_host: 0 = the runtime's DMA copy (production:
# a streaming round's finish at K=100 x P=25M measured 2.67 ms in steady state
# vs 3.0-3.1 ms for the 64-workgroup zero-copy kernel),
# > 0 = the zero-copy kernel with that grid.  FEDAVG_D2H_BLOCKS overrides it
# for measurements.
D2H_BLOCKS = int(os.environ.get("FEDAVG_D2H_BLOCKS", "0"))


def column_chunks(P: int) -> List[Tuple[int, int]]:
    """Column ranges the averaged model is reduced and fetched in (256-B aligned starts)."""
    n = max(1, min(D2H_MAX_CHUNKS, P // D2H_CHUNK_MIN_COLS))
    step = -(-P // n)
    step = -(-step // 64) * 64
    return [(c0, min(P, c0 + step)) for c0 in range(0, P, step)] or [(0, 0)]


# An fp32 row reduce with at most this many clients also forms the round's
# :291 sums of squares in the same pass over the rows (fedavg_reduce_sqdist_f32:
# 100 x 25M, 1.76 ms for both against 1.42 + 1.47 ms for the two passes,
# DESIGN.md section 3); client_distances then reads them instead of the rows.
# The reference runs :291 after every aggregate with clients (fedavg_trainer.py
# :289-291), so the drop-in fuses by default; FEDAVG_FUSE_DISTANCES=0 keeps
# the reduce alone.
FUSED_MAX_K = 1024  # rows kernels (fedavg_reduce_sqdist_f32's fused_plan; more clients: the two passes)
# device-resident clients' own tensors (fedavg_device_round_f32): LDS-DMA tiles to 256
# clients, split-row windows to 1024 (round 5)
FUSED_SEGMENTS_MAX_K = 1024
FUSE_DISTANCES = os.environ.get("FEDAVG_FUSE_DISTANCES", "1") != "0"


def fuse_eligible(devbuf: torch.Tensor) -> bool:
    """fp32 rows the one-read aggregate + :291 pass takes: K <= FUSED_MAX_K,
    16-B aligned rows (its loads are 16-B slices; the reduce alone also
    serves unaligned rows)."""
    return (FUSE_DISTANCES and devbuf.dtype == torch.float32 and 0 < devbuf.shape[0] <= FUSED_MAX_K
            and devbuf.data_ptr() % 16 == 0 and (devbuf.shape[0] == 1 or devbuf.stride(0) % 4 == 0)
            and devbuf.stride(-1) == 1)


def reduce_rows(devbuf: torch.Tensor, w_dev: torch.Tensor, P: int, out: torch.Tensor,
                sums: Optional[list] = None) -> None:
    """``reduce_packed`` of [K, ld] rows into ``out``; with ``sums`` (a list)
    and fused-eligible rows, the :291 sums of squares of the same columns are
    formed in the same pass and their [K] fp64 device tensor appended."""
    if sums is not None and fuse_eligible(devbuf):
        sums.append(reduce_with_sqdist(devbuf, w_dev, P, out)[1])
    else:
        reduce_packed(devbuf, w_dev, P, out)


def reduce_and_fetch(devbuf: torch.Tensor, w_dev: torch.Tensor, P: int, d2h_stream,
                     ready: Optional[Sequence] = None,
                     out_host: Optional[torch.Tensor] = None,
                     sums: Optional[dict] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reduce ``devbuf`` [K, ld] on the current stream in ``column_chunks(P)``
    and copy each chunk to a pinned host buffer on ``d2h_stream`` as soon as
    it is reduced.  ``ready[c]`` (optional): an event after which chunk c's
    input columns are in HBM -- the reduce of chunk c then waits only for
    that, so the last client's H2D, the reduce and the D2H pipeline.
    ``out_host`` (optional): a pinned [>=P] buffer allocated ahead (a fresh
    100 MB pinned allocation costs 5.6-8.6 ms); a new one
    otherwise.  ``sums`` (optional dict): fused-eligible fp32 rows also give
    the :291 sums of squares, ``sums[dtype]`` = their [K] fp64 device tensor
    (the chunks' sums added in chunk order).  Returns ``(out_dev, out_host)``;
    the caller synchronizes ``d2h_stream``."""
    dev = devbuf.device
    compute = torch.cuda.current_stream(dev)
    out_dev = torch.empty(P, dtype=devbuf.dtype, device=dev)
    if out_host is None:
        out_host = torch.empty(P, dtype=devbuf.dtype, pin_memory=True)
    chunks = column_chunks(P)
    parts = [] if sums is not None else None
    for c, (c0, c1) in enumerate(chunks):
        if ready is not None:
            compute.wait_event(ready[c])
        reduce_rows(devbuf[:, c0:c1] if len(chunks) > 1 else devbuf, w_dev, c1 - c0, out_dev[c0:c1], parts)
        d2h_stream.wait_stream(compute)
        _fetch(out_dev[c0:c1], out_host[c0:c1], d2h_stream)
    if parts:
        total = parts[0]
        for s in parts[1:]:
            total = total + s
        sums[devbuf.dtype] = total
    return out_dev, out_host


def _fetch(src: torch.Tensor, dst: torch.Tensor, stream) -> None:
    """Device -> pinned host copy on ``stream`` (fedavg_copy_to_host, engine D2H_BLOCKS)."""
    lib = _lib.load()
    _lib.check(lib.fedavg_copy_to_host(src.data_ptr(), dst.data_ptr(), src.numel() * src.element_size(),
                                       D2H_BLOCKS, stream.cuda_stream), "fedavg_copy_to_host")


class _Weights:
    """A pinned + device weight vector reused across calls (no pinned
    allocation per call)."""

    def __init__(self, K: int, wdt: torch.dtype, device: torch.device):
        self.K = K
        self.w_host = torch.empty(K, dtype=wdt, pin_memory=True)
        self.w_dev = torch.empty(K, dtype=wdt, device=device)
        self._w_done = torch.cuda.Event()  # the last weight copy has read w_host

    def upload(self, weights: Sequence[float], stream) -> torch.Tensor:
        """``weights`` (the reference's Python doubles n_i / N) rounded once to
        the group's weight dtype (round to nearest even: the cast ATen applies
        to the scalar at fedavg_trainer.py:455) and copied on ``stream``.
        Waits for the previous call's copy before rewriting the pinned buffer
        (a device-resident round returns without synchronizing)."""
        import numpy as np

        K = len(weights)
        self._w_done.synchronize()
        self.w_host[:K].numpy()[:] = np.array([float(w) for w in weights], dtype=np.float64)
        with torch.cuda.stream(stream):
            self.w_dev[:K].copy_(self.w_host[:K], non_blocking=True)
        self._w_done.record(stream)
        return self.w_dev[:K]


class _Staging(_Weights):
    """Reusable pinned host rows + device buffer for one dtype group, and the
    group's weight vector (pinned + device) so a call uploads the weights with
    its rows instead of allocating a pinned tensor per call."""

    def __init__(self, K: int, ld: int, dtype: torch.dtype, device: torch.device):
        super().__init__(K, torch.float64 if dtype == torch.float64 else torch.float32, device)
        self.ld, self.dtype = ld, dtype
        self._host = None  # pinned rows, allocated on first use (device-resident clients never need them)
        self.dev = torch.empty((K, ld), dtype=dtype, device=device)

    @property
    def host(self) -> torch.Tensor:
        if self._host is None:
            self._host = torch.empty((self.K, self.ld), dtype=self.dtype, pin_memory=True)
        return self._host

    def upload_weights(self, weights: Sequence[float], stream) -> torch.Tensor:
        return self.upload(weights, stream)


class DeviceAggregator:
    """Runs the FedAvg reduction of host state_dicts on one GPU.

    Keeps pinned staging and device buffers between rounds (a round's K and
    model are usually stable), packs client ``i`` into its pinned row and
    starts its H2D copy on a side stream before packing client ``i+1``, so the
    host packing overlaps the PCIe transfer.
    """

    def __init__(self, device: Optional[torch.device] = None):
        if device is None:
            if not torch.cuda.is_available():
                raise _lib.FedAvgLibraryError("no HIP device visible: the FedAvg reduction has no CPU fallback")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("DeviceAggregator needs a cuda (HIP) device")
        _lib.load()  # fail loudly and early if the HIP library is missing
        self._staging: Dict[torch.dtype, _Staging] = {}
        self._copy_stream = None
        self._d2h_stream = None
        self.last_profile: Dict[str, float] = {}
        # device state of the last aggregate call (client rows + averaged model per
        # dtype group), reused by client_distances for the same round
        self._last: Dict[str, object] = {}
        self._session = None  # weakref to the open RoundSession, if any
        self._table_hint: Optional[KeyTable] = None  # last round's key table (prepare reuses it)
        self._table_ws = None  # (pinned, device) staging of the device kernels' tables
        self._table_ws_done = None  # event: the last staged table has been copied and used
        self._seg_weights = None  # weights of the zero-copy (segments) reduce
        # one round at a time per aggregator: the staging buffers are shared
        self._lock = threading.Lock()
        # after a small fp32 round (fedavg_round_f32), the next round with the
        # same key table runs its whole host side in one native call
        # (fedavg_collect_ext.small_round); any other path clears this
        self._fast_small = None
        self.fast_rounds = 0  # rounds finished by the one-call native path
        self.arena_rounds = 0  # device rounds whose fp32 rows were the clients' own (client_arena layout)
        self._warm = False

    # A process's first round paid its HIP first-use costs on the round's
    # critical path.  The HIP API trace of round 0 at 100 x 25M (rocprofv3
    # --hip-trace, profiles/r04/stream/round0_first_use.json) put 64.6 ms in ONE
    # hipLaunchKernel: the first launch of torch's fp64 elementwise add (the
    # column chunks' :291 sums added), i.e. the lazy load of that torch code
    # object; the streams' hipStreamCreateWithPriority cost 6.2-6.6 ms each.
    # warm_up() pays them once, off the round: install() calls it before the
    # loop runs, and a RoundSession's first add() (while clients train).
    WARMUP = os.environ.get("FEDAVG_WARMUP", "1") != "0"
    WARMUP_COPIES = int(os.environ.get("FEDAVG_WARMUP_COPIES", "16"))

    def warm_up(self) -> None:
        """Create the aggregator's streams and launch, once, every kernel a
        round runs besides the reduction's own code object (torch's fp64 add,
        isfinite / all; one tiny fused reduce loads libfedavg_amd's), on a
        scratch problem.  Idempotent."""
        if self._warm or not self.WARMUP:
            return
        self._warm = True
        with torch.cuda.device(self.device):
            copy_s, d2h = self._copy_stream_for(), self._d2h_stream_for()
            with torch.cuda.stream(d2h):
                rows = torch.zeros((17, 64), dtype=torch.float32, device=self.device)
                w = torch.full((17,), 1.0 / 17, dtype=torch.float32, device=self.device)
                out, sums = reduce_with_sqdist(rows, w, 64)
                z = sums + sums
                bool(torch.isfinite(out).all())  # also waits for the work above
                del z
            # the runtime's first DMA copies each way: rounds 0-1 of a process
            # issued their D2H chunks 10x slower than later rounds (DESIGN.md
            # section 6); a few round-trips of a 4 MB scratch here
            host = torch.empty(1 << 20, dtype=torch.float32, pin_memory=True)
            dev = torch.empty(1 << 20, dtype=torch.float32, device=self.device)
            for _ in range(self.WARMUP_COPIES):
                with torch.cuda.stream(copy_s):
                    dev.copy_(host, non_blocking=True)
                d2h.wait_stream(copy_s)
                _fetch(dev, host, d2h)
                copy_s.wait_stream(d2h)
            d2h.synchronize()
            copy_s.synchronize()

    # ------------------------------------------------------------------
    def begin_round(self, template, max_clients: int):
        """Start a streaming round (see ``session.RoundSession``).

        A session owns this aggregator's staging buffers until ``finish``;
        ``aggregate`` and a second ``begin_round`` refuse to run meanwhile.
        """
        from .session import RoundSession

        self._check_no_open_session("begin_round")
        self._fast_small = None
        sess = RoundSession(self, template, max_clients)
        self._session = weakref.ref(sess)
        return sess

    def _check_no_open_session(self, what: str):
        sess = self._session() if self._session is not None else None
        if sess is not None and not sess._finished:
            raise RuntimeError(f"{what}: a RoundSession on this aggregator is still open (call finish first)")

    def _copy_stream_for(self):
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(self.device)
        return self._copy_stream

    def _d2h_stream_for(self):
        # its own stream: PCIe is full duplex, so result D2H runs beside pending H2D
        if self._d2h_stream is None:
            self._d2h_stream = torch.cuda.Stream(self.device)
        return self._d2h_stream

    def _staging_for(self, dtype: torch.dtype, K: int, ld: int) -> _Staging:
        st = self._staging.get(dtype)
        if st is None or st.K < K or st.ld != ld:
            st = _Staging(K, ld, dtype, self.device)
            self._staging[dtype] = st
        return st

    def aggregate(self, w_locals, model_global=None):
        """``FedAvgTrainer.aggregate`` semantics; see the module docstring."""
        fast = self._fast_small
        if fast is not None and type(w_locals) is list and w_locals:
            done = self._small_round_native(w_locals, fast)
            if done is not None:
                return done
        self._fast_small = None
        prep = prepare(w_locals, model_global, self._table_hint)
        if not isinstance(prep, _Prepared):
            return prep  # empty list / no keys: answered on the host like the reference
        self._check_no_open_session("aggregate")
        self._table_hint = prep[1]
        acc_dict, table, dicts, weights, ptrs, keepalive = prep
        on_device = self._client_device(table, dicts).type == "cuda"
        with self._lock:
            if on_device:
                results = self._reduce_groups_device(table, ptrs, weights, dicts)
            else:
                results = self._reduce_groups(table, ptrs, weights)
        del keepalive
        table.forget_tensors()  # retained as the next round's hint and in _last: keep no host tensors
        # weak references: the round's dicts are the caller's (the reference drops
        # them at the next round); a dead or replaced dict simply misses the cache
        try:
            self._last["refs"] = [weakref.ref(sd) for sd in dicts]
            self._last["acc"] = weakref.ref(acc_dict)
        except TypeError:  # plain dicts cannot be weakly referenced: no reuse
            self._last.pop("dev", None)
        if self._last.get("segments"):
            # client 0's own tensors: its dict is about to hold the average
            # (:449), and the rows of a zero-copy round are packed on demand
            # (its keys are exactly the table's: prepare checked them)
            # (names, tensors) -- a dict is made only if a later call needs one
            self._last["seg_keep0"] = (list(acc_dict), list(acc_dict.values()))
        # replace values in place, keeping client 0's key order (fedavg_trainer.py:450-457)
        if isinstance(results, _Flats):
            for g, flat in results:
                table.unpack_into(acc_dict, g, flat)
        else:
            for e in table.entries:
                acc_dict[e.name] = results[e.name]
        return acc_dict

    def _client_device(self, table: KeyTable, dicts) -> torch.device:
        dev = table.client_device(dicts)
        if dev.type == "cuda" and dev != self.device:
            raise ValueError(f"the clients' tensors are on {dev}; this aggregator runs on {self.device}")
        return dev

    def _pack_on_device(self, table: KeyTable, g, ptrs, row0: int, dst: torch.Tensor, stream) -> None:
        """Rows ``row0 ..`` of ``dst`` [K, ld] from device-resident clients
        ``ptrs``: one fedavg_pack_rows_device launch on ``stream``."""
        lib = _lib.load()
        items = table.pack_items(g, ptrs, row0, g.ld)
        n = items.shape[0]
        host_ws, dev_ws = self._stage_ws(lib.fedavg_pack_rows_device_workspace(n))
        _lib.check(lib.fedavg_pack_rows_device(items.ctypes.data, n, dst.data_ptr(), dst.element_size(),
                                               host_ws.data_ptr(), dev_ws.data_ptr(), host_ws.numel(),
                                               stream.cuda_stream), "fedavg_pack_rows_device")
        self._table_ws_done.record(stream)

    def _stage_ws(self, need: int):
        """The (pinned, device) table workspace, at least ``need`` bytes, once
        the previous user has consumed it; the caller records
        ``_table_ws_done`` on its stream after its call."""
        if self._table_ws_done is None:
            self._table_ws_done = torch.cuda.Event()
        self._table_ws_done.synchronize()
        ws = self._table_ws
        if ws is None or ws[0].numel() < need:
            cap = max(need, 1 << 16)
            ws = (torch.empty(cap, dtype=torch.uint8, pin_memory=True),
                  torch.empty(cap, dtype=torch.uint8, device=self.device))
            self._table_ws = ws
        return ws

    # device-resident fp32 groups are reduced straight from the clients'
    # tensors (fedavg_reduce_segments_f32: 4 B per element instead of the
    # rows' 12); FEDAVG_DEVICE_ROWS=1 packs rows first as the streaming path does
    DEVICE_SEGMENTS = os.environ.get("FEDAVG_DEVICE_ROWS", "0") != "1"
    # device rounds from this many fp32 row bytes check for the client_arena layout
    ARENA_MIN_BYTES = int(os.environ.get("FEDAVG_ARENA_MIN_BYTES", str(64 << 20)))

    @staticmethod
    def _segment_tables(g, ptrs):
        import numpy as np

        return (np.ascontiguousarray(ptrs[:, g.key_index]), np.ascontiguousarray(g.numel),
                np.ascontiguousarray(g.offset), np.ascontiguousarray(g.kind))

    @staticmethod
    def _round_meta(g, n_cols: int):
        """The group's key columns for fedavg_device_round_f32, built once per
        table: (n_cols, arrays, their addresses, per-K sizes).  The arrays --
        key_index (None when the group is every key in order), numel, offset,
        kind, contiguous int64 -- are kept alive here; the addresses are what
        the call takes (``ndarray.ctypes`` costs ~1 us per access); per K: the
        integer keys' scratch floats, the partials and the workspace bytes."""
        import numpy as np

        meta = g.__dict__.get("_round_meta")
        if meta is None or meta[0] != n_cols:
            ki = np.ascontiguousarray(g.key_index, dtype=np.int64)
            whole = len(ki) == n_cols and bool(np.array_equal(ki, np.arange(n_cols)))
            arrs = (None if whole else ki, np.ascontiguousarray(g.numel, dtype=np.int64),
                    np.ascontiguousarray(g.offset, dtype=np.int64), np.ascontiguousarray(g.kind, dtype=np.int64))
            addrs = tuple(None if a is None else a.ctypes.data for a in arrs)
            meta = g._round_meta = (n_cols, arrs, addrs, {})
        return meta

    def _device_round(self, g, ptrs, weights, stream):
        """The fp32 group of a device-resident round from the clients' own
        tensors in ONE native call (fedavg_device_round_f32): the walk's
        address table, the reference's weights and the key table go in; the
        averaged group and -- fused by default (K <= 1024, 16-B aligned fp32
        sources) -- the round's :291 sums come out.  Integer keys of a fused
        round are converted into a device scratch first (held here until the
        launches that read it are issued: freed earlier, the caching allocator
        would hand its block to the round's own output on the same stream).
        Returns ``(out, sumsq or None)``."""
        import numpy as np

        lib = _lib.load()
        K, n_cols = ptrs.shape
        if g.P == 0:  # every key of the group is empty: nothing to read (the reference's loop adds empty tensors)
            sums = torch.zeros(K, dtype=torch.float64, device=self.device) if FUSE_DISTANCES else None
            return torch.empty(0, dtype=torch.float32, device=self.device), sums
        _, arrs, (ki_p, numel_p, offset_p, kind_p), sizes = self._round_meta(g, n_cols)
        n = len(arrs[1])
        per_k = sizes.get(K)
        if per_k is None:
            per_k = sizes[K] = (lib.fedavg_device_round_scratch(numel_p, kind_p, n, K),
                                max(1, lib.fedavg_reduce_sqdist_segments_partials(K)),
                                lib.fedavg_device_round_workspace(K, n))
        n_s, n_part, ws_need = per_k
        dev = self.device
        scratch = partials = sumsq = None
        if FUSE_DISTANCES and K <= FUSED_SEGMENTS_MAX_K:
            if n_s:
                scratch = torch.empty(n_s, dtype=torch.float32, device=dev)
            partials = torch.empty(n_part, dtype=torch.float64, device=dev)
            sumsq = torch.empty(K, dtype=torch.float64, device=dev)
        if not ptrs.flags.c_contiguous:
            ptrs = np.ascontiguousarray(ptrs, dtype=np.int64)
        w64 = np.array(weights, dtype=np.float64)
        out_dev = torch.empty(g.P, dtype=torch.float32, device=dev)
        host_ws, dev_ws = self._stage_ws(ws_need)
        rc = lib.fedavg_device_round_f32(ptrs.ctypes.data, n_cols, ki_p, numel_p, offset_p, kind_p, n, K,
                                         w64.ctypes.data, out_dev.data_ptr(),
                                         None if partials is None else partials.data_ptr(),
                                         0 if partials is None else n_part,
                                         None if sumsq is None else sumsq.data_ptr(),
                                         None if scratch is None else scratch.data_ptr(),
                                         0 if scratch is None else n_s, host_ws.data_ptr(),
                                         dev_ws.data_ptr(), host_ws.numel(), stream.cuda_stream)
        self._table_ws_done.record(stream)
        if rc not in (0, 1):
            _lib.check(rc, "fedavg_device_round_f32")
        del scratch, partials  # freed in `stream` order, after the launches that read them
        return out_dev, (sumsq if rc == 0 else None)

    def _sqdist_segments(self, table: KeyTable, dicts, glob: torch.Tensor) -> torch.Tensor:
        """:291 sums of squares straight from device-resident clients' tensors."""
        lib = _lib.load()
        g = table.groups[torch.float32]
        ptrs, keep = table.collect(dicts, self.device)
        K = len(dicts)
        cptrs, numel, offset, kind = self._segment_tables(g, ptrs)
        stream = torch.cuda.current_stream(self.device)
        partials = torch.empty(max(1, lib.fedavg_segments_partials(numel.ctypes.data, len(numel), K)),
                               dtype=torch.float64, device=self.device)
        sumsq = torch.empty(K, dtype=torch.float64, device=self.device)
        host_ws, dev_ws = self._stage_ws(lib.fedavg_segments_workspace(K, len(numel)))
        _lib.check(lib.fedavg_client_sqdist_segments_f32(cptrs.ctypes.data, numel.ctypes.data, offset.ctypes.data,
                                                         kind.ctypes.data, len(numel), K, glob.data_ptr(),
                                                         partials.data_ptr(), partials.numel(), sumsq.data_ptr(),
                                                         host_ws.data_ptr(), dev_ws.data_ptr(), host_ws.numel(),
                                                         stream.cuda_stream), "fedavg_client_sqdist_segments_f32")
        self._table_ws_done.record(stream)
        del keep
        return sumsq

    @staticmethod
    def _client0_tensors(last) -> "OrderedDict[str, torch.Tensor]":
        """Client 0's own tensors of a zero-copy round as a dict (its dict
        holds the average since :449), made from the (names, tensors) the
        round kept."""
        keep = last["seg_keep0"]
        if isinstance(keep, tuple):
            keep = last["seg_keep0"] = OrderedDict(zip(*keep))
        return keep

    def materialize_rows(self):
        """The last round's client rows in HBM (``[K, ld]``), packing them on
        demand after a zero-copy round: client 0 from its original tensors
        (its dict now holds the average, :449), the others from their dicts.
        Returns the rows or None when the last round left none."""
        last = self._last
        if "seg_keep0" not in last:
            dev = last.get("dev", {}).get(torch.float32)
            return None if dev is None else dev[0]
        refs = last.get("refs")
        dicts = [self._client0_tensors(last)] + [r() for r in refs[1:]] if refs is not None else [None]
        if any(d is None for d in dicts):
            return None
        table, K = last["table"], last["K"]
        g = table.groups[torch.float32]
        st = self._staging_for(torch.float32, K, g.ld)
        ptrs, keep = table.collect(dicts, self.device)
        with torch.cuda.device(self.device):
            self._pack_on_device(table, g, ptrs, 0, st.dev, torch.cuda.current_stream(self.device))
        del keep
        last["dev"][torch.float32] = (st.dev[:K], last["dev"][torch.float32][1])
        del last["seg_keep0"]
        return st.dev[:K]

    @staticmethod
    def _arena_rows(g, ptrs, dicts) -> Optional[torch.Tensor]:
        """The clients' fp32 group as a ``[K, P]`` view with row stride ``ld``
        when their tensors already ARE the packed layout: every client's keys
        back to back at the group's offsets, clients one pitch apart, in one
        allocation (``client_arena`` makes such dicts; so does any simulator
        that keeps its client models in one buffer).  Then the row reduce runs
        on the clients' memory directly -- no packing, and one allocation's
        address translation instead of K.  None when
        the pointers do not form that layout."""
        import numpy as np

        meta = g.__dict__.get("_arena_meta")
        if meta is None:  # per table: the group's byte offsets, and whether it is every key in order
            whole = bool(np.array_equal(g.key_index, np.arange(len(g.key_index))))
            meta = g._arena_meta = (bool((g.kind == 0).all()) and len(g.key_index) > 0, whole, g.offset * 4)
        ok, whole, off4 = meta
        if dicts is None or not ok:
            return None
        K, j0, j1 = ptrs.shape[0], int(g.key_index[0]), int(g.key_index[-1])
        base = int(ptrs[0, j0]) - int(off4[0])
        pitch = int(ptrs[1, j0] - ptrs[0, j0]) if K > 1 else (g.P + 3) // 4 * 16
        if base % 16 or pitch % 16 or pitch < g.P * 4:
            return None
        if int(ptrs[K - 1, j1]) != base + (K - 1) * pitch + int(off4[-1]):  # the far corner first: O(1) reject
            return None
        cols = ptrs if whole and ptrs.shape[1] == len(off4) else ptrs[:, g.key_index]
        expect = off4 + base if K == 1 else (np.arange(base, base + K * pitch, pitch)[:, None] + off4)
        if not np.array_equal(cols, expect.reshape(cols.shape)):
            return None
        first = dicts[0][g.keys[0].name]
        last = dicts[-1][g.keys[-1].name]
        st = first.untyped_storage()
        if last.untyped_storage().data_ptr() != st.data_ptr() or (base - st.data_ptr()) % 4:
            return None
        # the row kernels read whole 16-B slices: the last row's final slice may
        # run up to 12 B past P, which as_strided's own check does not cover
        if (base - st.data_ptr()) + (K - 1) * pitch + (g.P + 3) // 4 * 16 > st.nbytes():
            return None
        try:
            return first.as_strided((K, g.P), (pitch // 4, 1), (base - st.data_ptr()) // 4)
        except RuntimeError:  # outside the storage
            return None

    def _reduce_groups_device(self, table: KeyTable, ptrs, weights, dicts=None) -> "OrderedDict[str, torch.Tensor]":
        """Device-resident clients: the fp32 group reduced straight from the
        clients' tensors (zero-copy: the row reduce on them when they already
        form the packed layout, else the segments kernel), other groups packed
        in HBM and reduced; the averaged model returned as device tensors on
        the current stream (no host round trip, no synchronization: like the
        reference's torch ops on device tensors)."""
        K, dev = ptrs.shape[0], self.device
        t0 = time.perf_counter()
        results = _Flats()
        with torch.cuda.device(dev):
            compute = torch.cuda.current_stream(dev)
            if self._copy_stream is not None:
                compute.wait_stream(self._copy_stream)  # earlier users of the staging are done
            self._last = {"table": table, "K": K, "dev": {}}
            for g in table.groups.values():
                # the layout check costs tens of us of host time: worth it where the
                # row kernel's advantage is (large rounds)
                rows = (self._arena_rows(g, ptrs, dicts)
                        if g.dtype == torch.float32 and K * g.P * 4 >= self.ARENA_MIN_BYTES else None)
                if rows is not None:
                    w = self._seg_weights
                    if w is None or w.K < K:
                        w = self._seg_weights = _Weights(K, torch.float32, self.device)
                    out_dev = torch.empty(g.P, dtype=torch.float32, device=dev)
                    sums = []
                    reduce_rows(rows, w.upload(weights, compute), g.P, out_dev, sums)
                    self._last["dev"][g.dtype] = (rows, out_dev)  # the clients' own rows: :291 / FPF read them
                    if sums:
                        self._last.setdefault("sumsq", {})[g.dtype] = sums[0]
                    self.arena_rounds += 1
                elif g.dtype == torch.float32 and self.DEVICE_SEGMENTS:
                    out_dev, sums = self._device_round(g, ptrs, weights, compute)
                    if sums is not None:
                        self._last.setdefault("sumsq", {})[g.dtype] = sums
                    self._last["dev"][g.dtype] = (None, out_dev)  # no rows: see materialize_rows
                    self._last["segments"] = True
                else:
                    st = self._staging_for(g.dtype, K, g.ld)
                    self._pack_on_device(table, g, ptrs, 0, st.dev, compute)
                    w_dev = st.upload_weights(weights, compute)
                    out_dev = torch.empty(g.P, dtype=g.dtype, device=dev)
                    sums = []
                    reduce_rows(st.dev[:K], w_dev, g.P, out_dev, sums)
                    self._last["dev"][g.dtype] = (st.dev[:K], out_dev)
                    if sums:
                        self._last.setdefault("sumsq", {})[g.dtype] = sums[0]
                results.append((g, out_dev))
        self.last_profile = {"pack_issue_ms": (time.perf_counter() - t0) * 1e3, "h2d_kernel_d2h_ms": 0.0}
        return results

    # rows per H2D chunk: big enough to amortise a copy launch, small enough
    # that the first chunk's DMA starts while the host still packs the rest
    CHUNK_BYTES = int(os.environ.get("FEDAVG_CHUNK_BYTES", str(32 << 20)))
    # fp32-only rounds whose rows are at most this many bytes run as ONE native
    # call (fedavg_round_f32): pack, upload, reduce, fetch, wait -- no per-step
    # Python/torch overhead, which is most of a tiny model's round.  Larger
    # rounds take the pipelined path below (packing overlapped with H2D, the
    # D2H overlapped with the reduce).  FEDAVG_SMALL_ROUND_BYTES overrides it.
    SMALL_ROUND_BYTES = int(os.environ.get("FEDAVG_SMALL_ROUND_BYTES", str(4 << 20)))

    def _reduce_small_round(self, table: KeyTable, ptrs, weights):
        """One native call for a small fp32-only round (see SMALL_ROUND_BYTES)."""
        import numpy as np

        g = table.groups[torch.float32]
        K, dev = ptrs.shape[0], self.device
        lib = _lib.load()
        t0 = time.perf_counter()
        with torch.cuda.device(dev):
            compute = torch.cuda.current_stream(dev)
            if self._copy_stream is not None:
                compute.wait_stream(self._copy_stream)  # earlier users of the staging are done
            st = self._staging_for(g.dtype, K, g.ld)
            st._w_done.synchronize()  # the native call rewrites w_host: an async device round may still read it
            items = table.pack_items(g, ptrs, 0, g.ld)
            w64 = np.array([float(w) for w in weights], dtype=np.float64)
            out_dev = torch.empty(g.P, dtype=torch.float32, device=dev)
            out_host = torch.empty(g.P, dtype=torch.float32, pin_memory=True)
            _lib.check(lib.fedavg_round_f32(items.ctypes.data, items.shape[0], st.host.data_ptr(), st.dev.data_ptr(),
                                            K, g.P, g.ld, w64.ctypes.data, st.w_host.data_ptr(), st.w_dev.data_ptr(),
                                            out_dev.data_ptr(), out_host.data_ptr(), max(1, torch.get_num_threads()),
                                            compute.cuda_stream), "fedavg_round_f32")
        self._last = {"table": table, "K": K, "dev": {torch.float32: (st.dev[:K], out_dev)}}
        results = table.unpack(g, out_host)
        self.last_profile = {"pack_issue_ms": 0.0, "h2d_kernel_d2h_ms": (time.perf_counter() - t0) * 1e3}
        ext = layout_collect_ext()
        if ext is not None and hasattr(ext, "small_round"):
            import ctypes

            es = g.keys
            self._fast_small = {
                "ext": ext, "table": table, "st": st, "names": [e.name for e in es],
                "numel": [int(e.numel) for e in es], "offset": [int(e.offset) for e in es],
                "kind": [int(k) for k in g.kind], "shapes": [tuple(int(d) for d in e.shape) for e in es],
                "fn": ctypes.cast(lib.fedavg_round_f32, ctypes.c_void_p).value,
                "threads": max(1, torch.get_num_threads()),
            }
        return results

    def _small_round_native(self, w_locals, fast):
        """The next small round with the same key table, host side in ONE
        native call (fedavg_collect_ext.small_round): weights, the walk over
        every client's tensors, packing, fedavg_round_f32 and the result views
        written into ``w_locals[0][1]``.  Returns that dict, or None when the
        round needs the general path (it then raises or handles whatever the
        native walk refused -- nothing has been written)."""
        table, st = fast["table"], fast["st"]
        K = len(w_locals)
        g = table.groups[torch.float32]
        if K > st.K or K * g.ld * 4 > self.SMALL_ROUND_BYTES or self._session_open():
            return None
        t0 = time.perf_counter()
        with self._lock:
            stream = torch.cuda.current_stream(self.device).cuda_stream
            status, out_dev, out_host = fast["ext"].small_round(
                w_locals, fast["names"], table._template, fast["numel"], fast["offset"], fast["kind"],
                fast["shapes"], g.P, g.ld, st.host.data_ptr(), st.dev.data_ptr(), st.w_host.data_ptr(),
                st.w_dev.data_ptr(), fast["fn"], fast["threads"], stream, self.device.index)
        if status == 1:
            return None
        _lib.check(status, "fedavg_round_f32")
        # the whole round is one native call (walk, pack, H2D, reduce, D2H, views)
        self.last_profile = {"pack_issue_ms": 0.0, "h2d_kernel_d2h_ms": (time.perf_counter() - t0) * 1e3}
        acc = w_locals[0][1]
        self.fast_rounds += 1
        self._last = {"table": table, "K": K, "dev": {torch.float32: (st.dev[:K], out_dev)}}
        try:
            self._last["refs"] = [weakref.ref(sd) for _, sd in w_locals]
            self._last["acc"] = weakref.ref(acc)
        except TypeError:  # plain dicts cannot be weakly referenced: no reuse
            self._last.pop("dev", None)
        return acc

    def _session_open(self) -> bool:
        sess = self._session() if self._session is not None else None
        return sess is not None and not sess._finished

    def _reduce_groups(self, table: KeyTable, ptrs, weights) -> "OrderedDict[str, torch.Tensor]":
        K = ptrs.shape[0]
        if (len(table.groups) == 1 and torch.float32 in table.groups
                and K * table.groups[torch.float32].ld * 4 <= self.SMALL_ROUND_BYTES):
            return self._reduce_small_round(table, ptrs, weights)
        dev = self.device
        lib = _lib.load()
        threads = max(1, torch.get_num_threads())
        results: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        with torch.cuda.device(dev):
            compute = torch.cuda.current_stream(dev)
            copy_s = self._copy_stream_for()
            copy_s.wait_stream(compute)  # earlier users of the device staging are done
            t0 = time.perf_counter()
            staged = []
            for g in table.groups.values():
                st = self._staging_for(g.dtype, K, g.ld)
                host, devbuf = st.host[:K], st.dev[:K]
                esize = host.element_size()
                rows = max(1, min(K, self.CHUNK_BYTES // max(1, g.ld * esize)))
                for i0 in range(0, K, rows):
                    i1 = min(K, i0 + rows)
                    items = table.pack_items(g, ptrs[i0:i1], i0, g.ld)
                    _lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], host.data_ptr(), esize,
                                                    threads), "fedavg_pack_rows")
                    with torch.cuda.stream(copy_s):
                        devbuf[i0:i1].copy_(host[i0:i1], non_blocking=True)
                w_dev = st.upload_weights(weights, copy_s)
                staged.append((g, devbuf, w_dev))
            compute.wait_stream(copy_s)
            t1 = time.perf_counter()
            outs = []
            self._last = {"table": table, "K": K, "dev": {}, "sumsq": {}}
            d2h = self._d2h_stream_for()
            for g, devbuf, w_dev in staged:
                out_dev, out_host = reduce_and_fetch(devbuf, w_dev, g.P, d2h, sums=self._last["sumsq"])
                outs.append((g, out_host))
                self._last["dev"][g.dtype] = (devbuf, out_dev)
            # the D2H stream waited on the compute stream after every chunk's
            # reduce, so its completion covers the kernels too
            d2h.synchronize()
            t2 = time.perf_counter()
        results = _Flats(outs)
        self.last_profile = {"pack_issue_ms": (t1 - t0) * 1e3, "h2d_kernel_d2h_ms": (t2 - t1) * 1e3}
        return results


    # ------------------------------------------------------------------
    def client_distances(self, w_locals, w_glob) -> "np.ndarray":
        """``[torch.norm(cat(w[k] - w_glob[k])).item() for _, w in w_locals]``
        (fedavg_trainer.py:291) on the GPU.

        Reuses the client rows and the averaged model left in HBM by the last
        ``aggregate`` when called with that round's ``w_locals``/``w_glob``
        (the reference's order: :217 then :291); otherwise uploads them.
        A client whose dict IS ``w_glob`` (client 0 after aggregate, :449)
        gets ``w_glob - w_glob``: 0.0, or NaN where ``w_glob`` holds inf/NaN.

        Every dtype group of the state_dict (fp32 with the integer keys,
        fp64, fp16, bf16) is one pass: the difference rounded in the group's
        dtype as ``w[para] - w_glob[para]`` rounds it, squares summed in fp64;
        the groups' sums are added and the root is rounded to torch.cat's
        promoted dtype (fp64 if any fp64 key; fp32 for fp32 or mixed 16-bit
        kinds; fp16/bf16 when every key is that type).  The reference's norm
        accumulates in its own dtype's SIMD lanes; this is the accurate value
        it approximates.
        """
        import numpy as np

        if not w_locals:
            return np.zeros(0)
        last = self._last
        refs = last.get("refs")
        devs = last.get("dev", {})
        cached = (refs is not None and last["acc"]() is w_glob and len(refs) == len(w_locals)
                  and all(r() is sd for r, (_, sd) in zip(refs, w_locals))
                  and bool(devs) and set(devs) == set(last["table"].groups)
                  and all(rows is not None or dt == torch.float32 for dt, (rows, _) in devs.items()))
        # the reference's `w[para] - w_glob[para]` raises on bool buffers; the
        # round's key table already holds every client's (validated) dtypes
        if cached:
            t = last["table"]
            has_bool = t.__dict__.get("_has_bool")
            if has_bool is None:
                has_bool = t._has_bool = any(e.src_dtype == torch.bool for e in t.entries)
        else:
            has_bool = any(t.dtype == torch.bool for _, sd in w_locals if sd is not w_glob for t in sd.values())
        if has_bool and any(sd is not w_glob for _, sd in w_locals):
            raise RuntimeError("Subtraction, the `-` operator, with a bool tensor is not supported "
                               "(fedavg_trainer.py:291 on a state_dict with bool buffers)")
        with torch.cuda.device(self.device):
            parts = []  # (group dtype, [K] fp64 sums on the device, the group's averaged model)
            if cached:
                table = last["table"]
                fused = last.get("sumsq") or {}
                for dt, (devbuf, out_dev) in devs.items():
                    P = table.groups[dt].P
                    if dt in fused:  # formed by the aggregate's own pass over the rows
                        parts.append((dt, fused[dt], out_dev[:P]))
                    elif devbuf is None:  # zero-copy round: read the clients' tensors where they lie
                        # the dict aliased to w_glob (client 0, :449) holds the average
                        # now; its own tensors stand in (its norm is overridden below)
                        keep0 = self._client0_tensors(last)
                        dicts = [keep0 if sd is w_glob else sd for _, sd in w_locals]
                        parts.append((dt, self._sqdist_segments(table, dicts, out_dev), out_dev[:P]))
                    else:
                        parts.append((dt, client_sqdist(devbuf, out_dev, P), out_dev[:P]))
            else:
                for dt, devbuf, glob, P in self._upload_for_distances(w_locals, w_glob):
                    parts.append((dt, client_sqdist(devbuf, glob, P), glob[:P]))
            sumsq_dev = parts[0][1]
            for _, s, _ in parts[1:]:
                sumsq_dev = sumsq_dev + s
            sumsq = sumsq_dev.cpu().numpy()
            glob_finite = all(bool(torch.isfinite(g).all()) for _, _, g in parts)
        cat_dtype = parts[0][0]
        for dt, _, _ in parts[1:]:
            cat_dtype = torch.promote_types(cat_dtype, dt)
        norms = _round_to_dtype(np.sqrt(sumsq), cat_dtype)
        for i, (_, sd) in enumerate(w_locals):
            if sd is w_glob:
                norms[i] = 0.0 if glob_finite else float("nan")
        return norms

    def _upload_for_distances(self, w_locals, w_glob):
        """[(dtype, rows [K, ld], glob [ld], P)] per dtype group: the clients'
        rows and the model, packed in HBM (on the device from device-resident
        tensors, else through pinned host staging)."""
        others = [sd for _, sd in w_locals if sd is not w_glob]
        template = others[0] if others else w_glob
        table = KeyTable(template)
        gtable = KeyTable(w_glob)
        if set(table.groups) != set(gtable.groups) or any(
                table.groups[dt].P != gtable.groups[dt].P for dt in table.groups):
            raise ValueError("w_glob's keys/dtypes do not match the clients' (fedavg_trainer.py:291 subtracts "
                             "w_glob[para] key by key; pass the aggregate's result)")
        K = len(w_locals)
        rows = [sd if sd is not w_glob else template for _, sd in w_locals]  # aliased rows are overridden
        cdev = self._client_device(table, rows)
        ptrs, keep = table.collect(rows, cdev)
        gptrs, gkeep = gtable.collect([w_glob], cdev)  # w - w_glob needs one device (TypeError otherwise)
        out = []
        if cdev.type == "cuda":
            stream = torch.cuda.current_stream(self.device)
            for dt, g in table.groups.items():
                gg = gtable.groups[dt]
                dev = torch.empty((K + 1, g.ld), dtype=dt, device=self.device)
                self._pack_on_device(table, g, ptrs, 0, dev, stream)
                self._pack_on_device(gtable, gg, gptrs, K, dev, stream)
                out.append((dt, dev[:K], dev[K], g.P))
            del keep, gkeep
            return out
        lib = _lib.load()
        for dt, g in table.groups.items():
            gg = gtable.groups[dt]
            host = torch.empty((K + 1, g.ld), dtype=dt, pin_memory=True)
            es = host.element_size()
            items = table.pack_items(g, ptrs, 0, g.ld)
            _lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], host.data_ptr(), es,
                                            max(1, torch.get_num_threads())), "fedavg_pack_rows")
            gitems = gtable.pack_items(gg, gptrs, K, g.ld)
            _lib.check(lib.fedavg_pack_rows(gitems.ctypes.data, gitems.shape[0], host.data_ptr(), es, 1),
                       "fedavg_pack_rows")
            dev = host.to(self.device, non_blocking=True)
            out.append((dt, dev[:K], dev[K], g.P))
        torch.cuda.current_stream(self.device).synchronize()
        del keep, gkeep
        return out


def _round_to_dtype(x, dtype: torch.dtype):
    """float64 array -> the values rounded to ``dtype`` (what ``.item()`` of
    a norm of that dtype returns), as float64."""
    import numpy as np

    if dtype == torch.float64:
        return np.asarray(x, dtype=np.float64).copy()
    return torch.from_numpy(np.asarray(x, dtype=np.float64)).to(dtype).to(torch.float64).numpy()


def client_arena(template, K: int, device=None):
    """K device state_dicts shaped like ``template`` whose tensors are views
    into ONE ``[K, ld]`` fp32 buffer in the aggregate's packed layout (row i
    = client i, keys back to back in ``template``'s order, ``ld`` = the
    row length rounded to 64 elements).  Returns ``(rows, dicts)``.

    A device-resident round whose clients write their results into these
    dicts (``copy_`` into the views, or models whose parameters are these
    views) is reduced by the row kernel straight from ``rows`` -- the
    zero-copy path without per-client allocations (DESIGN.md section 6:
    7.1 TB/s on one buffer against 6.3-6.5 on separately allocated tensors,
    whose address translation costs the difference).  fp32 state_dicts
    only (every key of one dtype group, as the reference's models)."""
    table = KeyTable(template)
    if set(table.groups) != {torch.float32} or any(e.src_dtype != torch.float32 for e in table.entries):
        raise TypeError("client_arena holds fp32 state_dicts (every key fp32)")
    g = table.groups[torch.float32]
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    rows = torch.zeros((K, g.ld), dtype=torch.float32, device=device)
    dicts = []
    for i in range(K):
        sd = OrderedDict()
        for e in table.entries:
            sd[e.name] = rows[i, e.offset:e.offset + e.numel].view(e.shape)
        dicts.append(sd)
    return rows, dicts


_default: Dict[int, DeviceAggregator] = {}
_default_lock = threading.Lock()


def default_aggregator(device: Optional[torch.device] = None) -> DeviceAggregator:
    if device is None:
        if not torch.cuda.is_available():
            raise _lib.FedAvgLibraryError("no HIP device visible: the FedAvg reduction has no CPU fallback")
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with _default_lock:
        agg = _default.get(idx)
        if agg is None:
            agg = DeviceAggregator(torch.device("cuda", idx))
            _default[idx] = agg
    return agg


def _devices_arg(device, devices):
    """The device list a functional call routes to: ``devices`` when given,
    else FEDAVG_DEVICES when no single ``device`` was named; None = one GPU
    (``_single_device`` names it)."""
    if devices is None and device is None:
        from .multi import devices_from_env

        devices = devices_from_env()
    if devices is not None and len(devices) > 1:
        return list(devices)
    return None


def _single_device(device, devices):
    """The one GPU a call runs on when ``_devices_arg`` gives no list: ``device``,
    else the single entry of ``devices`` / FEDAVG_DEVICES, else None (the
    current device, or where device-resident clients lie)."""
    if device is not None:
        return device
    if devices is None:
        from .multi import devices_from_env

        devices = devices_from_env()
    if devices is not None and len(devices) == 1:
        from .multi import normalize_device

        return normalize_device(devices[0])
    return None


def aggregate(w_locals, model_global=None, device: Optional[torch.device] = None, devices=None):
    """Functional form of ``FedAvgTrainer.aggregate``.  ``devices`` (or
    FEDAVG_DEVICES=0,1,...): host rounds split by columns over those GPUs,
    each over its own PCIe link (multi.ShardedAggregator, same bits)."""
    done, answer = _trivial(w_locals, model_global)
    if done:
        return answer  # answered on the host: no GPU needed
    devs = _devices_arg(device, devices)
    if devs is not None:
        from .multi import sharded_aggregator

        return sharded_aggregator(devs).aggregate(w_locals, model_global=model_global)
    device = _single_device(device, devices)
    if device is None:  # device-resident clients are reduced on their own device
        first = next(iter(w_locals[0][1].values()))
        if isinstance(first, torch.Tensor) and first.is_cuda:
            device = first.device
    return default_aggregator(device).aggregate(w_locals, model_global=model_global)


def client_distances(w_locals, w_glob, device: Optional[torch.device] = None, devices=None):
    """Functional form of fedavg_trainer.py:291 (see DeviceAggregator.client_distances)."""
    devs = _devices_arg(device, devices)
    if devs is not None:
        from .multi import sharded_aggregator

        return sharded_aggregator(devs).client_distances(w_locals, w_glob)
    return default_aggregator(_single_device(device, devices)).client_distances(w_locals, w_glob)


def estimate_delta(w_locals, w_glob, lr, device: Optional[torch.device] = None, devices=None):
    """fedavg_trainer.py:289-293: ``sum(n_i * ||w_i - w_glob||) / sum(n_i) / lr``."""
    import numpy as np

    sample_nums = np.array([n for n, _ in w_locals])
    norms = client_distances(w_locals, w_glob, device, devices)
    return np.sum(sample_nums * norms) / np.sum(sample_nums) / lr


class FedAvgAggregateMixin:
    """Mix in ahead of the reference ``FedAvgTrainer`` to run ``aggregate`` on the GPU."""

    fedavg_device: Optional[torch.device] = None

    def aggregate(self, w_locals):  # fedavg_trainer.py:441
        return aggregate(w_locals, getattr(self, "model_global", None), self.fedavg_device)


def _feed_of(trainer):
    """The trainer's ClientFeed (autostream), created on first use.  Its
    rounds stream into the installed device's DeviceAggregator, or -- with
    ``install(devices=[...])`` / FEDAVG_DEVICES -- into the devices'
    ShardedAggregator (every client's column shards over every device's link)."""
    from .autostream import ClientFeed

    feed = trainer.__dict__.get("_mfl_feed")
    if feed is None:
        cls = type(trainer)
        device = getattr(cls, "_mfl_stream_device", None)
        devs = getattr(cls, "_mfl_stream_devices", None)
        clients = getattr(trainer, "client_list", None)  # fedavg_trainer.py:88: the Client objects of a round
        max_clients = len(clients) if clients else 128
        if devs is not None:
            from .multi import sharded_aggregator

            feed = ClientFeed(lambda: sharded_aggregator(devs), max_clients)
        else:
            feed = ClientFeed(lambda: default_aggregator(device), max_clients)
        trainer.__dict__["_mfl_feed"] = feed
    return feed


def stream_distinct_ok(devs) -> bool:
    """Whether ``install(devices=devs)`` streams: always for one distinct
    device (N shards on one GPU, the rehearsed form); for several distinct
    GPUs only with ``FEDAVG_STREAM_DISTINCT_DEVICES=1`` -- streaming over
    distinct devices (several DMA engines reading one pinned staging block,
    per-device event waits, one pinned output filled by several D2H streams)
    is parity-unpinned until a multi-GPU node runs tests/test_gpu_multi.py."""
    from .multi import normalize_device

    if len({normalize_device(d) for d in devs}) <= 1:
        return True
    return os.environ.get("FEDAVG_STREAM_DISTINCT_DEVICES", "0") == "1"


def install(trainer_cls, device: Optional[torch.device] = None, client_cls=None, stream_clients: Optional[bool] = None,
            devices=None):
    """Patch ``trainer_cls.aggregate`` (e.g. the reference ``FedAvgTrainer``) in place.

    With ``stream_clients`` (default: on unless ``FEDAVG_STREAM_CLIENTS=0``)
    also wrap ``trainer_cls.train`` (the round loop, fedavg_trainer.py:95) and
    ``client_cls.train`` (client.py:38; default: the ``Client`` that
    ``trainer_cls``'s module imported) so each valid client result is packed
    and uploaded while the loop goes on, and ``aggregate`` at :217 only
    reduces (autostream.py; falls back to the plain path whenever
    ``w_locals`` is not what was streamed).

    ``devices`` (or FEDAVG_DEVICES=0,1,... when ``device`` is None): host
    rounds run over those GPUs by columns, one PCIe link each, with the
    single-GPU bits (multi.ShardedAggregator).  Streaming over them
    (multi.ShardedRoundSession: each client's column shards uploaded to every
    device as it arrives) has only run as same-GPU rehearsals, so a list of
    DISTINCT devices streams only with ``FEDAVG_STREAM_DISTINCT_DEVICES=1``;
    otherwise its rounds take the plain sharded path at :217.

    GPU initialisation is eager: install() creates every listed device's
    streams and runs each first-use kernel and copy once (warm_up), before
    the loop's round 0, so fork the process, if at all, before install().
    ``FEDAVG_WARMUP=0`` leaves that to the first round."""
    from . import autostream

    if stream_clients is None:
        stream_clients = autostream.enabled()
    if client_cls is None:
        import sys

        client_cls = getattr(sys.modules.get(trainer_cls.__module__), "Client", None)
    streaming = bool(stream_clients) and client_cls is not None and hasattr(trainer_cls, "train")
    # install() may run again (another device, streaming switched off): the
    # wrappers below are installed once and read these per-class settings on
    # every call, so a later install(stream_clients=False) stops the feed
    # instead of leaving wrappers that upload clients nobody reduces
    devs = _devices_arg(device, devices)
    if devs is None:
        device = _single_device(device, devices)  # install(devices=[3]) runs on cuda:3
    elif streaming and not stream_distinct_ok(devs):
        streaming = False  # plain sharded rounds (multi.ShardedAggregator) until distinct GPUs have run it
    trainer_cls._mfl_stream_on = streaming
    trainer_cls._mfl_stream_device = device
    trainer_cls._mfl_stream_devices = devs
    if torch.cuda.is_available() and DeviceAggregator.WARMUP:  # the HIP first-use costs, before round 0
        for d in (devs or [device]):
            default_aggregator(d).warm_up()
        if devs is not None:
            from .multi import sharded_aggregator

            sharded_aggregator(devs)  # the shards' streams

    def aggregate_method(self, w_locals):
        feed = self.__dict__.get("_mfl_feed") if streaming else None
        if feed is not None and autostream.active_trainer() is self:
            out = feed.take(w_locals)
            if out is not None:
                return out
        return aggregate(w_locals, getattr(self, "model_global", None), device, devs)

    aggregate_method.__doc__ = FedAvgAggregateMixin.aggregate.__doc__
    aggregate_method.__wrapped_reference__ = getattr(trainer_cls, "aggregate", None)
    trainer_cls.aggregate = aggregate_method
    if not streaming or getattr(trainer_cls.train, "__mfl_stream__", False):
        return trainer_cls
    loop = trainer_cls.train

    def train_method(self, *args, **kwargs):  # fedavg_trainer.py:95, the round loop
        if not getattr(type(self), "_mfl_stream_on", False):
            return loop(self, *args, **kwargs)
        with autostream.trainer_scope(self):
            return loop(self, *args, **kwargs)

    train_method.__doc__ = loop.__doc__
    train_method.__mfl_stream__ = True
    train_method.__wrapped_reference__ = loop
    trainer_cls.train = train_method
    if not getattr(client_cls.train, "__mfl_stream__", False):
        client_train = client_cls.train

        def client_train_method(self, *args, **kwargs):  # client.py:38
            res = client_train(self, *args, **kwargs)
            trainer = autostream.active_trainer()
            if trainer is None or not getattr(type(trainer), "_mfl_stream_on", False):
                return res
            if getattr(type(self), "train", None) is not client_train_method:
                # a Client subclass overrides train() (and reached this one
                # through super()): what it returns to the loop may differ
                # from `res` -- nothing of this round is streamed
                _feed_of(trainer).refuse(
                    "Client.train is overridden by a subclass")
                return res
            if autostream.valid_train_result(res):  # fedavg_trainer.py:190
                _feed_of(trainer).feed(
                    self.get_sample_number(), res[0])
            return res

        client_train_method.__doc__ = client_train.__doc__
        client_train_method.__mfl_stream__ = True
        client_train_method.__wrapped_reference__ = client_train
        client_cls.train = client_train_method
    return trainer_cls
