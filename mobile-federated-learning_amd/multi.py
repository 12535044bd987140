"""One process, several GPUs: the drop-in's host path over N PCIe links.

The reference drives ``aggregate`` from one process (main_fedavg.py:337-338,
fedavg_trainer.py:217) with host state_dicts in and a host state_dict out
(client.py:96, :219).  On one GPU that round is bound by one PCIe link:
100 clients x 25M fp32 = 10 GB of rows at ~56 GB/s.
SURVEY.md section 8e's host-consumer form needs no collective: every output
column depends only on the same column of the K clients
(fedavg_trainer.py:451-457), so

* the K client rows are packed once into pinned host staging (the native
  packer, row chunks of ``CHUNK_BYTES``);
* GPU d takes the contiguous column shard ``[c_d, c_{d+1})`` of every row
  with ONE strided DMA per row chunk over ITS OWN PCIe link
  (``fedavg_upload_shard`` = hipMemcpy2DAsync: height = rows, width = the
  shard, source pitch = the staging row), overlapped with the packing of the
  next row chunk;
* each GPU reduces its shard with the exact sequential kernel (same bits as
  one GPU: a column's chain is the same wherever it runs) -- fused with the
  :291 sums of squares where the single-GPU path fuses them -- and copies its
  finished columns straight to their global positions in the one pinned
  output buffer, whose key views become ``w_locals[0][1]``'s values.

The streamed form (``begin_round`` -> :class:`ShardedRoundSession`, what
``install(devices=[...])``'s zero-edit feed uses) does the same per client as
it arrives: the client is packed once into its pinned row, and every device's
column shard of that row goes over that device's own link while the loop
trains the next client; at :217 each device reduces its shard and copies it
to its global positions (N kernels on N/8 of the bytes, N D2Hs of P/N).

Rounds the extra links cannot help are handed to the first device's
``DeviceAggregator`` unchanged: small rounds (one native call,
``SMALL_ROUND_BYTES``) and device-resident clients (reduced where they lie),
streamed or not.  ``client_distances`` (:291) after a sharded round, streamed
or plain, adds the per-device fp64 sums of squares in device order.

Only same-device rehearsals (N shards on one GPU) have run on hardware: the
pinned staging read by N devices' DMA engines, cross-device stream ordering
and the per-link rates are parity-unpinned on distinct GPUs until a
multi-GPU node runs tests/test_gpu_multi.py (its distinct-device test skips
on fewer than 2 visible GPUs).

Use: ``mfl_amd.install(FedAvgTrainer, devices=[0, 1, ..., 7])``,
``FEDAVG_DEVICES=0,1,...,7 python -m mfl_amd.launch main_fedavg.py ...`` or
``mfl_amd.sharded_aggregator([0, 1, ...]).aggregate(w_locals)``.  The same
device may appear more than once (tests rehearse N shards on one GPU).
"""
from __future__ import annotations

import os
import threading
import time
import weakref
from collections import OrderedDict
from typing import List, Optional, Sequence

import torch

from . import _lib
from .distributed import upload_segments
from .layout import KeyTable
from .reduce import ALIGN_ELEMS, client_sqdist
from .session import RoundSession

__all__ = ["ShardedAggregator", "ShardedRoundSession", "sharded_aggregator", "shard_bounds", "devices_from_env",
           "normalize_device"]


def shard_bounds(P: int, n: int, align: int = ALIGN_ELEMS) -> List[int]:
    """Column boundaries ``[c_0 = 0, c_1, ..., c_n = P]`` of n contiguous
    shards; every interior boundary a multiple of ``align`` (a shard's rows
    then start 256-B aligned in HBM and its host source 256-B aligned in the
    staging row).  Shards may be empty when P is small."""
    if n < 1:
        raise ValueError("need at least one shard")
    bounds = [0]
    for d in range(1, n):
        b = -(-P * d // n)
        bounds.append(min(P, -(-b // align) * align))
    bounds.append(P)
    return bounds


def devices_from_env() -> Optional[List[torch.device]]:
    """``FEDAVG_DEVICES=0,1,2,3`` -> those HIP devices (None when unset)."""
    v = os.environ.get("FEDAVG_DEVICES", "").strip()
    if not v:
        return None
    return [torch.device("cuda", int(t)) for t in v.split(",") if t.strip()]


class _Shard:
    """One device's part: its column range, rows buffer, weights and streams."""

    def __init__(self, device: torch.device):
        from .aggregate import _Weights

        self.device = device
        self.copy = torch.cuda.Stream(device)
        self.d2h = torch.cuda.Stream(device)
        self.rows = {}  # dtype -> [K, ld_d] device buffer
        self.weights = {}  # weight dtype -> _Weights
        self._Weights = _Weights

    def rows_for(self, dtype, K, cols):
        ld = max(-(-cols // ALIGN_ELEMS) * ALIGN_ELEMS, ALIGN_ELEMS)
        buf = self.rows.get(dtype)
        if buf is None or buf.shape[0] < K or buf.shape[1] != ld:
            buf = torch.empty((K, ld), dtype=dtype, device=self.device)
            self.rows[dtype] = buf
        return buf[:K]

    def weights_for(self, dtype, K):
        wdt = torch.float64 if dtype == torch.float64 else torch.float32
        w = self.weights.get(wdt)
        if w is None or w.K < K:
            w = self._Weights(K, wdt, self.device)
            self.weights[wdt] = w
        return w


class ShardedAggregator:
    """``FedAvgTrainer.aggregate`` over several GPUs (module docstring)."""

    CHUNK_BYTES = int(os.environ.get("FEDAVG_CHUNK_BYTES", str(32 << 20)))
    SMALL_ROUND_BYTES = None  # rounds up to this many row bytes stay on one device (None: DeviceAggregator's)

    def __init__(self, devices: Sequence):
        if not devices:
            raise ValueError("ShardedAggregator needs at least one device")
        self.devices = [normalize_device(d) for d in devices]
        self._shards = [_Shard(d) for d in self.devices]
        self._host = {}  # dtype -> pinned [K, ld] staging
        self._lock = threading.Lock()
        self._table_hint = None
        self._last = {}
        self.last_profile = {}
        self.rounds_sharded = 0
        self.rounds_delegated = 0
        self.rounds_streamed = 0  # ShardedRoundSession rounds finished
        self._session = None  # weakref to the open ShardedRoundSession, if any

    @property
    def primary(self):
        from .aggregate import default_aggregator

        return default_aggregator(self.devices[0])

    def begin_round(self, template, max_clients: int):
        """Start a streaming round over the devices (:class:`ShardedRoundSession`:
        each added client is packed once and its column shards go over every
        device's own link as it arrives).  Rounds the extra links cannot help
        get the first device's ``RoundSession``: one device, small rounds
        (``SMALL_ROUND_BYTES``: one native call) and device-resident clients."""
        from .layout import KeyTable

        self._check_no_open_session("begin_round")
        first = next(iter(template.values()), None) if len(template) else None
        on_device = isinstance(first, torch.Tensor) and first.is_cuda
        small = self.primary.SMALL_ROUND_BYTES if self.SMALL_ROUND_BYTES is None else self.SMALL_ROUND_BYTES
        row_bytes = sum(v.numel() * max(4, v.element_size()) for v in template.values()
                        if isinstance(v, torch.Tensor))
        if len(self.devices) == 1 or on_device or max_clients * row_bytes <= small:
            self.rounds_delegated += 1
            return self.primary.begin_round(template, max_clients)
        sess = ShardedRoundSession(self, KeyTable(template), max_clients)
        self._session = weakref.ref(sess)
        return sess

    def _check_no_open_session(self, what: str):
        sess = self._session() if self._session is not None else None
        if sess is not None and not sess._finished:
            raise RuntimeError(f"{what}: a ShardedRoundSession on these devices is still open (call finish first)")

    # ------------------------------------------------------------------
    def aggregate(self, w_locals, model_global=None):
        from .aggregate import _Prepared, _trivial, prepare

        done, answer = _trivial(w_locals, model_global)
        if done:
            return answer  # empty list / no keys: answered on the host
        sd0 = w_locals[0][1]
        first = next(iter(sd0.values()))
        if isinstance(first, torch.Tensor) and first.is_cuda:
            # device-resident clients are reduced where they lie (zero-copy)
            from .aggregate import default_aggregator

            self.rounds_delegated += 1
            return default_aggregator(first.device).aggregate(w_locals, model_global)
        row_bytes = sum(v.numel() * max(4, v.element_size()) for v in sd0.values() if isinstance(v, torch.Tensor))
        small = self.primary.SMALL_ROUND_BYTES if self.SMALL_ROUND_BYTES is None else self.SMALL_ROUND_BYTES
        if len(self.devices) == 1 or len(w_locals) * row_bytes <= small:
            # a small round is one native call on one device (fedavg_round_f32)
            self.rounds_delegated += 1
            return self.primary.aggregate(w_locals, model_global)
        prep = prepare(w_locals, model_global, self._table_hint)
        if not isinstance(prep, _Prepared):
            return prep
        self._check_no_open_session("aggregate")  # a session owns the staging until it finishes
        acc_dict, table, dicts, weights, ptrs, keepalive = prep
        self._table_hint = table
        if table.client_device(dicts).type == "cuda":  # mixed placement: the primary raises the reference's error
            del keepalive
            return self.primary.aggregate(w_locals, model_global)
        with self._lock:
            results = self._reduce_sharded(table, ptrs, weights)
        del keepalive
        table.forget_tensors()
        try:
            self._last["refs"] = [weakref.ref(sd) for sd in dicts]
            self._last["acc"] = weakref.ref(acc_dict)
        except TypeError:
            self._last = {}
        for e in table.entries:
            acc_dict[e.name] = results[e.name]
        self.rounds_sharded += 1
        return acc_dict

    def _host_for(self, dtype, K: int, ld: int) -> torch.Tensor:
        """The pinned ``[>=K, ld]`` host staging of a dtype group (kept across rounds)."""
        host = self._host.get(dtype)
        if host is None or host.shape[0] < K or host.shape[1] != ld:
            host = None
            self._host.pop(dtype, None)  # free the old block before pinning the new one
            host = torch.empty((K, ld), dtype=dtype, pin_memory=True)
            self._host[dtype] = host
        return host

    def _reduce_sharded(self, table: KeyTable, ptrs, weights):
        from .aggregate import _fetch, reduce_rows

        lib = _lib.load()
        K = ptrs.shape[0]
        n = len(self._shards)
        threads = max(1, torch.get_num_threads())
        t0 = time.perf_counter()
        for sh in self._shards:  # earlier users of the shard's rows are done
            sh.copy.wait_stream(torch.cuda.current_stream(sh.device))
        plan = []
        for g in table.groups.values():
            es = _elem(g.dtype)
            host = self._host_for(g.dtype, K, g.ld)[:K]
            bounds = shard_bounds(g.P, n)
            rows = [sh.rows_for(g.dtype, K, bounds[d + 1] - bounds[d]) for d, sh in enumerate(self._shards)]
            step = max(1, min(K, self.CHUNK_BYTES // max(1, g.ld * es)))
            for i0 in range(0, K, step):
                i1 = min(K, i0 + step)
                items = table.pack_items(g, ptrs[i0:i1], i0, g.ld)
                _lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], host.data_ptr(), es, threads),
                           "fedavg_pack_rows")
                for d, sh in enumerate(self._shards):  # each device's columns over its own link
                    c0, c1 = bounds[d], bounds[d + 1]
                    if c1 > c0:
                        with torch.cuda.device(sh.device):
                            upload_segments(rows[d][i0:i1], host[i0:i1], [(0, c0, c1 - c0)], sh.copy)
            plan.append((g, bounds, rows))
        t1 = time.perf_counter()
        outs = []
        per_dev = [dict() for _ in self._shards]
        for g, bounds, rows in plan:
            out_host = torch.empty(g.P, dtype=g.dtype, pin_memory=True)
            for d, sh in enumerate(self._shards):
                c0, c1 = bounds[d], bounds[d + 1]
                if c1 <= c0:
                    continue
                with torch.cuda.device(sh.device):
                    compute = torch.cuda.current_stream(sh.device)
                    compute.wait_stream(sh.copy)
                    w_dev = sh.weights_for(g.dtype, K).upload(weights, compute)
                    out_dev = torch.empty(c1 - c0, dtype=g.dtype, device=sh.device)
                    sums = []
                    reduce_rows(rows[d], w_dev, c1 - c0, out_dev, sums)
                    sh.d2h.wait_stream(compute)
                    _fetch(out_dev, out_host[c0:c1], sh.d2h)
                    per_dev[d][g.dtype] = (rows[d], out_dev, sums[0] if sums else None, c0, c1)
            outs.append((g, out_host))
        for sh in self._shards:
            sh.d2h.synchronize()
        t2 = time.perf_counter()
        results = OrderedDict()
        for g, out_host in outs:
            results.update(table.unpack(g, out_host))
        self._last = {"table": table, "K": K, "per_dev": per_dev}
        self.last_profile = {"pack_and_h2d_issue_ms": (t1 - t0) * 1e3, "reduce_d2h_wait_ms": (t2 - t1) * 1e3,
                             "shards": n}
        return results

    # ------------------------------------------------------------------
    def client_distances(self, w_locals, w_glob):
        """fedavg_trainer.py:291 after a sharded round: every device's fp64
        sums of squares of its columns (fused into the aggregate's pass, or
        one client_sqdist pass over its rows), added in device order; other
        calls go to the first device's DeviceAggregator."""
        import numpy as np

        from .aggregate import _round_to_dtype

        last = self._last
        refs = last.get("refs")
        cached = (refs is not None and last["acc"]() is w_glob and len(refs) == len(w_locals)
                  and all(r() is sd for r, (_, sd) in zip(refs, w_locals)))
        if not cached or not w_locals:
            return self.primary.client_distances(w_locals, w_glob)
        table = last["table"]
        if any(e.src_dtype == torch.bool for e in table.entries) and any(sd is not w_glob for _, sd in w_locals):
            raise RuntimeError("Subtraction, the `-` operator, with a bool tensor is not supported "
                               "(fedavg_trainer.py:291 on a state_dict with bool buffers)")
        total = np.zeros(len(w_locals), dtype=np.float64)
        glob_finite = True
        for d, parts in enumerate(last["per_dev"]):
            for dt, (rows, out_dev, sums, c0, c1) in parts.items():
                with torch.cuda.device(out_dev.device):
                    s = sums if sums is not None else client_sqdist(rows, out_dev, c1 - c0)
                    total += s.cpu().numpy()
                    glob_finite = glob_finite and bool(torch.isfinite(out_dev).all())
        cat_dtype = None
        for dt in table.groups:
            cat_dtype = dt if cat_dtype is None else torch.promote_types(cat_dtype, dt)
        norms = _round_to_dtype(np.sqrt(total), cat_dtype)
        for i, (_, sd) in enumerate(w_locals):
            if sd is w_glob:
                norms[i] = 0.0 if glob_finite else float("nan")
        return norms


class _HostRows:
    """A group's pinned staging rows, as RoundSession's ``_staging[dtype].host``
    (what autostream's verify_rows compares w_locals against)."""

    def __init__(self, host: torch.Tensor):
        self.host = host


class ShardedRoundSession(RoundSession):
    """A streaming round (session.RoundSession's contract) over N devices.

    ``add`` packs the client ONCE into the pinned host row (the native
    packer) and then issues, for every device d, the H2D of the row's column
    shard ``[c_d, c_{d+1})`` on d's copy stream -- over d's own PCIe link --
    in the column chunks d's finish reduces in, recording an event per chunk.
    ``finish`` forms the weights, and for every device runs the reduce of its
    shard (fused with the :291 sums of squares where the single-GPU finish
    fuses them), each chunk waiting only for its own uploads, and copies the
    finished columns straight to their global positions in the one pinned
    output whose key views become ``w_locals[0][1]``'s values.  Every column
    is reduced by the same sequential kernel over the same K rows as on one
    GPU, so the bits are the single-GPU (and the reference's) bits.

    Host clients only (device-resident and small rounds are the first
    device's RoundSession, ``ShardedAggregator.begin_round``)."""

    def __init__(self, sagg: "ShardedAggregator", table: KeyTable, max_clients: int):
        if max_clients < 1:
            raise ValueError("max_clients must be >= 1")
        from .aggregate import column_chunks

        self.agg = sagg
        self.table = table
        self.max_clients = max_clients
        self.counts = []
        self.dicts = []
        self._keepalive = []
        self._finished = False
        self._verify = None
        self._lib = _lib.load()
        self._threads = max(1, torch.get_num_threads())
        self.finish_profile = {}
        self.add_ms = 0.0
        self.add_profile = {}
        self.keep_dicts = True
        self.defer_release = None
        self._small = False
        self._client_dev = torch.device("cpu")
        shards = sagg._shards
        self.dev = shards[0].device
        for sh in shards:  # earlier users of the shards' rows (a plain round's reduce) are done
            sh.copy.wait_stream(torch.cuda.current_stream(sh.device))
        self._staging = {}
        self._plan = {}  # dtype -> [(shard, c0, c1, rows [max_clients, ld_d], chunks)] for non-empty shards
        self._ready = {}  # dtype -> per plan entry, the latest add's chunk events
        self._out_host = {}
        self._views = {}
        for g in table.groups.values():
            self._staging[g.dtype] = _HostRows(sagg._host_for(g.dtype, max_clients, g.ld))
            bounds = shard_bounds(g.P, len(shards))
            plan = []
            for d, sh in enumerate(shards):
                c0, c1 = bounds[d], bounds[d + 1]
                if c1 > c0:
                    plan.append((sh, c0, c1, sh.rows_for(g.dtype, max_clients, c1 - c0), column_chunks(c1 - c0)))
            self._plan[g.dtype] = plan
            # the result's pinned buffer and its key views, made while clients
            # train instead of inside finish() (session.RoundSession.add)
            self._out_host[g.dtype] = torch.empty(g.P, dtype=g.dtype, pin_memory=True)
            self._views[g.dtype] = table.unpack(g, self._out_host[g.dtype])

    def add(self, sample_num, state_dict) -> None:
        """Pack one host client into its pinned row and start every device's
        shard upload (fedavg_trainer.py:199)."""
        if self._finished:
            raise RuntimeError("session already finished")
        i = len(self.counts)
        if i >= self.max_clients:
            raise ValueError(f"more than max_clients={self.max_clients} clients added")
        t0 = time.perf_counter()
        if self.table.client_device([state_dict]).type != "cpu":
            raise TypeError("a ShardedRoundSession streams host clients (device-resident rounds run where they lie)")
        ptrs, keep = self.table.collect([state_dict], torch.device("cpu"))
        for g in self.table.groups.values():
            host = self._staging[g.dtype].host
            t1 = time.perf_counter()
            items = self.table.pack_items(g, ptrs, i, g.ld)
            _lib.check(self._lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], host.data_ptr(),
                                                  host.element_size(), self._threads), "fedavg_pack_rows")
            t2 = time.perf_counter()
            ready = []
            for sh, c0, c1, rows, chunks in self._plan[g.dtype]:
                events = []
                with torch.cuda.device(sh.device), torch.cuda.stream(sh.copy):
                    for a, b in chunks:  # this device's columns, over its own link
                        rows[i, a:b].copy_(host[i, c0 + a:c0 + b], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(sh.copy)
                        events.append(ev)
                ready.append(events)  # each copy stream is FIFO: covers earlier rows too
            self._ready[g.dtype] = ready
            t3 = time.perf_counter()
            self.add_profile["pack_ms"] = self.add_profile.get("pack_ms", 0.0) + (t2 - t1) * 1e3
            self.add_profile["h2d_issue_ms"] = self.add_profile.get("h2d_issue_ms", 0.0) + (t3 - t2) * 1e3
        del keep
        self.counts.append(sample_num)
        self.dicts.append(state_dict if self.keep_dicts else None)
        self.add_ms += (time.perf_counter() - t0) * 1e3

    def abandon(self) -> None:
        if self._finished:
            return
        self._finished = True
        for sh in self.agg._shards:
            sh.copy.synchronize()
        self._forget_table()

    def finish(self, w_locals=None, verify=None):
        """Reduce the added clients over the devices; ``aggregate``'s contract
        (fedavg_trainer.py:441-458), as RoundSession.finish."""
        if self._finished:
            raise RuntimeError("session already finished")
        self._finished = True
        if w_locals is not None:
            if len(w_locals) != len(self.counts):
                raise ValueError(f"w_locals has {len(w_locals)} clients, session has {len(self.counts)}")
            for i, ((n, sd), n2, sd2) in enumerate(zip(w_locals, self.counts, self.dicts)):
                if (verify is None and sd is not sd2) or n != n2:
                    raise ValueError(f"w_locals[{i}] is not the client added as #{i}")
        if verify is not None and w_locals is not None:
            self.dicts = [sd for _, sd in w_locals]
        if not self.counts:
            raise ValueError("no clients added (the reference returns the global model then: use aggregate([]))")
        K = len(self.counts)
        acc_dict = w_locals[0][1] if w_locals is not None else OrderedDict()
        from .aggregate import reduce_and_fetch, sample_weights

        weights = sample_weights(self.counts)  # ZeroDivisionError like the reference
        per_dev = [dict() for _ in self.agg._shards]
        index = {id(sh): d for d, sh in enumerate(self.agg._shards)}
        t0 = time.perf_counter()
        issue = []
        for g in self.table.groups.values():
            out_host = self._out_host[g.dtype]
            for (sh, c0, c1, rows, _), ready in zip(self._plan[g.dtype], self._ready[g.dtype]):
                issue.append(time.perf_counter())
                with torch.cuda.device(sh.device):
                    cur = torch.cuda.current_stream(sh.device)
                    w_dev = sh.weights_for(g.dtype, K).upload(weights, cur)
                    sums = {}
                    out_dev, _ = reduce_and_fetch(rows[:K], w_dev, c1 - c0, sh.d2h, ready=ready,
                                                  out_host=out_host[c0:c1], sums=sums)
                    per_dev[index[id(sh)]][g.dtype] = (rows[:K], out_dev, sums.get(g.dtype), c0, c1)
        t1 = time.perf_counter()
        ok = self._verify_now(verify)  # overlaps the GPU work just issued
        t_v = time.perf_counter()
        for sh in self.agg._shards:
            with torch.cuda.device(sh.device):
                cur = torch.cuda.current_stream(sh.device)
                sh.d2h.synchronize()
                cur.synchronize()
                cur.wait_stream(sh.copy)  # nothing else may reuse the rows before their copies end
        t2 = time.perf_counter()
        issue.append(t1)
        self.finish_profile = {"issue_ms": (t1 - t0) * 1e3, "verify_ms": (t_v - t1) * 1e3,
                               "wait_ms": (t2 - t_v) * 1e3, "shards": len(self.agg._shards),
                               "issue_ms_per_shard": [round((b - a) * 1e3, 3) for a, b in zip(issue, issue[1:])]}
        if not ok:
            self._forget_table()
            return None
        for g in self.table.groups.values():
            self._set_results(acc_dict, self._views[g.dtype], keys_verified=verify is not None)
        self.finish_profile["unpack_ms"] = (time.perf_counter() - t2) * 1e3
        self._forget_table()
        sagg = self.agg
        sagg._last = {"table": self.table, "K": K, "per_dev": per_dev}
        try:
            sagg._last["refs"] = [weakref.ref(sd) for sd in self.dicts]
            sagg._last["acc"] = weakref.ref(acc_dict)
        except TypeError:
            sagg._last = {}
        sagg.rounds_streamed += 1
        return acc_dict

    @staticmethod
    def _verify_now(verify) -> bool:
        return verify() if verify is not None else True


def normalize_device(d) -> torch.device:
    """``3``, ``"cuda:3"``, ``torch.device("cuda", 3)`` -> ``cuda:3``; a device
    without an index (``"cuda"``) is the current device, as
    ``default_aggregator`` takes it.  HIP devices only (no CPU fallback)."""
    dev = torch.device("cuda", d) if isinstance(d, int) else torch.device(d)
    if dev.type != "cuda":
        raise ValueError(f"{dev}: HIP devices only (no CPU fallback)")
    return torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())


def _elem(dtype: torch.dtype) -> int:
    return torch.empty(0, dtype=dtype).element_size()


_sharded = {}
_sharded_lock = threading.Lock()


def sharded_aggregator(devices: Sequence) -> ShardedAggregator:
    """The process-wide ShardedAggregator for this device list."""
    key = tuple(normalize_device(d).index for d in devices)
    with _sharded_lock:
        agg = _sharded.get(key)
        if agg is None:
            agg = ShardedAggregator(list(key))
            _sharded[key] = agg
    return agg
