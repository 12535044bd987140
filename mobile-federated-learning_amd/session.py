"""Streaming aggregation: pack and upload each client as it arrives.

In the reference round loop (fedavg_trainer.py:172-217) clients train one
after another and each result is appended to ``w_locals`` at :199; the
reduction only starts at :217.  With the drop-in's ``aggregate`` every client
row is packed and copied to HBM at :217, so the whole PCIe transfer sits on
the round's critical path.  A ``RoundSession`` moves that work next to the
client loop: ``add`` validates the client, packs its row into pinned staging
with the native packer and starts the row's H2D on a side stream, while the
next client trains; ``finish`` then only forms the weights, runs the kernel
and copies the averaged model back.

Integration (two lines in the reference loop)::

    session = aggregator.begin_round(self.model_global.state_dict(), len(client_indexes))
    ...
    w_locals.append((client.get_sample_number(), copy.deepcopy(w)))       # :199
    session.add(*w_locals[-1])                                              # new
    ...
    w_glob = session.finish(w_locals)                                       # :217, replaces aggregate

``finish(w_locals)`` keeps ``aggregate``'s contract: it returns
``w_locals[0][1]`` with its values replaced, raises ``ZeroDivisionError`` on
a zero sample total, and checks that ``w_locals`` holds exactly the clients
that were added (same count, sample numbers and dict objects, in order).
Results are bit-identical to ``aggregate`` (and to the reference).
"""
from __future__ import annotations

import os
import time
import weakref
from collections import OrderedDict
from typing import Mapping

import torch

from . import _lib
from .layout import KeyTable

__all__ = ["RoundSession"]


class RoundSession:
    """One round's streaming reduction on a ``DeviceAggregator``'s device."""

    def __init__(self, aggregator, template: Mapping[str, torch.Tensor], max_clients: int):
        if max_clients < 1:
            raise ValueError("max_clients must be >= 1")
        self.agg = aggregator
        self.table = KeyTable(template)
        self.max_clients = max_clients
        self.counts = []
        self.dicts = []
        self._keepalive = []
        self._finished = False
        self._verify = None
        self.dev = aggregator.device
        self._lib = _lib.load()
        self._threads = max(1, torch.get_num_threads())
        with torch.cuda.device(self.dev):
            self._compute = torch.cuda.current_stream(self.dev)
            self._copy = aggregator._copy_stream_for()
            self._copy.wait_stream(self._compute)
        self._staging = {g.dtype: aggregator._staging_for(g.dtype, max_clients, g.ld)
                         for g in self.table.groups.values()}
        from .aggregate import column_chunks

        # each row is uploaded in the column chunks finish() reduces in; the
        # events of the latest add tell finish() when chunk c is complete
        self._chunks = {g.dtype: column_chunks(g.P) for g in self.table.groups.values()}
        self._ready = {}
        self._client_dev = None
        self._out_host = {}
        self._views = {}  # dtype -> the result's key views of _out_host[dtype], made before finish()
        self.finish_profile = {}
        self.add_ms = 0.0
        self.add_profile = {}  # host ms per phase of add(), summed over the round's clients
        self.keep_dicts = True
        self.defer_release = None  # callable(list): where displaced host tensors are dropped
        # a round whose fp32 rows fit in SMALL_ROUND_BYTES finishes in ONE
        # native call (fedavg_round_f32 over the rows add() already packed):
        # its kernel reads them from pinned memory, so add() skips the H2D
        groups = self.table.groups
        self._small = (len(groups) == 1 and torch.float32 in groups
                       and max_clients * groups[torch.float32].ld * 4 <= aggregator.SMALL_ROUND_BYTES)

    def add(self, sample_num, state_dict: Mapping[str, torch.Tensor]) -> None:
        """Validate, pack and start uploading one client's row (fedavg_trainer.py:199)."""
        if self._finished:
            raise RuntimeError("session already finished")
        i = len(self.counts)
        if i >= self.max_clients:
            raise ValueError(f"more than max_clients={self.max_clients} clients added")
        t0 = time.perf_counter()
        if self._client_dev is None:  # fixed by the first client: host or this aggregator's device
            self._client_dev = self.agg._client_device(self.table, [state_dict])
            if self._client_dev.type == "cuda":
                self._small = False
            elif not self._small:
                # the result's pinned buffers, allocated while clients still
                # train instead of inside finish(): a fresh 100 MB pinned
                # allocation costs 5.6-8.6 ms
                self._out_host = {g.dtype: torch.empty(g.P, dtype=g.dtype, pin_memory=True)
                                  for g in self.table.groups.values()}
                self._warm_finish_path()
                # the averaged model's key views of those buffers: a view needs
                # no data, so they are made here, while clients train, instead
                # of in finish() (350 views: ~0.5 ms, resnet56)
                self._views = {g.dtype: self.table.unpack(g, self._out_host[g.dtype])
                               for g in self.table.groups.values()}
        ptrs, keep = self.table.collect([state_dict], self._client_dev)
        if self._client_dev.type == "cuda":
            # device-resident client: one packing kernel on the copy stream,
            # after the work that produced the client's tensors
            self._copy.wait_stream(torch.cuda.current_stream(self.dev))
            for g in self.table.groups.values():
                self.agg._pack_on_device(self.table, g, ptrs, i, self._staging[g.dtype].dev, self._copy)
            if keep:
                self._keepalive.append(keep)  # until the packing kernel has read them
        else:
            self._add_host(i, ptrs)  # packed synchronously: contiguous copies may go now
        self.counts.append(sample_num)
        # the dicts are kept for finish()'s identity check; a caller that
        # verifies copies instead (autostream) sets keep_dicts = False so that
        # a round's client tensors are not all held until finish
        self.dicts.append(state_dict if self.keep_dicts else None)
        self.add_ms += (time.perf_counter() - t0) * 1e3

    # The first finish() of a process paid ~10 ms of one-time runtime work on
    # its critical path: creating the D2H stream (6.4 ms in
    # hipStreamCreateWithPriority) and the first launch of the reduce kernel
    # (3.8 ms in hipExtLaunchKernel: code-object load), per the HIP API trace
    # of scripts/stream_probe.py.  The first session of
    # an aggregator does both at its first add(), while clients still train:
    # it creates the stream, reduces column chunk 0 of the staging rows into a
    # scratch output with the finish() schedule (same K, chunk width and row
    # stride, so the same kernel) and copies that chunk to the result buffer
    # on the D2H stream.  Scratch bytes only; finish() overwrites them in
    # stream order.  FEDAVG_FINISH_WARMUP=0 turns it off.
    FINISH_WARMUP = os.environ.get("FEDAVG_FINISH_WARMUP", "1") != "0"

    def _warm_finish_path(self):
        agg = self.agg
        if getattr(agg, "_finish_warm", False) or not self.FINISH_WARMUP:
            return
        agg._finish_warm = True
        agg.warm_up()  # streams, torch's kernels of the finish and :291 (DeviceAggregator.warm_up)
        from .aggregate import _fetch, reduce_rows

        with torch.cuda.device(self.dev):
            d2h = agg._d2h_stream_for()
            for g in self.table.groups.values():
                st = self._staging[g.dtype]
                c0, c1 = self._chunks[g.dtype][0]
                K = self.max_clients
                # all on the D2H stream: the caller's (training) stream is not touched
                w = st.upload_weights([1.0 / K] * K, d2h)
                scratch = torch.empty(c1 - c0, dtype=g.dtype, device=self.dev)
                with torch.cuda.stream(d2h):
                    # the finish's own kernel: the fused aggregate + :291 pass when
                    # the rows qualify (its own code object), else the row reduce
                    reduce_rows(st.dev[:K, c0:c1], w, c1 - c0, scratch, [])
                _fetch(scratch, self._out_host[g.dtype][c0:c1], d2h)
                scratch.record_stream(d2h)

    def _add_host(self, i, ptrs):
        """Pack host client ``i`` into its pinned row and start its H2D (unless the round is small)."""
        for g in self.table.groups.values():
            st = self._staging[g.dtype]
            t0 = time.perf_counter()
            items = self.table.pack_items(g, ptrs, i, g.ld)
            _lib.check(self._lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], st.host.data_ptr(),
                                                  st.host.element_size(), self._threads), "fedavg_pack_rows")
            t1 = time.perf_counter()
            self.add_profile["pack_ms"] = self.add_profile.get("pack_ms", 0.0) + (t1 - t0) * 1e3
            if self._small:
                continue
            events = []
            with torch.cuda.stream(self._copy):
                for c0, c1 in self._chunks[g.dtype]:
                    st.dev[i, c0:c1].copy_(st.host[i, c0:c1], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self._copy)
                    events.append(ev)
            self._ready[g.dtype] = events  # the copy stream is FIFO: covers earlier rows too
            self.add_profile["h2d_issue_ms"] = (self.add_profile.get("h2d_issue_ms", 0.0)
                                                + (time.perf_counter() - t1) * 1e3)

    def abandon(self) -> None:
        """Close the session without a result (its staging is free once the
        uploads already issued have ended)."""
        if self._finished:
            return
        self._finished = True
        with torch.cuda.device(self.dev):
            self._copy.synchronize()
        self._keepalive.clear()
        self._forget_table()

    def finish(self, w_locals=None, verify=None):
        """Reduce the added clients; ``aggregate``'s contract (fedavg_trainer.py:441-458).

        ``verify`` (optional, for callers whose ``w_locals`` holds COPIES of
        the added dicts, e.g. the reference's ``copy.deepcopy(w)`` at :199):
        replaces the identity check of each dict; it is called once the GPU
        work is issued, while it runs, and a False answer makes finish()
        return None without touching ``w_locals`` (the caller then takes the
        plain path)."""
        if self._finished:
            raise RuntimeError("session already finished")
        self._finished = True
        if w_locals is not None:
            if len(w_locals) != len(self.counts):
                raise ValueError(f"w_locals has {len(w_locals)} clients, session has {len(self.counts)}")
            for i, ((n, sd), n2, sd2) in enumerate(zip(w_locals, self.counts, self.dicts)):
                if (verify is None and sd is not sd2) or n != n2:
                    raise ValueError(f"w_locals[{i}] is not the client added as #{i}")
        self._verify = verify
        if verify is not None and w_locals is not None:
            self.dicts = [sd for _, sd in w_locals]  # the round _close() leaves for :291 reuse
        if not self.counts:
            raise ValueError("no clients added (the reference returns the global model then: use aggregate([]))")
        K = len(self.counts)
        acc_dict = w_locals[0][1] if w_locals is not None else OrderedDict()
        from .aggregate import reduce_and_fetch, sample_weights

        weights = sample_weights(self.counts)  # ZeroDivisionError like the reference
        if self._small:
            return self._finish_small(K, weights, acc_dict)
        if self._client_dev.type == "cuda":
            return self._finish_device(K, weights, acc_dict)
        outs = []
        dev_state = {}
        sums = {}
        t0 = time.perf_counter()
        with torch.cuda.device(self.dev):
            # weights, reduce and the staging's release all on the stream
            # current at finish() (reduce_and_fetch launches there), which
            # need not be the one current at begin_round
            cur = torch.cuda.current_stream(self.dev)
            d2h = self.agg._d2h_stream_for()
            for g in self.table.groups.values():
                st = self._staging[g.dtype]
                # the staging's own pinned weight buffer: no pinned allocation
                # inside finish (a fresh one costs milliseconds to issue)
                w_dev = st.upload_weights(weights, cur)
                out_dev, out_host = reduce_and_fetch(st.dev[:K], w_dev, g.P,
                                                     d2h, ready=self._ready[g.dtype],
                                                     out_host=self._out_host.get(g.dtype), sums=sums)
                outs.append((g, out_host))
                dev_state[g.dtype] = (st.dev[:K], out_dev)
            t1 = time.perf_counter()
            ok = self._verify() if self._verify is not None else True  # overlaps the GPU work just issued
            t_v = time.perf_counter()
            d2h.synchronize()
            cur.synchronize()
            cur.wait_stream(self._copy)  # nothing else may reuse the staging before its copies end
        t2 = time.perf_counter()
        self.finish_profile = {"issue_ms": (t1 - t0) * 1e3, "verify_ms": (t_v - t1) * 1e3, "wait_ms": (t2 - t_v) * 1e3}
        if not ok:
            self._keepalive.clear()
            self._forget_table()
            return None
        for g, out_host in outs:
            views = self._views.get(g.dtype)
            self._set_results(acc_dict, views if views is not None else self.table.unpack(g, out_host),
                              keys_verified=self._verify is not None)
        # host-side phases of the finish (ms): issuing weights/reduce/D2H, waiting for them, unpacking
        self.finish_profile = {"issue_ms": (t1 - t0) * 1e3, "verify_ms": (t_v - t1) * 1e3, "wait_ms": (t2 - t_v) * 1e3,
                               "unpack_ms": (time.perf_counter() - t2) * 1e3}
        return self._close(K, dev_state, acc_dict, sums)

    def _finish_small(self, K, weights, acc_dict):
        """Rows already packed by add(): weights, one kernel, result copy, in one native call."""
        import numpy as np

        g = self.table.groups[torch.float32]
        st = self._staging[torch.float32]
        w64 = np.array([float(w) for w in weights], dtype=np.float64)
        with torch.cuda.device(self.dev):
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_stream(self._copy)  # earlier users of the device staging are done
            st._w_done.synchronize()  # the native call rewrites w_host: an async device round may still read it
            out_dev = torch.empty(g.P, dtype=torch.float32, device=self.dev)
            out_host = torch.empty(g.P, dtype=torch.float32, pin_memory=True)
            _lib.check(self._lib.fedavg_round_f32(None, 0, st.host.data_ptr(), st.dev.data_ptr(), K, g.P, g.ld,
                                                  w64.ctypes.data, st.w_host.data_ptr(), st.w_dev.data_ptr(),
                                                  out_dev.data_ptr(), out_host.data_ptr(), self._threads,
                                                  cur.cuda_stream), "fedavg_round_f32")
        if self._verify is not None and not self._verify():
            self._keepalive.clear()
            self._forget_table()
            return None
        self._set_results(acc_dict, self.table.unpack(g, out_host))
        return self._close(K, {torch.float32: (st.dev[:K], out_dev)}, acc_dict)

    def _finish_device(self, K, weights, acc_dict):
        """Device-resident clients: the averaged model stays in HBM (device
        tensors, ordered on the current stream, no host round trip)."""
        from .aggregate import reduce_rows

        dev_state = {}
        sums = {}
        with torch.cuda.device(self.dev):
            cur = torch.cuda.current_stream(self.dev)  # the reduce runs here, so the weights go here too
            cur.wait_stream(self._copy)  # every client's packing kernel
            for g in self.table.groups.values():
                st = self._staging[g.dtype]
                w_dev = st.upload_weights(weights, cur)
                out_dev = torch.empty(g.P, dtype=g.dtype, device=self.dev)
                parts = []
                reduce_rows(st.dev[:K], w_dev, g.P, out_dev, parts)
                if parts:
                    sums[g.dtype] = parts[0]
                dev_state[g.dtype] = (st.dev[:K], out_dev)
            if self._verify is not None and not self._verify():
                self._keepalive.clear()
                self._forget_table()
                return None
            for g in self.table.groups.values():
                self._set_results(acc_dict, self.table.unpack(g, dev_state[g.dtype][1]))
        return self._close(K, dev_state, acc_dict, sums)

    def _release(self, objs) -> None:
        """Drop references to a round's displaced host tensors -- freeing
        100 MB of host memory costs ~10 ms of munmap -- on the caller's
        release hook (autostream: its worker thread) when one is set."""
        if self.defer_release is not None and objs:
            self.defer_release(objs)

    def _forget_table(self) -> None:
        self._release(list(self.table._template))  # client 0's tensors, held for the native walk's checks
        self.table.forget_tensors()

    def _set_results(self, acc_dict, results, keys_verified: bool = False) -> None:
        """acc_dict[name] = result (fedavg_trainer.py:455 replaces client 0's values).
        ``keys_verified``: verify_rows has just seen acc_dict hold exactly the
        table's keys in order, so one group's results replace every value."""
        if keys_verified and len(self.table.groups) == 1 or (
                len(results) == len(acc_dict) and acc_dict.keys() == results.keys()):
            # every value replaced (one dtype group): two C-level calls
            old = list(acc_dict.values())
            acc_dict.update(results)
        else:
            old = []
            for name, t in results.items():
                old.append(acc_dict.get(name))
                acc_dict[name] = t
        self._release(old)

    def _close(self, K, dev_state, acc_dict, sums=None):
        self._keepalive.clear()
        self._forget_table()
        # leave the round's device rows + averaged model for client_distances (:291)
        try:
            self.agg._last = {"table": self.table, "K": K, "dev": dev_state, "sumsq": sums or {},
                              "refs": [weakref.ref(sd) for sd in self.dicts], "acc": weakref.ref(acc_dict)}
        except TypeError:
            self.agg._last = {}
        return acc_dict
