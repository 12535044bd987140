"""Zero-edit streaming: each client's upload overlaps the round loop.

The reference trains the selected clients one after another
(fedavg_trainer.py:172-214): ``client.train`` at :189 returns
``net.cpu().state_dict()`` (client.py:96), a valid result (:190) is appended
as ``(client.get_sample_number(), copy.deepcopy(w))`` at :199, and only at
:217 does ``self.aggregate(w_locals)`` see the round.  A drop-in that patches
``aggregate`` alone therefore packs and uploads all K clients at :217: at
100 clients x 25M parameters that is 10 GB over PCIe on the round's critical
path (178.8 ms).

``install`` (aggregate.py) also wraps ``Client.train`` and
``FedAvgTrainer.train``, so the unchanged loop streams:

* while ``FedAvgTrainer.train`` runs, every valid ``Client.train`` result --
  the same validity test as :190 -- is handed to a per-trainer
  :class:`ClientFeed` together with ``client.get_sample_number()``; a
  background thread packs it into pinned staging and starts its H2D
  (``RoundSession.add``) while the loop deep-copies it (:199) and the next
  client trains;
* the patched ``aggregate(w_locals)`` waits for the feed to drain, checks
  that ``w_locals`` is what was fed and then only the weights, the kernel
  and the result's D2H remain.  The check (``fedavg_collect_ext.verify_rows``,
  one native walk while the reduce runs): the same count and sample numbers
  in order, distinct dicts, every client's keys exactly the table's in order,
  EVERY (client, key) tensor an exact host Tensor, contiguous, with the
  table's dtype and shape and the version counter a fresh ``copy.deepcopy``
  gives (measured once on the running torch, ``DEEPCOPY_VERSION``), and
  element values at ~4,096 (client, key, position) probes drawn afresh every
  round -- every key at least once, the rest uniform over clients and keys --
  against the pinned staging rows the GPU reduces (converted as the packer
  converts).  The version counter makes in-place edits of w_locals between
  :199 and :217 (clipping, noise, ``copy_``, slice assignment: any in-place
  op) a deterministic fallback whatever elements they touch.  A replaced
  tensor object is one too: every fed (Ordered)dict gets a one-shot
  ``__deepcopy__`` hook that records the tensors of the loop's :199 deep copy
  (``_hook_deepcopy``), and each ``w_locals`` value must BE one of them -- so
  a replacement by another ``copy.deepcopy`` (whose version counter is a
  deep copy's as well) is caught without any probe landing on it.  The hook
  is an instance attribute between ``Client.train``'s return and that deep
  copy (pickling the result in that window would fail on it); a plain
  ``dict`` result (no instance attributes) gets no hook, and its
  replacements are left to the value probes.  An in-place edit of a ``Client.train`` result between :189 and
  its :199 deep copy is seen on the fed dict itself: the worker keeps the
  last packed dict with its counters and re-reads them when the next client
  arrives (status 9 at :217 for the round's last client).  What the counter
  cannot see -- writes through ``.data``/numpy views or raw pointers, which
  bypass autograd's bookkeeping -- is left to the value probes.

Anything else falls back to the plain drop-in on ``w_locals`` (same bits,
the reference's exceptions): a count or sample-number mismatch, a retried
client the loop did not append, a key-table change, device-resident
clients, more clients than the trainer's ``client_list``, any error inside
the feed, a Client subclass that overrides ``train`` (it may change what it
returns after the wrapped reference method fed it), a client tensor whose
version counter moved while the worker packed it (a ``Client.train`` that
returns tensors the next client's training updates in place; the
reference's returns a fresh deep copy, client.py:96 / fedavg_trainer.py:189),
or ``FEDAVG_STREAM_CLIENTS=0``.

Contract for Client.train implementations under streaming: the returned
state_dict's tensors must not change after train() returns -- the reference
(``net.cpu().state_dict()`` of a per-call ``copy.deepcopy`` of the global
model) keeps it.
"""
from __future__ import annotations

import copy
import os
import queue
import random
import threading
import time
import weakref
from typing import Optional

import torch

__all__ = ["ClientFeed", "enabled", "valid_train_result", "active_trainer", "trainer_scope"]

_tls = threading.local()


def enabled() -> bool:
    return os.environ.get("FEDAVG_STREAM_CLIENTS", "1") != "0"


def valid_train_result(res) -> bool:
    """fedavg_trainer.py:190: ``loss``, ``local_beta``, ``local_rho`` and
    ``local_acc`` all not None (a diverged client returns Nones, client.py:71-73)."""
    try:
        _, loss, beta, rho, acc = res[0], res[1], res[2], res[3], res[4]
    except (TypeError, IndexError, KeyError):
        return False
    return loss is not None and beta is not None and rho is not None and acc is not None


def active_trainer():
    """The trainer whose ``train()`` (the round loop) is running on this thread."""
    return getattr(_tls, "trainer", None)


class trainer_scope:
    """``with trainer_scope(trainer):`` -- Client.train results on this thread feed ``trainer``."""

    def __init__(self, trainer):
        self.trainer = trainer

    def __enter__(self):
        self.prev = getattr(_tls, "trainer", None)
        _tls.trainer = self.trainer
        return self.trainer

    def __exit__(self, *exc):
        _tls.trainer = self.prev
        feed = self.trainer.__dict__.get("_mfl_feed")
        if feed is not None:
            feed.close()
        return False


def deepcopy_version() -> int:
    """``copy.deepcopy(t)._version`` for a host tensor on this torch (cached)."""
    v = ClientFeed.DEEPCOPY_VERSION
    if v is None:
        import copy

        v = ClientFeed.DEEPCOPY_VERSION = int(copy.deepcopy(torch.zeros(1))._version)
    return v


class _Release(list):
    """Host tensors a finished round displaced, for the feed worker to drop."""


class ClientFeed:
    """One trainer's streaming state: at most one open ``RoundSession`` (the
    round being fed), filled by a background thread."""

    VERIFY_PROBES = 4096  # (client, key) pairs whose values are compared per round (two positions each)
    # the version counter of a tensor fresh from copy.deepcopy (fedavg_trainer.py:199):
    # 1 on torch 2.x (Tensor.__deepcopy__ ends in set_()); measured, not assumed
    DEEPCOPY_VERSION = None
    VERIFY_FULL_ELEMS = 1 << 20  # rounds of at most this many elements (K x P) are compared in full

    def __init__(self, aggregator_fn, max_clients: int):
        self._aggregator_fn = aggregator_fn  # () -> DeviceAggregator (created lazily, on first use)
        self.max_clients = max(1, int(max_clients))
        self.session = None
        self.broken = False
        self._small = False  # this round fits SMALL_ROUND_BYTES: left to the plain path
        self.fed = []  # sample numbers in feed order
        self._fed_keys = []  # each fed dict's key objects, in feed order
        # per fed client: the values of the loop's :199 deep copy of it (recorded
        # by _hook_deepcopy), or None; the round generation the hooks belong to
        self._copies = []
        self._gen = 0
        # the last packed client's dict and its version counters at packing:
        # re-read when the next client arrives (the loop's :199 copy of this
        # one is done by then) and, for the round's last client, inside the
        # :217 check -- an in-place edit of a Client.train result between
        # :189 and :199 after the worker packed it is a fallback (the loop's
        # deep copy would hold the edited values with a fresh counter)
        self._prev = None
        self._vplan = None  # verify_rows' table arrays for the open session (worker-made)
        self._graveyard = []  # _Release lists waiting for the next round (worker thread only)
        self._q: Optional[queue.Queue] = None
        self._worker: Optional[threading.Thread] = None
        self._err: Optional[BaseException] = None
        self._add_ms = []
        self._t_fed = self._t_done = 0.0
        self.stats = {"rounds_streamed": 0, "rounds_fallback": 0, "rounds_small": 0, "last_fallback": "", "last_round": {}}

    # -- producer side (Client.train wrapper) ---------------------------------
    # A round whose rows fit this many bytes is not streamed: the plain drop-in
    # finishes it in ONE native call (fedavg_round_f32, ~45 us for MNIST-LR x 10),
    # where a feed thread would only add hand-offs (MNIST-LR x 10: 1.25 vs
    # 0.29 ms at :217 in the loop-replay probe, profiles/r03/stream/).
    SMALL_ROUND_BYTES = 4 << 20

    def feed(self, sample_num, state_dict) -> None:
        if self.broken:
            return
        if len(self.fed) >= self.max_clients or not self._host_dict(state_dict):
            self._break("more clients than max_clients" if len(self.fed) >= self.max_clients
                        else "not a host state_dict")
            return
        if not self.fed and self._row_bytes(state_dict) * self.max_clients <= self.SMALL_ROUND_BYTES:
            self.broken = self._small = True  # by design: not counted as a fallback
            return
        self.fed.append(sample_num)  # the dict itself goes to the worker only (no round-long reference)
        # its key objects (the :199 deep copy shares them): verify_rows matches w_locals' keys by identity
        self._fed_keys.append(tuple(state_dict))
        self._copies.append(None)
        self._hook_deepcopy(state_dict, len(self.fed) - 1)
        if self._worker is None:
            self._q = queue.Queue()
            self._worker = threading.Thread(target=self._run, name="mfl-client-feed", daemon=True)
            self._worker.start()
        self._t_fed = time.perf_counter()
        # version counters now, before the loop trains the next client: the
        # worker re-reads them after packing (an in-place update meanwhile
        # means the packed row may mix two states)
        self._q.put((sample_num, state_dict, [v._version for v in state_dict.values()]))

    def _hook_deepcopy(self, sd, slot: int) -> None:
        """Give the fed dict a one-shot ``__deepcopy__`` (an instance
        attribute: ``copy.deepcopy`` looks it up on an OrderedDict instance)
        that makes the standard deep copy -- the hook removes itself first, so
        the copy and its ``__dict__`` are exactly what ``copy.deepcopy`` gives
        without it -- and records the copy's tensors as fed client ``slot``'s
        :199 copy.  At :217 ``verify_rows`` then requires every ``w_locals``
        value to BE one of those tensors: a tensor replaced between :199 and
        :217, even by another deep copy, is a deterministic fallback.  Plain
        ``dict`` results (no instance attributes) and dicts the loop never
        deep-copies keep ``None`` (version counters and value probes only)."""
        # copy.deepcopy dispatches on the exact type first (dict, list, ...): those never reach an
        # instance __deepcopy__, and objects without a __dict__ cannot carry one
        if (type(sd) in getattr(copy, "_deepcopy_dispatch", {dict: None}) or not hasattr(sd, "__dict__")
                or "__deepcopy__" in sd.__dict__):
            return
        ref, feed_ref, gen = weakref.ref(sd), weakref.ref(self), self._gen

        def hook(memo):
            d = ref()
            d.__dict__.pop("__deepcopy__", None)  # one shot: the copy below is the plain one
            y = copy.deepcopy(d, memo)
            feed = feed_ref()
            if feed is not None and feed._gen == gen and slot < len(feed._copies):
                feed._copies[slot] = tuple(y.values()) if isinstance(y, dict) else None
            return y

        try:
            sd.__deepcopy__ = hook
        except (AttributeError, TypeError):
            pass

    def refuse(self, why: str) -> None:
        """This round is not streamed (the plain drop-in runs at :217)."""
        if not self._small:
            self._break(why)

    @staticmethod
    def _row_bytes(sd) -> int:
        return sum(4 * v.numel() for v in sd.values())  # the packed fp32 row (wider dtypes: more)

    @staticmethod
    def _host_dict(sd) -> bool:
        try:
            return all(isinstance(v, torch.Tensor) and v.device.type == "cpu" for v in sd.values())
        except AttributeError:
            return False

    def _run(self):
        while True:
            item = self._q.get()
            if item is None:
                self._q.task_done()
                return
            if type(item) is _Release:
                # displaced tensors of a finished round: kept until the next
                # round's first client arrives and dropped then, while the loop
                # trains -- dropping them now would hold the GIL through ~10 ms
                # of munmap per 100 MB right after :217, beside the caller
                self._graveyard.append(item)
                item = None
                self._q.task_done()
                continue
            if self._graveyard:
                self._graveyard.clear()
            t0 = time.perf_counter()
            try:
                if not self.broken and self._err is None:
                    n, sd, vers = item
                    prev, self._prev = self._prev, None
                    if prev is not None and [v._version for v in prev[0].values()] != prev[1]:
                        raise RuntimeError("a fed client's tensors changed after they were packed")
                    prev = None
                    if self.session is None:
                        self.session = self._aggregator_fn().begin_round(sd, self.max_clients)
                        self.session.keep_dicts = False
                        self.session.defer_release = self._defer_release
                        self._vplan = self._verify_plan(self.session)
                    self.session.add(n, sd)
                    if [v._version for v in sd.values()] != vers:
                        raise RuntimeError("a client's tensors changed while they were packed")
                    self._prev = (sd, vers)  # until the next client (the loop's `w` holds it as long)
            except BaseException as e:  # noqa: BLE001 -- any failure means: fall back at aggregate
                self._err = e
                self._prev = None
            finally:
                item = n = sd = vers = prev = None  # no other reference to the client's tensors
                t1 = time.perf_counter()
                self._add_ms.append((t1 - t0) * 1e3)
                self._t_done = t1
                self._q.task_done()

    def _defer_release(self, objs):
        q = self._q
        if q is not None:
            q.put(_Release(objs))

    def _drain(self):
        if self._q is not None:
            self._q.join()

    def _break(self, why: str):
        self.broken = True
        self.stats["last_fallback"] = why

    # -- consumer side (patched aggregate) --------------------------------------
    def take(self, w_locals):
        """The streamed result for ``w_locals``, or None (the caller runs the
        plain drop-in).  Always leaves the feed empty for the next round."""
        try:
            if self._small:
                self.stats["rounds_small"] += 1
                return None
            t_call = time.perf_counter()
            self._drain()
            if self._add_ms:  # the worker's per-client cost and how far it trailed the loop
                self.stats["last_round"] = {
                    "clients": len(self._add_ms), "add_ms_median": sorted(self._add_ms)[len(self._add_ms) // 2],
                    "add_ms_max": max(self._add_ms), "drain_wait_ms": (time.perf_counter() - t_call) * 1e3,
                    "worker_done_after_last_feed_ms": (self._t_done - self._t_fed) * 1e3,
                    "session_add_profile": dict(getattr(self.session, "add_profile", {}))}
            sess = self.session
            why = self._mismatch(w_locals, sess)
            if why:
                self.stats["last_fallback"] = why
                self.stats["rounds_fallback"] += 1
                return None
            t_f = time.perf_counter()
            out = sess.finish(w_locals, verify=lambda: self._same_values(w_locals))
            self.stats["last_round"]["finish_ms"] = (time.perf_counter() - t_f) * 1e3
            self.stats["last_round"]["finish_profile"] = dict(getattr(sess, "finish_profile", {}))
            if out is None:
                self.stats["last_fallback"] = ("w_locals differs from the fed clients (verify_rows status "
                                               f"{self.stats.get('last_verify', {}).get('status')})")
                self.stats["rounds_fallback"] += 1
            else:
                self.stats["rounds_streamed"] += 1
            return out
        finally:
            self._reset()

    def _mismatch(self, w_locals, sess) -> str:
        if self.broken:
            return self.stats["last_fallback"] or "feed broken"
        if self._err is not None:
            return f"feed error: {self._err!r}"
        if sess is None or self._vplan is None:
            return "nothing fed"
        if type(w_locals) is not list or len(w_locals) != len(self.fed) or len(sess.counts) != len(self.fed):
            return "client count differs from the fed clients"
        for (n, _), n2 in zip(w_locals, self.fed):
            if n != n2:
                return "sample numbers differ from the fed clients"
        return ""

    @staticmethod
    def _verify_plan(sess):
        """verify_rows' arrays for a session: the key table (names, meta
        templates, dtype group, offset and packer kind per key) and each
        group's pinned staging rows (what the H2D copies upload)."""
        from .layout import _PACK_KIND, _collect_ext

        ext = _collect_ext()
        if ext is None or not hasattr(ext, "verify_rows"):
            return None
        table = sess.table
        gidx = {dt: k for k, dt in enumerate(table.groups)}
        stag = [sess._staging[dt].host for dt in table.groups]
        return (ext, [e.name for e in table.entries],
                table.meta_template(),
                [gidx[e.dtype] for e in table.entries], [int(e.offset) for e in table.entries],
                [0 if e.src_dtype == e.dtype else _PACK_KIND[e.src_dtype] for e in table.entries],
                [t.data_ptr() for t in stag], [int(t.stride(0)) for t in stag], [t.element_size() for t in stag])

    def _same_values(self, w_locals) -> bool:
        """``verify_rows`` (module docstring).  Never raises: it runs while the
        round's GPU work is in flight, and anything unexpected means the
        round is not the fed one."""
        try:
            prev, self._prev = self._prev, None  # the last client's dict as fed (the worker is drained)
            if prev is None or [v._version for v in prev[0].values()] != prev[1]:
                self.stats["last_verify"] = {"status": 9, "client": len(self.fed) - 1, "key": -1, "probes": 0}
                return False
            prev = None
            ext, names, templ, group, offset, kind, sptr, sld, ses = self._vplan
            st = ext.verify_rows(w_locals, list(self.fed), names, templ, group, offset, kind, sptr, sld, ses,
                                 self.VERIFY_PROBES, random.getrandbits(64), self.VERIFY_FULL_ELEMS,
                                 deepcopy_version(), self._fed_keys, list(self._copies))
            self.stats["last_verify"] = {"status": int(st[0]), "client": int(st[1]), "key": int(st[2]),
                                         "probes": int(st[3])}
            if len(st) > 4:  # native phase times (us) and the walk's thread count
                self.stats["last_verify"].update(prep_us=round(st[4][0], 1), walk_us=round(st[4][1], 1),
                                                 tail_us=round(st[4][2], 1), threads=int(st[4][3]))
            return st[0] == 0
        except Exception:  # noqa: BLE001
            return False

    def _reset(self):
        sess = self.session
        if sess is not None and not sess._finished:
            sess.abandon()
        self.session = None
        self.fed = []
        if self._fed_keys:
            # 35,000 key references at resnet56 x 100: their decrefs (cold
            # objects, ~0.2 ms) go to the worker, off the :217 call
            self._defer_release(self._fed_keys)
        if self._copies:
            self._defer_release(self._copies)
        self._fed_keys = []
        self._copies = []
        self._gen += 1  # hooks of dicts fed in this round (not yet deep-copied) record nothing now
        self._vplan = None
        self._prev = None
        self.broken = self._small = False
        self._err = None
        self._add_ms = []

    def close(self):
        """End of the round loop: abandon an open round, stop the worker."""
        try:
            self._drain()
        finally:
            self._reset()
            if self._worker is not None:
                self._q.put(None)
                self._worker.join(timeout=60)
                self._worker = None
                self._q = None
            self._graveyard.clear()
