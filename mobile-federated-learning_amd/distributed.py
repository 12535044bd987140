"""P-sharded FedAvg reduction across the GPUs of one node.

The reference runs everything in one process (no
collectives).  On MI355X the flattened parameter vector of the global model is
partitioned over G ranks (one process per GPU, ``torch.distributed`` with the
``nccl`` backend = RCCL over xGMI).  Every output element depends only on the
same element of the K clients (fedavg_trainer.py:451-457), so each rank
reduces its columns with the exact sequential kernel -- no data-path
communication, bit-identical results -- and ONE exchange step, an all-gather,
reassembles the averaged model on every rank.

Layout (block-cyclic, so that an all-gather chunk lands contiguously in the
final vector): with G ranks, C chunks and a block of ``S_c`` columns
(a multiple of ``ALIGN_ELEMS``), rank ``r`` owns global columns

    [c*G*S_c + r*S_c, c*G*S_c + (r+1)*S_c)    for c = 0..C-1,

stored contiguously as local columns ``[c*S_c, (c+1)*S_c)`` of its
``[K, C*S_c]`` client buffer.  ``all_gather_into_tensor`` of chunk ``c``
writes global columns ``[c*G*S_c, (c+1)*G*S_c)`` in order, so the reassembled
vector needs no permutation.  C = 1 is plain contiguous sharding.

Overlap: the reduce of chunk c+1 runs on the compute stream while RCCL
gathers chunk c (torch issues the collective on its own stream, ordered after
the kernel that produced the chunk).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from .reduce import ALIGN_ELEMS, PreparedReduce, reduce_packed

__all__ = ["ShardPlan", "plan_shards", "ShardedReducer", "upload_segments"]


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


@dataclass(frozen=True)
class ShardPlan:
    P: int  # valid global columns
    world_size: int
    rank: int
    chunks: int
    block: int  # S_c: columns per (rank, chunk)

    @property
    def local_cols(self) -> int:
        return self.chunks * self.block

    @property
    def padded_P(self) -> int:
        return self.chunks * self.world_size * self.block

    def global_range(self, chunk: int, rank: Optional[int] = None):
        r = self.rank if rank is None else rank
        start = chunk * self.world_size * self.block + r * self.block
        return start, start + self.block

    def valid_local_cols(self) -> int:
        """Local columns that map to global columns < P (the rest is padding)."""
        n = 0
        for c in range(self.chunks):
            s, e = self.global_range(c)
            n += max(0, min(e, self.P) - s)
        return n

    def local_segments(self):
        """[(local_start, global_start, length)] of valid columns owned by this rank."""
        segs = []
        for c in range(self.chunks):
            s, e = self.global_range(c)
            n = max(0, min(e, self.P) - s)
            if n > 0:
                segs.append((c * self.block, s, n))
        return segs


def plan_shards(P: int, world_size: int, rank: int, chunks: int = 1, align: int = ALIGN_ELEMS) -> ShardPlan:
    if P < 0 or world_size < 1 or not (0 <= rank < world_size) or chunks < 1:
        raise ValueError("bad shard plan arguments")
    block = max(_round_up(-(-P // (world_size * chunks)), align), align)
    return ShardPlan(P, world_size, rank, chunks, block)


def upload_segments(dst: torch.Tensor, host: torch.Tensor, segs, stream: Optional[torch.cuda.Stream] = None) -> None:
    """``dst[:, l:l+n] = host[:, g:g+n]`` for every ``(l, g, n)`` in ``segs``.

    ``dst`` is a device ``[K, ld]`` buffer, ``host`` a host ``[K, >=P]`` one.
    From pinned host memory with unit column stride every segment is one
    strided DMA (``fedavg_upload_shard``: height K, src pitch = the host row);
    otherwise torch's per-segment copy.  Asynchronous on ``stream`` (default:
    the current stream) when pinned."""
    K = dst.shape[0]
    if dst.device.type == "cuda" and host.is_pinned() and host.stride(1) == 1 and dst.stride(1) == 1:
        from . import _lib

        lib = _lib.load()
        es = host.element_size()
        s = stream if stream is not None else torch.cuda.current_stream(dst.device)
        dpitch = (dst.stride(0) if K > 1 else dst.shape[1]) * es
        spitch = (host.stride(0) if K > 1 else host.shape[1]) * es
        for lstart, gstart, n in segs:
            if lstart + n > dst.shape[1] or gstart + n > host.shape[1]:
                raise ValueError(f"segment ({lstart}, {gstart}, {n}) out of range")
            rc = lib.fedavg_upload_shard(dst.data_ptr() + lstart * es, dpitch, host.data_ptr() + gstart * es, spitch,
                                         n * es, K, s.cuda_stream)
            _lib.check(rc, "fedavg_upload_shard")
        return
    ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctx:
        for lstart, gstart, n in segs:
            dst[:, lstart:lstart + n].copy_(host[:, gstart:gstart + n], non_blocking=True)


LocalReduce = Callable[[torch.Tensor, torch.Tensor, int, torch.Tensor], None]


def _hip_local_reduce(clients: torch.Tensor, weights: torch.Tensor, P: int, out: torch.Tensor) -> None:
    reduce_packed(clients, weights, P, out)


class ShardedReducer:
    """One rank's part of the P-sharded reduction plus the all-gather.

    ``clients`` is this rank's ``[K, local_cols]`` device buffer (fill it with
    :meth:`load_from_host` or generate synthetic data in place).  ``step``
    runs the exact kernel chunk by chunk and all-gathers every chunk into
    ``self.full`` (``[padded_P]``; the model is ``self.full[:P]``).

    ``local_reduce`` is injectable so the sharding/gather logic can be tested
    with the ``gloo`` backend on CPU; the product default is the HIP kernel.

    ``gather``: None (default) all-gathers when the group has more than one
    rank; True forces the collective even at world size 1 (so the RCCL
    exchange runs, and is tested, on a single GPU); False never gathers.

    ``as_rank=(G, r)``: plan rank r's shard of a G-rank run in this process
    (no exchange) -- bench.py's single-GPU rehearsal of the per-rank kernel
    at the 8-GPU geometry.

    ``host_out`` (SURVEY §8e's alternative for a host consumer): a pinned
    host tensor of >= P elements -- e.g. one mapping shared by all ranks of
    the node.  Each rank then copies its finished chunks straight to their
    global positions in it (D2H on a side stream, overlapped with the next
    chunk's reduce) and no collective runs: the consumer of
    ``fedavg_trainer.py:219`` is host memory anyway.
    """

    def __init__(self, K: int, P: int, *, chunks: int = 1, group=None, device=None,
                 dtype: torch.dtype = torch.float32, local_reduce: Optional[LocalReduce] = None,
                 gather: Optional[bool] = None, host_out: Optional[torch.Tensor] = None,
                 as_rank: Optional[tuple] = None):
        self.group = group
        ws = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        if as_rank is not None:  # (world_size, rank): one rank's shard of a larger plan, no exchange
            if gather:
                raise ValueError("as_rank plans a shard of another world size; it cannot gather")
            ws, rank = int(as_rank[0]), int(as_rank[1])
            gather = False
        self.plan = plan_shards(P, ws, rank, chunks)
        self.K = K
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.local_reduce = local_reduce or _hip_local_reduce
        self.host_out = host_out
        if host_out is not None:
            if host_out.device.type != "cpu" or host_out.dtype != dtype or host_out.numel() < P:
                raise ValueError(f"host_out must be a host {dtype} tensor of >= {P} elements")
            if self.device.type == "cuda" and not host_out.is_pinned():
                raise ValueError("host_out must be pinned (async D2H)")
            gather = False
        if gather and not dist.is_initialized():
            raise ValueError("gather=True needs an initialised process group")
        # None: gather whenever there is more than one rank.  True forces the
        # collective at world size 1 too (the RCCL path under test on one GPU).
        self.gather = (ws > 1) if gather is None else bool(gather)
        self._copy_stream = (torch.cuda.Stream(self.device)
                             if host_out is not None and self.device.type == "cuda" else None)
        # per chunk: (local start, global start, n) of its valid columns
        S = self.plan.block
        self._chunk_segments = [[(l, g, n) for l, g, n in self.plan.local_segments() if c * S <= l < (c + 1) * S]
                                for c in range(self.plan.chunks)]
        self.clients = torch.empty((K, self.plan.local_cols), dtype=dtype, device=self.device)
        self.local_out = torch.empty(self.plan.local_cols, dtype=dtype, device=self.device)
        self.full = (torch.empty(self.plan.padded_P, dtype=dtype, device=self.device)
                     if self.gather else None)

    # ------------------------------------------------------------------
    def load_from_host(self, host_clients: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Copy this rank's columns of a host ``[K, >=P]`` buffer.

        SURVEY.md section 8e's input distribution: from pinned host memory each
        of this rank's column segments is ONE strided DMA (``fedavg_upload_shard``,
        src pitch = the host row, height = K) straight into the device rows --
        no host-side gather of the shard.  Padding columns are zeroed.
        Asynchronous on ``stream`` (default: the current stream) when pinned.
        """
        if host_clients.dim() != 2 or host_clients.shape[0] != self.K:
            raise ValueError("host buffer must be [K, >=P] with K = the reducer's client count")
        if host_clients.shape[1] < self.plan.P or host_clients.dtype != self.dtype:
            raise ValueError(f"host buffer must hold >= {self.plan.P} {self.dtype} columns")
        segs = self.plan.local_segments()
        self._zero_padding(segs)
        upload_segments(self.clients, host_clients, segs, stream)

    def _zero_padding(self, segs) -> None:
        """Zero the local columns no global column maps to (tail of the plan)."""
        covered = sorted((l, l + n) for l, _, n in segs)
        pos = 0
        for a, b in covered + [(self.plan.local_cols, self.plan.local_cols)]:
            if a > pos:
                self.clients[:, pos:a].zero_()
            pos = max(pos, b)

    def _prepared_calls(self, weights: torch.Tensor):
        """Per-chunk PreparedReduce calls of the HIP kernel for these weights
        and the current ``local_out`` (rebuilt when either changes)."""
        key = (weights.data_ptr(), weights.numel(), self.local_out.data_ptr())
        cache = self.__dict__.setdefault("_calls", {})
        calls = cache.get(key)
        if calls is None:
            S = self.plan.block
            # each PreparedReduce keeps its tensors (and so these weights) alive
            calls = [PreparedReduce(self.clients[:, c * S:(c + 1) * S], weights, S, self.local_out[c * S:(c + 1) * S])
                     for c in range(self.plan.chunks)]
            if len(cache) >= 8:
                cache.clear()
            cache[key] = calls
        return calls

    def step(self, weights: torch.Tensor, timing: Optional[Callable[[int], Optional[tuple]]] = None,
             span: Optional[tuple] = None) -> Optional[torch.Tensor]:
        """Reduce every local chunk; all-gather each as soon as it is ready.

        On a HIP device with the collective, every chunk's reduce is launched
        back to back on the current stream (an event recorded after each),
        THEN the chunks' all-gathers are issued from a side stream that waits
        on chunk c's event before gather c: the gather of chunk c still
        overlaps the reduce of chunk c+1 on the GPU, and the reduce launches
        are no longer spaced by the collective's host-side issue cost (tens of
        microseconds per all_gather_into_tensor against a ~46-90 us chunk
        kernel at N = 8).  The current stream waits for the gathers at the end.

        ``timing(c)`` (optional): a recorded (start, stop) event pair for
        chunk c's reduce, or None -- launch-attached kernel timing for the
        HIP kernel (bench.py); ignored by an injected ``local_reduce``.
        ``span`` (optional): a (start, stop) event pair recorded on the current
        stream right before the first chunk's launch and right after the last
        one's -- the chunk kernels back to back, with no host work between
        them on the GPU's side (bench.py divides it by the launches)."""
        plan = self.plan
        S = plan.block
        works: List = []
        fast = (self.local_reduce is _hip_local_reduce and self.device.type == "cuda"
                and weights.dtype == torch.float32 and self.dtype == torch.float32)
        calls = self._prepared_calls(weights) if fast else None
        cuda = self.device.type == "cuda"
        deferred = self.gather and cuda
        # the stream object only when an event goes on it (~2 us of host time
        # per step otherwise: a cache-resident model's whole step is ~10 us)
        cur = torch.cuda.current_stream(self.device) if cuda and (deferred or span is not None) else None
        if deferred and self.__dict__.get("_chunk_events") is None:
            self._chunk_events = [torch.cuda.Event() for _ in range(plan.chunks)]
            self._gather_stream = torch.cuda.Stream(self.device)
        if span is not None:
            span[0].record(cur)
        for c in range(plan.chunks):
            if calls is not None:
                calls[c](events=timing(c) if timing is not None else None)
            else:
                self.local_reduce(self.clients[:, c * S:(c + 1) * S], weights, S, self.local_out[c * S:(c + 1) * S])
            if deferred:
                self._chunk_events[c].record(cur)
            elif self.gather:
                works.append(self._gather_chunk(c))
            elif self.host_out is not None:
                self._to_host(c)
        if span is not None:
            span[1].record(cur)
        if deferred:
            gs = self._gather_stream
            with torch.cuda.stream(gs):
                for c in range(plan.chunks):
                    gs.wait_event(self._chunk_events[c])  # chunk c's reduce only
                    works.append(self._gather_chunk(c))
        for w in works:
            w.wait()  # the current stream (again `cur`) waits for the exchange
        if self._copy_stream is not None:
            self._copy_stream.synchronize()
        if self.host_out is not None:
            return self.host_out[:plan.P]
        return self.full[:plan.P] if self.gather else None

    def _gather_chunk(self, c: int):
        """The async all-gather of chunk c into its contiguous slice of ``full``."""
        plan, S = self.plan, self.plan.block
        out_c = self.local_out[c * S:(c + 1) * S]
        dst = self.full[c * plan.world_size * S:(c + 1) * plan.world_size * S]
        return dist.all_gather_into_tensor(dst, out_c, group=self.group, async_op=True)

    def gather_only(self) -> None:
        """The exchange step alone: all-gather every chunk of ``local_out``
        (diagnostics: bench.py times it next to the full step)."""
        if not self.gather:
            return
        plan, S = self.plan, self.plan.block
        works = [dist.all_gather_into_tensor(self.full[c * plan.world_size * S:(c + 1) * plan.world_size * S],
                                             self.local_out[c * S:(c + 1) * S], group=self.group, async_op=True)
                 for c in range(plan.chunks)]
        for w in works:
            w.wait()

    def _to_host(self, c: int) -> None:
        segs = self._chunk_segments[c]
        if self._copy_stream is None:  # CPU (gloo tests): plain copies
            for l, g, n in segs:
                self.host_out[g:g + n].copy_(self.local_out[l:l + n])
            return
        self._copy_stream.wait_stream(torch.cuda.current_stream(self.device))  # chunk c is reduced
        with torch.cuda.stream(self._copy_stream):
            for l, g, n in segs:
                self.host_out[g:g + n].copy_(self.local_out[l:l + n], non_blocking=True)

    def local_model_columns(self):
        """(local_out views, global ranges) of the valid columns this rank reduced."""
        return [(self.local_out[l:l + n], (g, g + n)) for l, g, n in self.plan.local_segments()]
