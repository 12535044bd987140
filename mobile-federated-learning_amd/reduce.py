"""Device-level entry points: the reduction over device-resident buffers.

These wrap the C ABI (include/fedavg_amd.h) for torch device tensors; torch is
only plumbing here (HBM allocation and the current HIP stream).  Every call
is stream-ordered on ``torch.cuda.current_stream()`` unless ``stream`` is
given, and raises ``FedAvgLibraryError`` if the HIP library is unavailable.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import _lib

__all__ = ["reduce_packed", "reduce_tensors", "weights_tensor", "client_sqdist", "reduce_with_sqdist",
           "ALIGN_ELEMS"]

# Row stride granule of the packed [K, ld] layout: 64 elements (256 B for
# fp32) keeps every client row 16-B aligned for the float4/double2/8xhalf
# vector paths and starts each row on its own 256-B boundary.
ALIGN_ELEMS = 64

_ENTRY = {
    torch.float32: "fedavg_reduce_f32",
    torch.float64: "fedavg_reduce_f64",
    torch.float16: "fedavg_reduce_f16",
    torch.bfloat16: "fedavg_reduce_bf16",
}


def _stream_handle(stream: Optional[torch.cuda.Stream], device: torch.device) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


def weights_tensor(weights: Sequence[float], dtype: torch.dtype, device) -> torch.Tensor:
    """Device weight vector: fp32 for fp32/fp16/bf16 groups, fp64 for fp64.

    ``weights`` are the reference's Python doubles ``n_i / N``
    (fedavg_trainer.py:453); ``torch.tensor(..., float32)`` rounds each one to
    nearest fp32, exactly the cast ATen applies to the scalar in ``p * w``.
    """
    wdt = torch.float64 if dtype == torch.float64 else torch.float32
    host = torch.tensor([float(w) for w in weights], dtype=wdt)
    if torch.device(device).type == "cuda":
        host = host.pin_memory()
    return host.to(device, non_blocking=True)


def _check_device_tensor(t: torch.Tensor, name: str):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise ValueError(f"{name} must be a CUDA (HIP) device tensor")


def _check_packed(clients: torch.Tensor, weights: torch.Tensor, P: Optional[int], out: Optional[torch.Tensor]):
    """reduce_packed's argument checks; returns (K, ld, P, dtype, out), allocating ``out`` if None."""
    _check_device_tensor(clients, "clients")
    _check_device_tensor(weights, "weights")
    if clients.dim() != 2 or clients.stride(1) != 1:
        raise ValueError("clients must be 2-D [K, ld] with unit column stride")
    K = clients.shape[0]
    ld = clients.stride(0) if K > 1 else clients.shape[1]
    if P is None:
        P = clients.shape[1]
    if P > clients.shape[1]:
        raise ValueError(f"P={P} exceeds clients.shape[1]={clients.shape[1]}")
    dtype = clients.dtype
    if dtype not in _ENTRY:
        raise TypeError(f"unsupported client dtype {dtype}")
    wdt = torch.float64 if dtype == torch.float64 else torch.float32
    if weights.dtype != wdt or weights.numel() != K or not weights.is_contiguous():
        raise ValueError(f"weights must be a contiguous [{K}] {wdt} tensor")
    if weights.device != clients.device:
        raise ValueError("weights and clients must be on the same device")
    if out is None:
        out = torch.empty(P, dtype=dtype, device=clients.device)
    else:
        _check_device_tensor(out, "out")
        if out.dtype != dtype or out.numel() < P or not out.is_contiguous() or out.device != clients.device:
            raise ValueError(f"out must be a contiguous device tensor of >= {P} {dtype}")
    return K, ld, P, dtype, out


def reduce_packed(
    clients: torch.Tensor,
    weights: torch.Tensor,
    P: Optional[int] = None,
    out: Optional[torch.Tensor] = None,
    *,
    splits: int = 1,
    stream: Optional[torch.cuda.Stream] = None,
    tuned: Optional[tuple] = None,
    events: Optional[tuple] = None,
) -> torch.Tensor:
    """out[p] = sum_i clients[i, p] * weights[i], client 0 first (bit-exact).

    clients : [K, ld] device tensor, row stride ld >= P, unit column stride.
    weights : [K] device tensor (fp32; fp64 for fp64 clients).
    P       : number of valid columns (default ``clients.shape[1]``).
    splits  : 1 = exact sequential kernel; 2/4/8 = split-client fp32 variant
              (tolerance-gated, not bit-exact).
    events  : (start, stop) torch.cuda.Event pair, each recorded once before
              (so the HIP event exists): the fp32 production launches are
              bracketed by them at the launches themselves
              (fedavg_reduce_f32_timed, hipExtLaunchKernel) -- kernel time
              without the stream serialisation of a separate record pair.
    tuned   : benchmarking hook for the fp32 kernel: (unroll, nontemporal) or
              (unroll, nontemporal, cols, pipelined, max_blocks), see
              include/fedavg_amd_tuning.h (probe library).  Every variant gives
              the same bits.
    """
    K, ld, P, dtype, out = _check_packed(clients, weights, P, out)
    lib = _lib.load()
    s = _stream_handle(stream, clients.device)
    if splits != 1:
        if dtype != torch.float32:
            raise TypeError("the split-client variant is fp32 only")
        rc = lib.fedavg_reduce_splitk_f32(clients.data_ptr(), K, P, ld, weights.data_ptr(), out.data_ptr(), splits, s)
        _lib.check(rc, "fedavg_reduce_splitk_f32")
    elif tuned is not None:
        if dtype != torch.float32:
            raise TypeError("tuned variants are fp32 only")
        lib = _lib.load_probe()  # tuning hooks live in the probe library only
        if len(tuned) == 2:
            unroll, nt = tuned
            rc = lib.fedavg_reduce_f32_tuned(clients.data_ptr(), K, P, ld, weights.data_ptr(), out.data_ptr(),
                                             int(unroll), int(nt), s)
            _lib.check(rc, "fedavg_reduce_f32_tuned", lib)
        else:
            unroll, nt, cols, pipe, max_blocks = tuned
            rc = lib.fedavg_reduce_f32_variant(clients.data_ptr(), K, P, ld, weights.data_ptr(), out.data_ptr(),
                                               int(unroll), int(nt), int(cols), int(pipe), int(max_blocks), s)
            _lib.check(rc, "fedavg_reduce_f32_variant", lib)
    elif events is not None:
        if dtype != torch.float32:
            raise TypeError("launch-attached timing events are fp32 only")
        e0, e1 = events
        if not e0.cuda_event or not e1.cuda_event:
            raise ValueError("record each timing event once before use (torch creates the HIP event lazily)")
        rc = lib.fedavg_reduce_f32_timed(clients.data_ptr(), K, P, ld, weights.data_ptr(), out.data_ptr(), s,
                                         e0.cuda_event, e1.cuda_event)
        _lib.check(rc, "fedavg_reduce_f32_timed")
    else:
        fn = getattr(lib, _ENTRY[dtype])
        rc = fn(clients.data_ptr(), K, P, ld, weights.data_ptr(), out.data_ptr(), s)
        _lib.check(rc, _ENTRY[dtype])
    return out


def _raw_stream(device: torch.device) -> int:
    """The current stream's hipStream_t for ``device`` (torch's raw getter
    when present: ~0.3 us instead of ~1.5 us for the Stream object)."""
    get = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if get is not None:
        return int(get(device.index if device.index is not None else torch.cuda.current_device()))
    return int(torch.cuda.current_stream(device).cuda_stream)


class PreparedReduce:
    """One fp32 ``reduce_packed`` call on fixed tensors, validated once and
    re-issued with a single ctypes call -- the per-step host path of the
    sharded reducer (small, cache-resident workloads are launch-bound: the
    Python checks of ``reduce_packed`` cost about as much as the kernel).
    ``__call__(stream=None, events=None)``: on ``stream`` (default: the
    device's current stream); ``events`` = a recorded (start, stop)
    torch.cuda.Event pair attached to the launches (fedavg_reduce_f32_timed)."""

    def __init__(self, clients: torch.Tensor, weights: torch.Tensor, P: int, out: torch.Tensor):
        K, ld, P, dtype, out = _check_packed(clients, weights, P, out)
        if dtype != torch.float32:
            raise TypeError("PreparedReduce is the fp32 path")
        self._args = (clients.data_ptr(), K, P, ld, weights.data_ptr(), out.data_ptr())
        self._keep = (clients, weights, out)
        self._device = clients.device
        self._lib = _lib.load()
        self._aligned = (clients.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0 and ld % 4 == 0 and P > 0)

    def __call__(self, stream: Optional[torch.cuda.Stream] = None, events: Optional[tuple] = None) -> None:
        s = int(stream.cuda_stream) if stream is not None else _raw_stream(self._device)
        if events is not None and self._aligned:
            rc = self._lib.fedavg_reduce_f32_timed(*self._args, s, events[0].cuda_event, events[1].cuda_event)
            if rc:
                _lib.check(rc, "fedavg_reduce_f32_timed")
            return
        rc = self._lib.fedavg_reduce_f32(*self._args, s)
        if rc:
            _lib.check(rc, "fedavg_reduce_f32")


def reduce_tensors(
    clients: Sequence[torch.Tensor],
    weights: torch.Tensor,
    out: Optional[torch.Tensor] = None,
    *,
    stream: Optional[torch.cuda.Stream] = None,
) -> torch.Tensor:
    """Pointer-array variant: K separate contiguous fp32 device tensors of P elements."""
    if not clients:
        raise ValueError("need at least one client")
    dev = clients[0].device
    P = clients[0].numel()
    for i, c in enumerate(clients):
        _check_device_tensor(c, f"clients[{i}]")
        if c.dtype != torch.float32 or c.numel() != P or not c.is_contiguous() or c.device != dev:
            raise ValueError(f"clients[{i}] must be a contiguous fp32 device tensor of {P} elements")
    _check_device_tensor(weights, "weights")
    if weights.dtype != torch.float32 or weights.numel() != len(clients):
        raise ValueError("weights must be [K] fp32")
    ptrs = torch.tensor([c.data_ptr() for c in clients], dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=dev)
    lib = _lib.load()
    rc = lib.fedavg_reduce_ptrs_f32(ptrs.data_ptr(), len(clients), P, weights.data_ptr(), out.data_ptr(),
                                    _stream_handle(stream, dev))
    _lib.check(rc, "fedavg_reduce_ptrs_f32")
    # keep the pointer array alive until the kernel has consumed it
    ptrs.record_stream(stream if stream is not None else torch.cuda.current_stream(dev))
    return out


_SQDIST_ENTRY = {
    torch.float32: "fedavg_client_sqdist_f32",
    torch.float64: "fedavg_client_sqdist_f64",
    torch.float16: "fedavg_client_sqdist_f16",
    torch.bfloat16: "fedavg_client_sqdist_bf16",
}


def client_sqdist(clients: torch.Tensor, glob: torch.Tensor, P: Optional[int] = None, *,
                  stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """sumsq[i] = sum_p d_i[p]^2 in fp64 (device [K] float64), with
    d_i = clients[i, p] - glob[p] rounded as the reference's
    ``w[para] - w_glob[para]`` rounds it in the rows' dtype (fp32; fp64;
    fp16/bf16 via fp32 opmath).

    The squared distance behind fedavg_trainer.py:291; the norm is
    ``sqrt(sumsq)`` rounded to torch.cat's dtype.  ``clients`` [K, ld]
    (16-B aligned rows), ``glob`` [>= P] of the same dtype and device.
    """
    _check_device_tensor(clients, "clients")
    _check_device_tensor(glob, "glob")
    dtype = clients.dtype
    if dtype not in _SQDIST_ENTRY or glob.dtype != dtype:
        raise TypeError(f"client_sqdist: unsupported dtypes {dtype} / {glob.dtype}")
    if clients.dim() != 2 or clients.stride(1) != 1:
        raise ValueError("clients must be 2-D [K, ld] with unit column stride")
    K = clients.shape[0]
    ld = clients.stride(0) if K > 1 else clients.shape[1]
    P = clients.shape[1] if P is None else P
    if glob.numel() < P or not glob.is_contiguous():
        raise ValueError("glob must be a contiguous tensor of >= P elements")
    lib = _lib.load()
    if dtype == torch.float32:
        n_ws = lib.fedavg_client_sqdist_workspace(K, P)
    else:
        n_ws = lib.fedavg_client_sqdist_workspace_elems(K, P, clients.element_size())
    work = torch.empty(max(n_ws, 1), dtype=torch.float64, device=clients.device)
    out = torch.empty(K, dtype=torch.float64, device=clients.device)
    entry = _SQDIST_ENTRY[dtype]
    rc = getattr(lib, entry)(clients.data_ptr(), K, P, ld, glob.data_ptr(), work.data_ptr(), n_ws, out.data_ptr(),
                             _stream_handle(stream, clients.device))
    _lib.check(rc, entry)
    return out


def reduce_with_sqdist(clients: torch.Tensor, weights: torch.Tensor, P: Optional[int] = None,
                       out: Optional[torch.Tensor] = None, *, stream: Optional[torch.cuda.Stream] = None):
    """One round's aggregate (fedavg_trainer.py:450-457) AND its :291 sums of
    squares in one pass over fp32 rows: returns ``(out, sumsq)`` with ``out``
    the bits of ``reduce_packed(clients, weights, P)`` and ``sumsq`` [K]
    float64 device sums as ``client_sqdist(clients, out, P)`` forms them.
    K <= 1024 reads the rows once (fedavg_reduce_sqdist_f32); larger K runs
    the two passes inside the same call."""
    K, ld, P, dtype, out = _check_packed(clients, weights, P, out)
    if dtype != torch.float32:
        raise TypeError("reduce_with_sqdist: fp32 rows only (other dtypes: reduce_packed + client_sqdist)")
    lib = _lib.load()
    n_ws = lib.fedavg_reduce_sqdist_workspace(K, P)
    work = torch.empty(max(n_ws, 1), dtype=torch.float64, device=clients.device)
    sumsq = torch.empty(K, dtype=torch.float64, device=clients.device)
    rc = lib.fedavg_reduce_sqdist_f32(clients.data_ptr(), K, P, ld, weights.data_ptr(), out.data_ptr(),
                                      work.data_ptr(), n_ws, sumsq.data_ptr(), _stream_handle(stream, clients.device))
    _lib.check(rc, "fedavg_reduce_sqdist_f32")
    return out, sumsq
