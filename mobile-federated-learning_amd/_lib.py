"""ctypes binding of libfedavg_amd.so (the C ABI in include/fedavg_amd.h).

There is no fallback: if the HIP library is missing or does not export the
declared entry points, every product call raises ``FedAvgLibraryError``.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path

from .build import LIB_PATH, PROBE_LIB_PATH

_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_vp = ctypes.c_void_p
_c_float = ctypes.c_float

# name -> (restype, argtypes); mirrors include/fedavg_amd.h
SIGNATURES = {
    "fedavg_abi_version": (_c_int, []),
    "fedavg_last_error": (ctypes.c_char_p, []),
    "fedavg_reduce_f32": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp]),
    "fedavg_reduce_f32_timed": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp]),
    "fedavg_reduce_ptrs_f32": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp]),
    "fedavg_reduce_f64": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp]),
    "fedavg_reduce_f16": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp]),
    "fedavg_reduce_bf16": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp]),
    "fedavg_reduce_splitk_f32": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _vp]),
    "fedavg_weights_f32": (_c_int, [_vp, _c_i64, _vp]),
    "fedavg_pack_rows": (_c_int, [_vp, _c_i64, _vp, _c_i64, _c_int]),
    "fedavg_pack_rows_device_workspace": (_c_i64, [_c_i64]),
    "fedavg_segments_workspace": (_c_i64, [_c_i64, _c_i64]),
    "fedavg_segments_partials": (_c_i64, [_vp, _c_i64, _c_i64]),
    "fedavg_reduce_segments_f32": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_i64, _vp]),
    "fedavg_client_sqdist_segments_f32": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _vp,
                                                   _vp, _c_i64, _vp]),
    "fedavg_reduce_sqdist_segments_partials": (_c_i64, [_c_i64]),
    "fedavg_reduce_sqdist_segments_f32": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _vp,
                                                   _vp, _vp, _c_i64, _vp]),
    "fedavg_pack_rows_device": (_c_int, [_vp, _c_i64, _vp, _c_i64, _vp, _vp, _c_i64, _vp]),
    "fedavg_device_round_workspace": (_c_i64, [_c_i64, _c_i64]),
    "fedavg_device_round_scratch": (_c_i64, [_vp, _vp, _c_i64, _c_i64]),
    "fedavg_device_round_f32": (_c_int, [_vp, _c_i64, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _vp,
                                         _vp, _c_i64, _vp, _vp, _c_i64, _vp]),
    "fedavg_round_f32": (_c_int, [_vp, _c_i64, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_int,
                                  _vp]),
    "fedavg_client_sqdist_workspace": (_c_i64, [_c_i64, _c_i64]),
    "fedavg_client_sqdist_f32": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _vp]),
    "fedavg_client_sqdist_workspace_elems": (_c_i64, [_c_i64, _c_i64, _c_i64]),
    "fedavg_reduce_sqdist_workspace": (_c_i64, [_c_i64, _c_i64]),
    "fedavg_fused_plan_of": (_c_i64, [_c_i64, _c_i64]),
    "fedavg_reduce_sqdist_f32": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _vp, _vp]),
    "fedavg_client_sqdist_f64": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _vp]),
    "fedavg_client_sqdist_f16": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _vp]),
    "fedavg_client_sqdist_bf16": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _vp]),
    "fedavg_fpf_set_rows_f32": (_c_int, [_vp, _c_i64, _c_i64, _vp, _c_i64, _vp, _c_i64, _vp, _c_i64, _vp]),
    "fedavg_fpf_workspace": (_c_i64, [_c_i64]),
    "fedavg_fpf_end_round_f32": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_i64, _c_float, _vp, _c_i64,
                                          _vp]),
    "fedavg_fpf_update_g": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_float, _c_int, _c_float, _vp]),
    "fedavg_fpf_index_f32": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "fedavg_fpf_index_lru": (_c_int, [_vp, _vp, _c_i64, _vp, _vp]),
    "fedavg_fpf_cat_diff": (_c_int, [_vp, _c_i64, _c_i64, _vp, _c_i64, _vp, _vp, _c_i64, _vp, _c_i64, _c_int, _vp]),
    "fedavg_fpf_end_round_promoted": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _c_int, _c_float, _vp,
                                               _c_i64, _vp]),
    "fedavg_fpf_index_f64": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "fedavg_copy_to_host": (_c_int, [_vp, _vp, _c_i64, _c_int, _vp]),
    "fedavg_upload_shard": (_c_int, [_vp, _c_i64, _vp, _c_i64, _c_i64, _c_i64, _vp]),
    "fedavg_f32_schedule": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "fedavg_f32_schedule_ld": (_c_int, [_c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp]),
}

# exported only by libfedavg_amd_probe.so (include/fedavg_amd_tuning.h)
TUNING_SIGNATURES = {
    "fedavg_reduce_f32_buf": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp]),
    "fedavg_reduce_segments_f32_variant": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_i64,
                                                    _c_int, _c_int, _c_int, _vp]),
    "fedavg_client_sqdist_segments_f32_variant": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp,
                                                           _vp, _vp, _c_i64, _c_int, _c_int, _vp]),
    "fedavg_device_round_phases": (_c_int, [_vp, _c_int]),
    "fedavg_fpf_index_workspace": (_c_i64, [_c_i64, _c_i64]),
    "fedavg_fpf_index_variant": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_i64, _c_int, _c_int,
                                          _c_int, _vp]),
    "fedavg_probe_cvt16": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp]),
    "fedavg_reduce_f32_tuned": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _c_int, _vp]),
    "fedavg_reduce_f32_variant": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _c_int, _c_int, _c_int,
                                           _c_int, _vp]),
    "fedavg_reduce_half_variant": (_c_int, [_c_int, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _c_int, _c_int,
                                            _vp]),
    "fedavg_half_schedule": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "fedavg_client_sqdist_variant": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _c_int, _c_int,
                                              _c_int, _vp]),
    "fedavg_client_sqdist_buf": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _c_int, _c_int,
                                          _c_int, _vp]),
    "fedavg_reduce_sqdist_f32_variant": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _vp, _c_int,
                                                  _c_int, _vp]),
    "fedavg_reduce_vec_buf": (_c_int, [_c_int, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _c_int, _c_int, _vp]),
    "fedavg_probe_busy_copy": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_int, _vp]),
    "fedavg_probe_clock": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp]),
    "fedavg_stream_create_masked": (_c_int, [_c_int, _c_int, _vp]),
    "fedavg_stream_destroy": (_c_int, [_vp]),
    "fedavg_reduce_f32_xcd": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_int, _vp]),
    "fedavg_probe_read_f32x4": (_c_int, [_vp, _c_i64, _c_int, _c_int, _c_int, _vp, _vp]),
    "fedavg_reduce_tiled_f32": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _c_int, _vp]),
}

ABI_VERSION = 1

FEDAVG_EINVAL = -10001
FEDAVG_EALIGN = -10002
FEDAVG_EMODE = -10003


class FpfGroups(ctypes.Structure):
    """fedavg_fpf_groups (include/fedavg_amd.h): row 0 of each dtype group,
    its row stride in elements, its kind (0 fp32, 1 fp64, 2 fp16, 3 bf16)."""

    _fields_ = [("base", ctypes.c_void_p * 4), ("ld", ctypes.c_int64 * 4), ("kind", ctypes.c_int32 * 4)]


class FedAvgLibraryError(RuntimeError):
    """libfedavg_amd.so is missing, stale, or a call into it failed."""


_lock = threading.Lock()
_lib = None
_probe = None


def library_path() -> Path:
    return LIB_PATH


def load() -> ctypes.CDLL:
    """Load (once) and type the HIP library; raise loudly if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise FedAvgLibraryError(
                f"{LIB_PATH} not built: run __graft_entry__.build() (hipcc --offload-arch=gfx950); "
                "there is no CPU fallback for the FedAvg reduction"
            )
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError as e:
                raise FedAvgLibraryError(f"{LIB_PATH} does not export {name}") from e
            fn.restype = res
            fn.argtypes = args
        ver = lib.fedavg_abi_version()
        if ver != ABI_VERSION:
            raise FedAvgLibraryError(f"ABI version {ver} != expected {ABI_VERSION}; rebuild the library")
        _lib = lib
    return _lib


def load_probe() -> ctypes.CDLL:
    """The probe library (product entry points + the tuning hooks of
    include/fedavg_amd_tuning.h).  Scripts and variant tests only; the
    product path never loads it."""
    global _probe
    if _probe is not None:
        return _probe
    with _lock:
        if _probe is not None:
            return _probe
        if not PROBE_LIB_PATH.exists():
            raise FedAvgLibraryError(f"{PROBE_LIB_PATH} not built: run __graft_entry__.build()")
        lib = ctypes.CDLL(str(PROBE_LIB_PATH))
        for name, (res, args) in {**SIGNATURES, **TUNING_SIGNATURES}.items():
            try:
                fn = getattr(lib, name)
            except AttributeError as e:
                raise FedAvgLibraryError(f"{PROBE_LIB_PATH} does not export {name}") from e
            fn.restype = res
            fn.argtypes = args
        _probe = lib
    return _probe


def f32_schedule(K: int, P: int, ld: int = 0) -> dict:
    """The schedule fedavg_reduce_f32 picks for an aligned [K, P] problem
    (P columns of rows with stride ld, when given)."""
    vals = [ctypes.c_int() for _ in range(4)]
    if ld:
        check(load().fedavg_f32_schedule_ld(K, P, ld, *[ctypes.byref(v) for v in vals]), "fedavg_f32_schedule_ld")
    else:
        check(load().fedavg_f32_schedule(K, P, *[ctypes.byref(v) for v in vals]), "fedavg_f32_schedule")
    sc = dict(zip(("unroll", "cols", "nontemporal", "launches"), (v.value for v in vals)))
    # launch_production_f32 (csrc/fedavg_reduce.hip): nontemporal == 2 marks
    # the per-row buffer-descriptor kernel (nontemporal loads), 1 / 0 the
    # global-pointer variant kernel with / without them; 256-thread workgroups
    sc["kernel"] = "reduce_f32x4_buf_kernel" if sc["nontemporal"] == 2 else "reduce_f32x4_var_kernel"
    sc["block"] = 256
    return sc


def check(rc: int, what: str, lib: ctypes.CDLL = None) -> None:
    """Raise on a non-zero status; the message comes from the library that
    made the call (``lib``; default: the product library, or the probe
    library when only that one is loaded)."""
    if rc != 0:
        src = lib if lib is not None else (_lib if _lib is not None or _probe is None else _probe)
        if src is None:
            src = load()
        msg = src.fedavg_last_error().decode(errors="replace")
        raise FedAvgLibraryError(f"{what} failed (rc={rc}): {msg}")
