"""The C-ABI library loads and exports every symbol include/*.h declares.

CPU only: argument validation runs before any HIP call, so rejected calls and
the host-side weight helper can be exercised without a GPU.
"""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

import mfl_amd
from mfl_amd import _lib, build

INCLUDE = Path(__file__).resolve().parents[1] / "include"


def declared_functions(headers=("fedavg_amd.h", "fedavg_amd_tuning.h")):
    names = []
    for h in [INCLUDE / n for n in headers]:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(fedavg_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    build.build()
    return _lib.load()


def test_header_parse_finds_entry_points():
    names = declared_functions()
    for required in ("fedavg_reduce_f32", "fedavg_reduce_ptrs_f32", "fedavg_reduce_f64", "fedavg_reduce_f16",
                     "fedavg_reduce_bf16", "fedavg_reduce_splitk_f32", "fedavg_last_error", "fedavg_weights_f32",
                     "fedavg_abi_version", "fedavg_reduce_f32_tuned", "fedavg_f32_schedule_ld"):
        assert required in names


def _exported(path):
    import subprocess
    nm = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True, check=True).stdout
    return sorted({ln.split()[-1] for ln in nm.splitlines() if ln.split() and ln.split()[-1].startswith("fedavg_")})


def test_library_exports_every_declared_symbol(lib):
    raw = ctypes.CDLL(str(_lib.library_path()))
    for name in declared_functions(("fedavg_amd.h",)):
        assert hasattr(raw, name), name
        assert name in _lib.SIGNATURES, f"{name} declared but not typed in _lib.SIGNATURES"


def test_every_exported_entry_point_is_declared(lib):
    """The reverse direction: the product .so exports exactly what
    include/fedavg_amd.h declares -- no tuning hook leaks into it."""
    exported = _exported(_lib.library_path())
    assert exported == declared_functions(("fedavg_amd.h",))


def test_probe_library_exports_product_and_tuning_hooks(lib):
    """libfedavg_amd_probe.so = the product entry points + every hook of
    include/fedavg_amd_tuning.h, each typed in _lib.TUNING_SIGNATURES."""
    probe = _lib.load_probe()
    assert probe is not lib
    exported = _exported(_lib.PROBE_LIB_PATH)
    assert exported == declared_functions()
    for name in declared_functions(("fedavg_amd_tuning.h",)):
        assert name in _lib.TUNING_SIGNATURES, name
        assert name not in _lib.SIGNATURES, name


def test_library_is_gfx950_code_object():
    data = _lib.library_path().read_bytes()
    assert b"gfx950" in data


def test_abi_version(lib):
    assert lib.fedavg_abi_version() == _lib.ABI_VERSION


@pytest.mark.parametrize("K,P,ld", [(0, 10, 10), (-1, 10, 10), (2, 10, 5), (2, -1, 0)])
def test_rejects_bad_sizes_without_gpu(lib, K, P, ld):
    rc = lib.fedavg_reduce_f32(None, K, P, ld, None, None, None)
    assert rc == _lib.FEDAVG_EINVAL
    assert lib.fedavg_last_error().startswith(b"fedavg_reduce_f32")


def test_null_buffers_rejected(lib):
    assert lib.fedavg_reduce_f64(None, 2, 8, 8, None, None, None) == _lib.FEDAVG_EINVAL
    assert lib.fedavg_reduce_bf16(None, 2, 8, 8, None, None, None) == _lib.FEDAVG_EINVAL
    assert lib.fedavg_reduce_ptrs_f32(None, 2, 8, None, None, None) == _lib.FEDAVG_EINVAL


def test_p_zero_is_noop(lib):
    assert lib.fedavg_reduce_f32(None, 3, 0, 0, None, None, None) == 0


def test_splitk_bad_mode(lib):
    buf = np.zeros(64, np.float32)
    w = np.ones(2, np.float32)
    out = np.zeros(32, np.float32)
    # validation happens before launch; an unsupported split count is refused
    rc = lib.fedavg_reduce_splitk_f32(buf.ctypes.data, 2, 32, 32, w.ctypes.data, out.ctypes.data, 3, None)
    assert rc in (_lib.FEDAVG_EMODE, _lib.FEDAVG_EALIGN)


@pytest.mark.parametrize("dpitch,spitch,width,rows", [(64, 64, 128, 2), (128, 32, 64, 2), (64, 64, 64, -1),
                                                      (64, 64, -4, 2)])
def test_upload_shard_rejects_bad_sizes_without_gpu(lib, dpitch, spitch, width, rows):
    rc = lib.fedavg_upload_shard(None, dpitch, None, spitch, width, rows, None)
    assert rc == _lib.FEDAVG_EINVAL
    assert lib.fedavg_last_error().startswith(b"fedavg_upload_shard")


def test_upload_shard_empty_is_noop_and_null_rejected(lib):
    assert lib.fedavg_upload_shard(None, 64, None, 64, 0, 5, None) == 0
    assert lib.fedavg_upload_shard(None, 64, None, 64, 64, 0, None) == 0
    assert lib.fedavg_upload_shard(None, 64, None, 64, 64, 3, None) == _lib.FEDAVG_EINVAL


def test_weights_helper_matches_python(lib):
    rng = np.random.default_rng(7)
    for K in (1, 2, 3, 10, 100, 1000):
        n = rng.integers(0, 10**6, size=K).astype(np.int64)
        n[0] = max(n[0], 1)
        w = np.zeros(K, np.float32)
        assert lib.fedavg_weights_f32(n.ctypes.data, K, w.ctypes.data) == 0
        expect = np.array(mfl_amd.sample_weights([int(v) for v in n]), dtype=np.float64).astype(np.float32)
        assert w.tobytes() == expect.tobytes()


def test_device_round_sizes_without_gpu(lib):
    """fedavg_device_round_workspace / _scratch (host arithmetic, no GPU):
    the workspace holds the key table, the padded key-major pointer table,
    the fp32 weights, the integer keys' tables and the unit map's room; the
    scratch is K rows of the integer / bool keys' columns, each 4-aligned."""
    numel = np.array([432, 16, 1, 0, 7, 36864], dtype=np.int64)
    kind = np.array([0, 0, 1, 2, 6, 0], dtype=np.int64)  # fp32, fp32, int64, int32 (empty), bool, fp32
    for K in (1, 5, 100, 256):
        n = len(numel)
        ws = lib.fedavg_device_round_workspace(K, n)
        tables = n * 32 + (n * K + 128) * 8 + K * 4 + n * 24 + n * K * 8
        assert tables + 65536 * 4 <= ws <= tables + 65536 * 4 + 64 and ws % 16 == 0
        assert lib.fedavg_device_round_scratch(numel.ctypes.data, kind.ctypes.data, n, K) == K * (4 + 8)
    assert lib.fedavg_device_round_workspace(0, 3) == 0
    assert lib.fedavg_device_round_scratch(None, None, 3, 4) == 0


def test_weights_helper_zero_total(lib):
    n = np.zeros(3, np.int64)
    w = np.zeros(3, np.float32)
    assert lib.fedavg_weights_f32(n.ctypes.data, 3, w.ctypes.data) == _lib.FEDAVG_EINVAL
    assert b"ZeroDivisionError" in lib.fedavg_last_error()


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No silent fallback: without the .so every product entry raises."""
    import torch

    monkeypatch.setattr(_lib, "LIB_PATH", tmp_path / "libfedavg_amd.so")
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.FedAvgLibraryError):
        _lib.load()
    # the drop-in refuses too (before or at device use), never computing on the CPU
    from collections import OrderedDict
    w_locals = [(1, OrderedDict(w=torch.ones(4))), (3, OrderedDict(w=torch.zeros(4)))]
    with pytest.raises((_lib.FedAvgLibraryError, RuntimeError)):
        mfl_amd.aggregate(w_locals)
    assert torch.equal(w_locals[0][1]["w"], torch.ones(4))  # nothing was written


def test_plain_c_consumer_builds(lib):
    """examples/c_abi_demo.c links against the library with only the C header
    (no Python, no torch): the boundary is usable from a non-Python host."""
    import subprocess
    root = INCLUDE.parent
    proc = subprocess.run(["make", "-s", "-B", "-C", str(root / "examples"), "c_abi_demo"],
                          capture_output=True, text=True, timeout=120)
    assert proc.returncode == 0, proc.stderr
    assert (root / "examples" / "c_abi_demo").exists()
