"""The native host code under AddressSanitizer + UndefinedBehaviorSanitizer (no GPU).

* ``tests/native/staging_fuzz.cpp`` (always): g++ builds the HIP-free staging
  header (``csrc/staging.hpp``: the workspace sizes and the host writes of
  fedavg_device_round_f32, stage_tables and fedavg_pack_rows_device) and the
  host packer (``csrc/fedavg_host.cpp``) with ``-fsanitize=address,undefined``
  and fuzzes key counts 1..5,000, client counts 1..1,024 and every plan form
  (tiles with and without the unit map, every window instance with its
  descriptor table, the split-row windows): every staged byte must lie inside
  the reserved room and below the bytes the H2D ships.  Reintroducing round
  5's descriptor-table overrun (dropping ``dbytes <= L.desc_room``) makes
  ASan abort here.
* ``fedavg_collect_ext`` (the state_dict walk, ``verify_rows``) built with
  ``-fsanitize=address,undefined`` and the CPU suites that drive it run under
  ``LD_PRELOAD=libasan`` -- opt-in (``MFL_ASAN_TESTS=1``; it compiles a torch
  extension, ~1 minute).  README.md has the one-line recipe.
"""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "mobile-federated-learning_amd" / "csrc"
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


def _gxx():
    return shutil.which("g++")


@pytest.mark.skipif(_gxx() is None, reason="g++ not found")
def test_staging_and_packer_fuzz_under_asan_ubsan(tmp_path):
    exe = tmp_path / "staging_fuzz"
    cmd = [_gxx(), "-std=c++17", "-O1", "-g", *SAN, f"-I{ROOT / 'include'}", f"-I{CSRC}",
           str(ROOT / "tests" / "native" / "staging_fuzz.cpp"), str(CSRC / "fedavg_host.cpp"), "-pthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    for seed in (1234, 99):
        r = subprocess.run([str(exe), "60", str(seed)], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "0 failures" in r.stdout and "ERROR" not in r.stderr, r.stdout + r.stderr


def _gcc_lib(name):
    out = subprocess.run([_gxx(), f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return out if out and os.path.isabs(out) and os.path.exists(out) else None


@pytest.mark.skipif(os.environ.get("MFL_ASAN_TESTS") != "1" or _gxx() is None,
                    reason="opt-in: MFL_ASAN_TESTS=1 (builds an ASan torch extension, ~1 min)")
def test_collect_ext_suites_under_asan(tmp_path):
    """fedavg_collect_ext.cpp with -fsanitize=address,undefined, loaded through
    FEDAVG_COLLECT_EXT_PATH, under LD_PRELOAD=libasan: test_verify_rows.py,
    test_host_logic.py and test_autostream.py (the walk, verify_rows with the
    :199 copies' identities) must pass with no sanitizer report."""
    asan, stdcxx = _gcc_lib("libasan.so"), _gcc_lib("libstdc++.so")
    assert asan and stdcxx, "libasan.so / libstdc++.so not found"
    # libstdc++ right after the runtime: ASan's __cxa_throw interceptor needs
    # the real one resolvable at start-up (python does not link libstdc++)
    preload = f"{asan} {stdcxx}"
    build = tmp_path / "asan_ext"
    build.mkdir()
    script = (
        "from torch.utils.cpp_extension import load\n"
        f"load(name='fedavg_collect_ext', sources=[{str(CSRC / 'fedavg_collect_ext.cpp')!r}], "
        f"build_directory={str(build)!r}, extra_cflags=['-O1', '-g', '-fopenmp', {SAN[0]!r}, {SAN[2]!r}], "
        f"extra_ldflags=['-fopenmp', {SAN[0]!r}], verbose=False)\n")
    env = dict(os.environ, LD_PRELOAD=preload, ASAN_OPTIONS="detect_leaks=0:alloc_dealloc_mismatch=0")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    ext = build / "fedavg_collect_ext.so"
    assert ext.exists()
    env["FEDAVG_COLLECT_EXT_PATH"] = str(ext)
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        str(ROOT / "tests" / "test_verify_rows.py"), str(ROOT / "tests" / "test_host_logic.py"),
                        str(ROOT / "tests" / "test_autostream.py")],
                       capture_output=True, text=True, timeout=1800, env=env, cwd=ROOT)
    out = r.stdout[-4000:] + r.stderr[-4000:]
    assert r.returncode == 0, out
    assert "AddressSanitizer" not in out and "runtime error" not in out, out
