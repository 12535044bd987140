"""Build recipe for libfedavg_amd.so and libfedavg_amd_probe.so (gfx950 only).

    python -m mfl_amd.build           # or __graft_entry__.build()

Compiles the HIP translation units in ``csrc/`` (``fedavg_reduce.hip``:
production kernels + C ABI; ``fedavg_dist.hip``: the distance pass; FPF,
transfer, device packing and zero-copy segment kernels) and
``csrc/fedavg_host.cpp`` (native host packer) in parallel with hipcc for
``--offload-arch=gfx950`` and links them into ``lib/libfedavg_amd.so`` inside
the package (in-tree, so the built library travels with the repo snapshot to
the GPU box).  ``-ffp-contract=off`` keeps every multiply and add separately
rounded (bit parity with the reference's ATen CPU ops,
fedavg_trainer.py:455-457).

The tuning hooks (``include/fedavg_amd_tuning.h``: kernel variants, probes)
are NOT in the product library.  The same sources plus
``fedavg_variants.hip``, compiled with ``-DFEDAVG_TUNING``, link into
``lib/libfedavg_amd_probe.so``, which scripts/ and the variant tests load.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC_DIR = PKG_DIR / "csrc"
# translation units of libfedavg_amd.so, compiled in parallel then linked
HIP_SOURCES = [CSRC_DIR / "fedavg_reduce.hip", CSRC_DIR / "fedavg_dist.hip",
               CSRC_DIR / "fedavg_fpf.hip", CSRC_DIR / "fedavg_xfer.hip", CSRC_DIR / "fedavg_pack.hip",
               CSRC_DIR / "fedavg_segments.hip"]
PROBE_SOURCES = [CSRC_DIR / "fedavg_variants.hip"]  # probe library only
CSRC_HOST = CSRC_DIR / "fedavg_host.cpp"
CSRC_COMMON = CSRC_DIR / "common.hpp"
CSRC_STAGING = CSRC_DIR / "staging.hpp"  # host-side staged layouts (also g++-built by tests/native)
CSRC_COLLECT = CSRC_DIR / "fedavg_collect_ext.cpp"
COLLECT_NAME = "fedavg_collect_ext"
INCLUDE = REPO_DIR / "include"
LIB_DIR = PKG_DIR / "lib"
OBJ_DIR = LIB_DIR / "obj"
PROBE_OBJ_DIR = LIB_DIR / "obj_probe"
LIB_PATH = LIB_DIR / "libfedavg_amd.so"
PROBE_LIB_PATH = LIB_DIR / "libfedavg_amd_probe.so"
ARCH = "gfx950"

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=off",
    "-fno-fast-math",
    "-Wall",
    "-pthread",
]


def hipcc_path() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libfedavg_amd.so)")


def sources():
    return [*HIP_SOURCES, *PROBE_SOURCES, CSRC_HOST, CSRC_COMMON, CSRC_STAGING, INCLUDE / "fedavg_amd.h",
            INCLUDE / "fedavg_amd_tuning.h", Path(__file__)]


def up_to_date() -> bool:
    for lib in (LIB_PATH, PROBE_LIB_PATH):
        if not lib.exists():
            return False
        t = lib.stat().st_mtime
        if any(p.stat().st_mtime > t for p in sources()):
            return False
    return True


def collect_ext_path() -> Path:
    return LIB_DIR / f"{COLLECT_NAME}.so"


def build_collect_ext(force: bool = False, verbose: bool = False) -> Path:
    """torch C++ extension for the host-side state_dict walk (layout.KeyTable.collect)."""
    out = collect_ext_path()
    if not force and out.exists() and out.stat().st_mtime >= CSRC_COLLECT.stat().st_mtime:
        return out
    from torch.utils.cpp_extension import load

    LIB_DIR.mkdir(parents=True, exist_ok=True)
    load(name=COLLECT_NAME, sources=[str(CSRC_COLLECT)], build_directory=str(LIB_DIR),
         extra_cflags=["-O2", "-fopenmp"], extra_ldflags=["-fopenmp"], verbose=verbose)
    return out


def _compile_all(jobs, verbose):
    """jobs: [(src, obj, extra_flags)] compiled in parallel (at most 16 at once)."""
    hipcc = hipcc_path()
    errors = []
    pending = list(jobs)
    running = []
    limit = max(1, min(16, os.cpu_count() or 8))
    while pending or running:
        while pending and len(running) < limit:
            src, obj, extra = pending.pop(0)
            cmd = [hipcc, *HIPCC_FLAGS, *extra, f"-I{INCLUDE}", "-c", "-o", str(obj), str(src)]
            if verbose:
                print(" ".join(cmd))
            running.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
        src, proc = running.pop(0)
        out, err = proc.communicate()
        if proc.returncode != 0:
            errors.append(f"{src.name}: hipcc failed ({proc.returncode}):\n{out}\n{err}")
    if errors:
        raise RuntimeError("\n".join(errors))


def _link(objs, lib_path, verbose):
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [hipcc_path(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"link failed ({proc.returncode}):\n{proc.stdout}\n{proc.stderr}")
    os.replace(tmp, lib_path)


def build(force: bool = False, verbose: bool = False) -> Path:
    """Build the product library and the probe library; returns the product path."""
    if not force and up_to_date():
        return LIB_PATH
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    PROBE_OBJ_DIR.mkdir(parents=True, exist_ok=True)
    jobs, objs, probe_objs = [], [], []
    for src in [*HIP_SOURCES, CSRC_HOST]:
        obj = OBJ_DIR / (src.name + ".o")
        jobs.append((src, obj, []))
        objs.append(obj)
    for src in [*HIP_SOURCES, *PROBE_SOURCES]:
        obj = PROBE_OBJ_DIR / (src.name + ".o")
        jobs.append((src, obj, ["-DFEDAVG_TUNING=1"]))
        probe_objs.append(obj)
    probe_objs.append(OBJ_DIR / (CSRC_HOST.name + ".o"))  # host packer: no tuning hooks
    _compile_all(jobs, verbose)
    _link(objs, LIB_PATH, verbose)
    _link(probe_objs, PROBE_LIB_PATH, verbose)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
