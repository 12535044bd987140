"""Build recipe for libfedavg_amd.so (gfx950 only).

    python -m mfl_amd.build           # or __graft_entry__.build()

Compiles the HIP translation units in ``csrc/`` (``fedavg_reduce.hip``:
production kernels + C ABI; ``fedavg_variants.hip``: benchmarking variants;
``fedavg_dist.hip``: the distance pass) and ``csrc/fedavg_host.cpp`` (native
host packer) in parallel with hipcc for ``--offload-arch=gfx950`` and links
them into ``lib/libfedavg_amd.so`` inside the package (in-tree, so the built
library travels with the repo snapshot to the GPU box).  ``-ffp-contract=off``
keeps every multiply and add separately rounded (bit parity with the
reference's ATen CPU ops, fedavg_trainer.py:455-457).
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
HIP_SOURCES = [CSRC_DIR / "fedavg_reduce.hip", CSRC_DIR / "fedavg_variants.hip", CSRC_DIR / "fedavg_dist.hip",
               CSRC_DIR / "fedavg_fpf.hip", CSRC_DIR / "fedavg_xfer.hip", CSRC_DIR / "fedavg_pack.hip",
               CSRC_DIR / "fedavg_segments.hip"]
CSRC_HOST = CSRC_DIR / "fedavg_host.cpp"
CSRC_COMMON = CSRC_DIR / "common.hpp"
CSRC_COLLECT = CSRC_DIR / "fedavg_collect_ext.cpp"
COLLECT_NAME = "fedavg_collect_ext"
INCLUDE = REPO_DIR / "include"
LIB_DIR = PKG_DIR / "lib"
OBJ_DIR = LIB_DIR / "obj"
LIB_PATH = LIB_DIR / "libfedavg_amd.so"
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
    return [*HIP_SOURCES, CSRC_HOST, CSRC_COMMON, INCLUDE / "fedavg_amd.h", INCLUDE / "fedavg_amd_tuning.h",
            Path(__file__)]


def up_to_date() -> bool:
    if not LIB_PATH.exists():
        return False
    t = LIB_PATH.stat().st_mtime
    return all(p.stat().st_mtime <= t for p in sources())


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
         extra_cflags=["-O2"], verbose=verbose)
    return out


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and up_to_date():
        return LIB_PATH
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    hipcc = hipcc_path()
    procs = []
    objs = []
    for src in [*HIP_SOURCES, CSRC_HOST]:
        obj = OBJ_DIR / (src.name + ".o")
        cmd = [hipcc, *HIPCC_FLAGS, f"-I{INCLUDE}", "-c", "-o", str(obj), str(src)]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
        objs.append(obj)
    errors = []
    for src, proc in procs:
        out, err = proc.communicate()
        if proc.returncode != 0:
            errors.append(f"{src.name}: hipcc failed ({proc.returncode}):\n{out}\n{err}")
    if errors:
        raise RuntimeError("\n".join(errors))
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"link failed ({proc.returncode}):\n{proc.stdout}\n{proc.stderr}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
