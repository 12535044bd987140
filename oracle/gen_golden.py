"""Generate golden vectors for the FedAvg reduction by running the REFERENCE.

Test infrastructure, run by hand in the build container only (the reference
is not present on the GPU box):

    python oracle/gen_golden.py            # writes tests/golden/*.npz

It imports ``FedAvgTrainer`` from ``/root/reference/src/fedavg_trainer.py``
(read-only, never copied) and calls ``FedAvgTrainer.aggregate``
(``fedavg_trainer.py:441-458``) on seeded synthetic client state_dicts.  The
reference imports ``wandb`` and ``hwcounter``, which are not installed here,
so tiny stub modules are written to a temp dir; ``config.py`` reads
``../data/*.csv`` relative to the CWD (``config.py:10,14-17``) and creates
``result/`` under the CWD (``config.py:34-36``), so the import runs in a temp
dir with ``data`` symlinked to the reference's CSVs.  Only data (inputs and
the reference's outputs) is written to ``tests/golden``.

Each ``.npz`` holds ``meta`` (JSON: case name, sample counts, key table,
whether the result aliased ``w_locals[0][1]``, sha256 of every output),
``in__<client>__<key>`` inputs and ``out__<key>`` outputs.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import textwrap
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
REF_SRC = Path("/root/reference/src")
REF_DATA = Path("/root/reference/data")
OUT_DIR = REPO / "tests" / "golden"

_STUB_WANDB = """
class _Cfg(dict):
    def update(self, *a, **k):
        pass
config = _Cfg()
def init(*a, **k):
    return None
def log(*a, **k):
    return None
def save(*a, **k):
    return None
"""

_STUB_HWCOUNTER = """
import time
def count():
    return time.perf_counter_ns()
def count_end():
    return time.perf_counter_ns()
class Timer:
    def __enter__(self):
        self.start = time.perf_counter_ns()
        return self
    def __exit__(self, *exc):
        self.cycles = time.perf_counter_ns() - self.start
        return False
"""

# The child process: build cases, run the reference aggregate, save npz.
_CHILD = r'''
import copy, hashlib, json, sys, types
from collections import OrderedDict
import numpy as np
import torch

import fedavg_trainer  # /root/reference/src/fedavg_trainer.py
ref_aggregate = fedavg_trainer.FedAvgTrainer.aggregate

out_dir = sys.argv[1]

def client_dicts(K, keys, seed, dist="model"):
    """keys: list of (name, shape, dtype-str).  Client k = base + small noise."""
    rng = np.random.default_rng(seed)
    base = {}
    for name, shape, dt in keys:
        if dt in ("int64", "int32", "uint8", "bool"):
            base[name] = None
        else:
            base[name] = rng.normal(0.0, 0.05, size=shape)
    dicts = []
    for k in range(K):
        r = np.random.default_rng(seed * 1000 + 1000 + k)
        sd = OrderedDict()
        for name, shape, dt in keys:
            if dt == "int64":
                v = r.integers(0, 1000, size=shape)
                sd[name] = torch.tensor(v, dtype=torch.int64)
            elif dt == "int64big":
                v = r.integers(2**30, 2**40, size=shape)
                sd[name] = torch.tensor(v, dtype=torch.int64)
            elif dt == "int32":
                sd[name] = torch.tensor(r.integers(-5000, 5000, size=shape), dtype=torch.int32)
            elif dt == "uint8":
                sd[name] = torch.tensor(r.integers(0, 256, size=shape), dtype=torch.uint8)
            elif dt == "bool":
                sd[name] = torch.tensor(r.integers(0, 2, size=shape).astype(bool))
            else:
                if dist == "adversarial":
                    v = r.normal(0.0, 1.0, size=shape) * r.uniform(0.01, 10.0, size=shape)
                else:
                    v = base[name] + r.normal(0.0, 1e-3, size=shape)
                tdt = {"float32": torch.float32, "float64": torch.float64,
                       "float16": torch.float16, "bfloat16": torch.bfloat16}[dt]
                sd[name] = torch.tensor(v, dtype=torch.float64).to(tdt)
        dicts.append(sd)
    return dicts

def np_of(t):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().copy(), "bfloat16"
    return t.numpy().copy(), str(t.dtype).replace("torch.", "")

def save_case(name, sample_nums, dicts, self_obj=None, note=""):
    w_locals = [(n, d) for n, d in zip(sample_nums, dicts)]
    saved_inputs = copy.deepcopy(w_locals)
    first = w_locals[0][1] if w_locals else None
    result = ref_aggregate(self_obj if self_obj is not None else types.SimpleNamespace(), w_locals)
    arrays = {}
    in_keys = []
    for i, (n, sd) in enumerate(saved_inputs):
        for key, t in sd.items():
            a, dts = np_of(t)
            arrays[f"in__{i}__{key}"] = a
            if i == 0:
                in_keys.append({"name": key, "shape": list(t.shape), "dtype": dts})
    out_keys = []
    for key, t in result.items():
        a, dts = np_of(t)
        arrays[f"out__{key}"] = a
        out_keys.append({"name": key, "shape": list(t.shape), "dtype": dts,
                         "sha256": hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()})
    meta = {
        "case": name,
        "note": note,
        "K": len(sample_nums),
        "sample_nums": [n if isinstance(n, int) else float(n) for n in sample_nums],
        "sample_num_types": [type(n).__name__ for n in sample_nums],
        "in_keys": in_keys,
        "out_keys": out_keys,
        "aliased": bool(first is not None and result is first),
        "generator": "oracle/gen_golden.py (reference FedAvgTrainer.aggregate, fedavg_trainer.py:441-458)",
        "torch": torch.__version__,
    }
    arrays["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(f"{out_dir}/{name}.npz", **arrays)
    print(f"{name}: K={len(sample_nums)} keys={len(out_keys)} aliased={meta['aliased']}")

def counts(K, seed, lo=1, hi=1000):
    return [int(v) for v in np.random.default_rng(seed).integers(lo, hi + 1, size=K)]

# --- single-key shape sweep (tails around float4 / 64-element boundaries)
for K, P in [(1, 1), (2, 3), (3, 4), (3, 63), (10, 64), (10, 65), (5, 257), (7, 1000)]:
    save_case(f"flat_k{K}_p{P}", counts(K, 1234 + K + P), client_dicts(K, [("w", [P], "float32")], seed=K * 7 + P))

# --- model-shaped: MNIST + LR (FedML LogisticRegression 784 -> 10), K = 10
save_case("mnist_lr_k10", counts(10, 1234),
          client_dicts(10, [("linear.weight", [10, 784], "float32"), ("linear.bias", [10], "float32")], seed=1),
          note="cfg1 shape: P = 7,850")

# --- K = 100 clients (cfg3's client count) on the MNIST+LR shape
save_case("mnist_lr_k100", counts(100, 99),
          client_dicts(100, [("linear.weight", [10, 784], "float32"), ("linear.bias", [10], "float32")], seed=2))

# --- conv/BN-shaped dict with int64 num_batches_tracked buffers (resnet-like)
bn_keys = []
for b in range(3):
    bn_keys += [(f"layer{b}.conv.weight", [8, 4, 3, 3], "float32"),
                (f"layer{b}.bn.weight", [8], "float32"),
                (f"layer{b}.bn.bias", [8], "float32"),
                (f"layer{b}.bn.running_mean", [8], "float32"),
                (f"layer{b}.bn.running_var", [8], "float32"),
                (f"layer{b}.bn.num_batches_tracked", [], "int64")]
bn_keys += [("fc.weight", [10, 8], "float32"), ("fc.bias", [10], "float32")]
save_case("resnet_like_bn_k5", counts(5, 5), client_dicts(5, bn_keys, seed=3),
          note="int64 scalar buffers are promoted to fp32 by the reference")

# --- survey-verified int64 promotion example: nbt 7,8,9 with n = 10,20,30
sds = []
for v in (7, 8, 9):
    sd = OrderedDict(); sd["nbt"] = torch.tensor(v, dtype=torch.int64); sds.append(sd)
save_case("int64_nbt_example", [10, 20, 30], sds)

# --- adversarial magnitudes, near-zero outputs, extreme sample counts
save_case("adversarial_k10", [1, 1000000, 3, 7, 1, 999983, 2, 65536, 5, 11],
          client_dicts(10, [("w", [4096], "float32")], seed=4, dist="adversarial"))

# --- non-representable weights
save_case("thirds_k3", [1, 1, 1], client_dicts(3, [("w", [129], "float32")], seed=5))
save_case("sixths_k3", [1, 2, 3], client_dicts(3, [("w", [2, 3, 5], "float32")], seed=6))

# --- float sample counts (Python division semantics)
save_case("float_counts_k4", [2.5, 0.75, 10.0, 1.125], client_dicts(4, [("w", [77], "float32")], seed=7))

# --- a zero sample count (weight exactly 0)
save_case("zero_count_k4", [0, 5, 0, 3], client_dicts(4, [("w", [100], "float32")], seed=8))

# --- IEEE specials: NaN, +-inf, subnormals, signed zeros, huge values
spec = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, -1e-45, 1.1754942e-38,
                 3.0e38, -3.0e38, 1.0, -1.0, 1e-30, 5e-39, 2.0**-126, 7.0], dtype=np.float32)
sds = []
for k in range(4):
    r = np.random.default_rng(900 + k)
    v = np.concatenate([np.roll(spec, k), r.normal(0, 1e-38, 48).astype(np.float32)])
    sd = OrderedDict(); sd["w"] = torch.tensor(v, dtype=torch.float32); sds.append(sd)
save_case("ieee_specials_k4", [3, 1, 4, 1], sds, note="NaN/inf/subnormal propagation")

# --- subnormal-producing products (tiny inputs x tiny weights)
sds = []
for k in range(3):
    r = np.random.default_rng(950 + k)
    sd = OrderedDict(); sd["w"] = torch.tensor(r.uniform(-1e-36, 1e-36, 256), dtype=torch.float32); sds.append(sd)
save_case("subnormal_products_k3", [1, 1000, 7], sds)

# --- large int64 values (int64 -> fp32 rounding) and other integer/bool dtypes
save_case("int_dtypes_k3", counts(3, 31),
          client_dicts(3, [("big", [40], "int64big"), ("i32", [9], "int32"),
                           ("u8", [17], "uint8"), ("flag", [5], "bool")], seed=9))

# --- 0-dim float key, fp64 key, fp16 / bf16 keys (dtype-preserving paths)
save_case("scalar_key_k3", counts(3, 41), client_dicts(3, [("s", [], "float32"), ("v", [3], "float32")], seed=10))
save_case("float64_key_k3", counts(3, 51), client_dicts(3, [("d", [33], "float64"), ("f", [33], "float32")], seed=11))
save_case("float16_key_k3", counts(3, 61), client_dicts(3, [("h", [70], "float16")], seed=12))
save_case("bfloat16_key_k3", counts(3, 71), client_dicts(3, [("b", [70], "bfloat16")], seed=13))

# --- K = 1 on a multi-key dict
save_case("single_client_k1", [17], client_dicts(1, bn_keys[:6], seed=14))

# --- state_dicts with no keys
save_case("no_keys_k2", [3, 4], [OrderedDict(), OrderedDict()])

# --- empty w_locals -> copy of the global model's CPU state (fedavg_trainer.py:442-443)
torch.manual_seed(0)
glob = torch.nn.Linear(5, 3)
save_case("empty_w_locals", [], [], self_obj=types.SimpleNamespace(model_global=glob))
'''


def main() -> int:
    if not (REF_SRC / "fedavg_trainer.py").exists():
        print("reference not present; golden vectors can only be generated in the build container")
        return 1
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory(prefix="fedavg_golden_") as tmp:
        tmp = Path(tmp)
        stubs = tmp / "stubs"
        stubs.mkdir()
        (stubs / "wandb.py").write_text(textwrap.dedent(_STUB_WANDB))
        (stubs / "hwcounter.py").write_text(textwrap.dedent(_STUB_HWCOUNTER))
        (tmp / "data").symlink_to(REF_DATA)
        run = tmp / "run"
        run.mkdir()
        child = tmp / "child.py"
        child.write_text(_CHILD)
        env = dict(os.environ)
        env["PYTHONPATH"] = f"{stubs}:{REF_SRC}"
        env["PYTHONDONTWRITEBYTECODE"] = "1"
        env["CUDA_VISIBLE_DEVICES"] = ""
        proc = subprocess.run([sys.executable, str(child), str(OUT_DIR)], cwd=run, env=env)
        return proc.returncode


if __name__ == "__main__":
    sys.exit(main())
