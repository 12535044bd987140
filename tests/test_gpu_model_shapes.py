"""The drop-in on the BASELINE models' own state_dict layouts:

* cfg3 CIFAR10 + resnet56: K = 100 clients of 350 keys (58 int64
  ``num_batches_tracked`` buffers), P = 600,372 -- host clients through the
  native collect/packer, and device-resident clients through the zero-copy
  segments kernel with its small (1,024-column) units;
* cfg4 fed_cifar100 + resnet18_gn: K = 500 clients of 62 keys, P =
  11,227,812 (22.5 GB of client tensors) -- host and device-resident.

Each aggregate is compared bit for bit with the reference's torch loop
(oracle.aggregate_torch, fedavg_trainer.py:441-458) on the same tensors, and
the :291 distances (fedavg_trainer.py:291) with the accurate restatement
(oracle.client_distances_exact) within one fp32 unit.
"""
import sys
from collections import OrderedDict
from pathlib import Path

import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd
from test_gpu_parity import DEV, assert_bits

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "scripts"))
from model_shapes import CONFIGS  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield


def _clients(name, seed, device):
    """K state_dicts of the model's layout on ``device`` (generated on the GPU:
    base ~ N(0, 0.05^2) + per-client N(0, 1e-3^2); int64 buffers 1000 + i)."""
    K, shapes = CONFIGS[name]
    g = torch.Generator(device=DEV).manual_seed(seed)
    base = {k: torch.randn(s, generator=g, device=DEV) * 0.05 for k, s in shapes}
    out = []
    for i in range(K):
        sd = OrderedDict()
        for k, s in shapes:
            if k.endswith("num_batches_tracked"):
                t = torch.tensor(1000 + 3 * i, dtype=torch.int64, device=DEV)
            else:
                t = base[k] + torch.randn(s, generator=g, device=DEV) * 1e-3
            sd[k] = t.to(device)
        out.append(sd)
    counts = [int(c) for c in np.random.default_rng(seed).integers(1, 1000, size=K)]
    return list(zip(counts, out))


def _oracle(w_locals):
    """The reference loop on the same tensors (host copies), without touching the caller's dicts."""
    return O.aggregate_torch([(n, OrderedDict((k, v.cpu()) for k, v in sd.items())) for n, sd in w_locals])


def _check_distances(w_locals, out, max_checked=64):
    """All K distances from the GPU; the exact restatement on client 0, the
    last client and a seeded sample (its fp64 pass over 45 MB per client is
    slow on the host for K = 500)."""
    got = np.asarray(mfl_amd.client_distances(w_locals, out, device=DEV), dtype=np.float64)
    K = len(w_locals)
    idx = list(range(K)) if K <= max_checked else sorted(
        {0, K - 1, *np.random.default_rng(K).choice(K, max_checked - 2, replace=False).tolist()})
    host = [(w_locals[i][0], OrderedDict((k, v.cpu()) for k, v in w_locals[i][1].items())) for i in idx]
    exp = O.client_distances_exact(host, OrderedDict((k, v.cpu()) for k, v in out.items()))
    assert got[0] == 0.0  # w_locals[0][1] IS w_glob after the aggregate (fedavg_trainer.py:449)
    ulp = np.spacing(np.abs(exp).astype(np.float32)).astype(np.float64)
    err = np.abs(got[idx] - exp)
    assert np.all(err <= ulp), (err / np.maximum(ulp, 1e-300)).max()


@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("name", ["resnet56", "resnet18_gn"])
def test_model_shaped_dropin_bit_exact(name, where):
    torch.cuda.empty_cache()
    dev = torch.device("cpu") if where == "host" else DEV
    w_locals = _clients(name, 17 + (name == "resnet18_gn"), dev)
    K, shapes = CONFIGS[name]
    assert len(w_locals) == K and len(w_locals[0][1]) == len(shapes)
    expected = _oracle(w_locals)
    first = w_locals[0][1]
    out = mfl_amd.aggregate(w_locals, device=DEV)
    assert out is first
    assert list(out.keys()) == list(expected.keys())
    for k, e in expected.items():
        assert out[k].device.type == dev.type
        assert_bits(out[k], e, f"{name}/{where}/{k}")
    _check_distances(w_locals, out)
    del w_locals, out, expected
    torch.cuda.empty_cache()


def test_resnet56_streaming_session_bit_exact():
    """The same layout through a RoundSession (per-client pack + H2D at add)."""
    w_locals = _clients("resnet56", 23, torch.device("cpu"))
    expected = _oracle(w_locals)
    agg = mfl_amd.DeviceAggregator(DEV)
    sess = agg.begin_round(w_locals[0][1], len(w_locals))
    for n, sd in w_locals:
        sess.add(n, sd)
    out = sess.finish(w_locals)
    for k, e in expected.items():
        assert_bits(out[k], e, k)
    got = np.asarray(agg.client_distances(w_locals, out), dtype=np.float64)
    exp = O.client_distances_exact(w_locals, out)
    ulp = np.spacing(np.abs(exp).astype(np.float32)).astype(np.float64)
    assert np.all(np.abs(got - exp) <= ulp)
