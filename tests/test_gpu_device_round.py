"""fedavg_device_round_f32: a device-resident round's fp32 group in one call.

The C-ABI entry the drop-in's device rounds take (aggregate.DeviceAggregator.
_device_round): the walk's address table [K, n_cols] (every key of the model,
the group's columns picked by key_index), the reference's weights as doubles
(fedavg_trainer.py:444-447, :453) and the key table go in; the average
(:450-457) and, fused, the :291 sums of squares come out.  Checked here
through the C ABI against the torch oracle: bit-exact averages, sums within
fp64 accumulation-order error of the exact fp64 sum of fl32(x - g)^2, the
"reduce only" return (1) for rounds that cannot fuse, integer keys
converted through the scratch, and the refusals.
"""
from collections import OrderedDict

import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd
from test_gpu_parity import assert_bits

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
EINVAL = -10001


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield


# (shape, dtype): fp32 keys around the window / tile widths, integer and bool
# keys (BatchNorm's num_batches_tracked), an empty key
_SPECS = [((64, 3, 3, 3), torch.float32), ((64,), torch.float32), ((), torch.int64), ((127,), torch.float32),
          ((129,), torch.float32), ((0,), torch.float32), ((5, 2), torch.bool), ((3000,), torch.float32),
          ((7,), torch.int32), ((1,), torch.float32), ((40_001,), torch.float32)]


def _clients(K, specs, seed, misalign_client=None):
    """K device clients, every tensor its own allocation (16-B aligned), or
    client `misalign_client`'s first fp32 key a view at a 4-B offset."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    out = []
    for i in range(K):
        sd = OrderedDict()
        for j, (shape, dt) in enumerate(specs):
            if dt == torch.float32:
                t = torch.randn(shape, generator=g, device=DEV) * 0.05
                if i == misalign_client and j == 0:
                    base = torch.empty(t.numel() + 1, device=DEV)
                    base[1:] = t.reshape(-1)
                    t = base[1:].view(shape)
            elif dt == torch.bool:
                t = torch.rand(shape, generator=g, device=DEV) > 0.5
            else:
                t = torch.randint(-3000, 3000, shape, generator=g, device=DEV).to(dt)
            sd[f"k{j}"] = t
        out.append(sd)
    counts = [int(c) for c in np.random.default_rng(seed).integers(1, 1000, size=K)]
    return counts, out


class _Round:
    """The tables the drop-in passes, built from the same KeyTable."""

    def __init__(self, counts, dicts, extra_cols=0):
        from mfl_amd import KeyTable

        self.lib = mfl_amd._lib.load()
        self.table = KeyTable(dicts[0])
        self.g = self.table.groups[torch.float32]
        ptrs, _ = self.table.collect(dicts, DEV)
        K, n_all = ptrs.shape
        # a wider address table: columns the group does not name hold 0
        # (never read); the group's columns keep their order
        self.ptrs = np.zeros((K, n_all + extra_cols), dtype=np.int64)
        self.ptrs[:, :n_all] = ptrs
        self.key_index = np.ascontiguousarray(self.g.key_index, dtype=np.int64)
        self.numel = np.ascontiguousarray(self.g.numel, dtype=np.int64)
        self.offset = np.ascontiguousarray(self.g.offset, dtype=np.int64)
        self.kind = np.ascontiguousarray(self.g.kind, dtype=np.int64)
        self.K, self.n = K, len(self.numel)
        total = sum(counts)
        self.w64 = np.array([n / total for n in counts], dtype=np.float64)

    def run(self, sums=True, scratch=True):
        lib, K, n = self.lib, self.K, self.n
        out = torch.full((self.g.P,), float("nan"), device=DEV)
        partials = torch.empty(max(1, lib.fedavg_reduce_sqdist_segments_partials(max(1, min(K, 1024)))),
                               dtype=torch.float64, device=DEV)
        sumsq = torch.full((K,), -1.0, dtype=torch.float64, device=DEV) if sums else None
        n_s = lib.fedavg_device_round_scratch(self.numel.ctypes.data, self.kind.ctypes.data, n, K)
        scr = torch.empty(max(1, n_s), device=DEV) if scratch and n_s else None
        need = lib.fedavg_device_round_workspace(K, n)
        ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
        ws_d = torch.empty(need, dtype=torch.uint8, device=DEV)
        rc = lib.fedavg_device_round_f32(self.ptrs.ctypes.data, self.ptrs.shape[1], self.key_index.ctypes.data,
                                         self.numel.ctypes.data, self.offset.ctypes.data, self.kind.ctypes.data, n, K,
                                         self.w64.ctypes.data, out.data_ptr(), partials.data_ptr(), partials.numel(),
                                         None if sumsq is None else sumsq.data_ptr(),
                                         None if scr is None else scr.data_ptr(), 0 if scr is None else scr.numel(),
                                         ws_h.data_ptr(), ws_d.data_ptr(), need, None)
        torch.cuda.synchronize()
        return rc, out, sumsq


def _expected(counts, dicts, g):
    ref = O.aggregate_torch([(n, OrderedDict((k, v.cpu()) for k, v in sd.items())) for n, sd in
                             zip(counts, [OrderedDict(d) for d in dicts])])
    flat = torch.zeros(g.P, dtype=torch.float32)
    for e in g.keys:
        flat[e.offset:e.offset + e.numel] = ref[e.name].reshape(-1).to(torch.float32)
    return flat


def _exact_sums(dicts, g, glob):
    """fp64 sums of fl32(x - g)^2 over the group (the fused pass's definition)."""
    gl = glob.double().numpy().astype(np.float32)
    sums = []
    for sd in dicts:
        row = np.zeros(g.P, dtype=np.float32)
        for e in g.keys:
            row[e.offset:e.offset + e.numel] = sd[e.name].cpu().reshape(-1).to(torch.float32).numpy()
        d = (row - gl).astype(np.float32).astype(np.float64)
        sums.append(float(np.sum(d * d)))
    return np.array(sums)


@pytest.mark.parametrize("K", [1, 5, 16, 17, 40, 64, 65, 100, 128, 129, 130, 256])
def test_device_round_fused_bit_exact(K):
    counts, dicts = _clients(K, _SPECS, seed=K)
    r = _Round(counts, dicts, extra_cols=3)
    rc, out, sumsq = r.run()
    assert rc == 0
    exp = _expected(counts, dicts, r.g)
    assert_bits(out.cpu(), exp, f"device round K={K}")
    got = sumsq.cpu().numpy()
    ref = _exact_sums(dicts, r.g, exp)
    assert np.allclose(got, ref, rtol=1e-11, atol=0.0), (got[:4], ref[:4])
    # the reduce alone: the same bits, sums untouched
    rc1, out1, _ = r.run(sums=False)
    assert rc1 == 1
    assert_bits(out1.cpu(), exp, f"device round reduce-only K={K}")


@pytest.mark.parametrize("K", [20, 600])
def test_device_round_misaligned_source_reduces_only(K):
    """A 4-B aligned fp32 source (the tiles' LDS-DMA and the split windows'
    loads need 16 B) sends the round to the reduce alone: same bits, sums
    untouched (the caller then runs the :291 pass)."""
    counts, dicts = _clients(K, _SPECS, seed=3, misalign_client=7)
    r = _Round(counts, dicts)
    rc, out, sumsq = r.run()
    assert rc == 1
    assert_bits(out.cpu(), _expected(counts, dicts, r.g), f"misaligned device round K={K}")
    assert bool((sumsq == -1.0).all())


@pytest.mark.parametrize("K", [257, 300, 513, 1024])
def test_device_round_split_windows_bit_exact(K):
    """257-1024 clients fuse on the zero-copy split-row windows (ceil(K / 64)
    waves per 64-column window): every key kind of _SPECS (integer and bool
    keys through the fp32 scratch, an empty key, keys shorter than a window
    and ragged last windows), the reference's bits and the exact sums."""
    counts, dicts = _clients(K, _SPECS, seed=K)
    r = _Round(counts, dicts, extra_cols=2)
    rc, out, sumsq = r.run()
    assert rc == 0
    exp = _expected(counts, dicts, r.g)
    assert_bits(out.cpu(), exp, f"split-row device round K={K}")
    got = sumsq.cpu().numpy()
    ref = _exact_sums(dicts, r.g, exp)
    assert np.allclose(got, ref, rtol=1e-11, atol=0.0), (got[:4], ref[:4])
    _, _, again = r.run()
    assert torch.equal(sumsq, again)  # deterministic


@pytest.mark.parametrize("K", [129, 160, 200, 256])
def test_device_round_split_windows_from_129(K):
    """129-256 clients on a long enough model (>= 8 windows of 64 columns per
    workgroup) take the zero-copy split windows too (round 6): every key kind
    of _SPECS plus a long key, the reference's bits and the exact sums."""
    specs = _SPECS + [((600_001,), torch.float32)]
    counts, dicts = _clients(K, specs, seed=K + 1)
    r = _Round(counts, dicts)
    rc, out, sumsq = r.run()
    assert rc == 0
    exp = _expected(counts, dicts, r.g)
    assert_bits(out.cpu(), exp, f"split-row device round K={K}")
    ref = _exact_sums(dicts, r.g, exp)
    assert np.allclose(sumsq.cpu().numpy(), ref, rtol=1e-10, atol=0.0)
    _, _, again = r.run()
    assert torch.equal(sumsq, again)


@pytest.mark.parametrize("K", [1025])
def test_device_round_many_clients_reduce_only(K):
    counts, dicts = _clients(K, [((300,), torch.float32), ((), torch.int64)], seed=9)
    r = _Round(counts, dicts)
    rc, out, sumsq = r.run()
    assert rc == 1
    assert_bits(out.cpu(), _expected(counts, dicts, r.g), f"K={K} device round")


def test_device_round_long_model_windows():
    """A long model at 100 clients (>= 16 windows of 128 columns per wave)
    takes the wave-owned windows, its int64 key through the scratch."""
    specs = [((4_500_000,), torch.float32), ((), torch.int64), ((4097,), torch.float32)]
    counts, dicts = _clients(100, specs, seed=5)
    r = _Round(counts, dicts)
    rc, out, sumsq = r.run()
    assert rc == 0
    exp = _expected(counts, dicts, r.g)
    assert_bits(out.cpu(), exp, "window device round")
    ref = _exact_sums(dicts, r.g, exp)
    # 4.5M fp64 terms: the sums' order differs from numpy's pairwise one
    assert np.allclose(sumsq.cpu().numpy(), ref, rtol=1e-9, atol=0.0)


def test_device_round_refusals():
    counts, dicts = _clients(6, _SPECS, seed=1)
    r = _Round(counts, dicts)
    rc, out, _ = r.run(scratch=False)  # integer keys of a fused round need the scratch
    assert rc == EINVAL
    assert bool(torch.isnan(out).all())
    host = torch.ones(100)
    r.ptrs[2, int(r.key_index[0])] = host.data_ptr()
    r.ptrs[0, int(r.key_index[0])] = host.data_ptr()  # the spot-checked first source
    rc, out, _ = r.run()
    assert rc == EINVAL
    r2 = _Round(counts, dicts)
    r2.ptrs[1, int(r2.key_index[3])] = 0  # a null source of a non-empty key
    assert r2.run()[0] == EINVAL
    lib = mfl_amd._lib.load()
    assert lib.fedavg_device_round_workspace(0, 5) == 0
    assert lib.fedavg_device_round_f32(None, 0, None, None, None, None, 0, 0, None, None, None, 0, None, None, 0,
                                       None, None, 0, None) == EINVAL


def test_drop_in_device_round_takes_the_one_call(monkeypatch):
    """aggregate() on device clients goes through fedavg_device_round_f32 and
    the fused sums feed client_distances."""
    counts, dicts = _clients(12, [s for s in _SPECS if s[1] != torch.bool], seed=12)  # :291 raises on bool
    agg = mfl_amd.DeviceAggregator(DEV)
    calls = []
    lib = mfl_amd._lib.load()
    orig = lib.fedavg_device_round_f32

    def spy(*a):
        rc = orig(*a)
        calls.append(rc)
        return rc

    monkeypatch.setattr(lib, "fedavg_device_round_f32", spy)
    wl = [(n, OrderedDict(sd)) for n, sd in zip(counts, dicts)]
    glob = agg.aggregate(wl)
    assert calls == [0]
    assert torch.float32 in agg._last.get("sumsq", {})
    ref_locals = [(n, OrderedDict((k, v.cpu()) for k, v in sd.items())) for n, sd in zip(counts, dicts)]
    ref_glob = O.aggregate_torch([(n, OrderedDict(sd)) for n, sd in ref_locals])
    for k in ref_glob:
        assert_bits(glob[k].cpu(), ref_glob[k], k)
    d = agg.client_distances(wl, glob)
    ref_locals[0] = (ref_locals[0][0], ref_glob)
    exact = O.client_distances_exact(ref_locals, ref_glob)
    assert d[0] == 0.0
    assert np.all(np.abs(d - exact) <= np.spacing(exact.astype(np.float32)).astype(np.float64))


@pytest.mark.parametrize("K", [5, 40, 100])
def test_legacy_fused_segments_entry_matches(K):
    """fedavg_reduce_sqdist_segments_f32 (the separate-table entry, integer
    keys converted inside the tiles, no unit map) gives the bits and sums of
    the one-call round on the same clients."""
    _legacy_entry_matches(K, _SPECS, seed=50 + K)


@pytest.mark.parametrize("K", [129, 200])
def test_legacy_fused_segments_entry_split_windows(K):
    """The separate-table entry on all-fp32 clients long enough for the
    zero-copy split windows (129-256 clients, round 6): the one-call round's
    bits and sums."""
    specs = [((64, 3, 3, 3), torch.float32), ((127,), torch.float32), ((600_001,), torch.float32),
             ((0,), torch.float32), ((40_001,), torch.float32)]
    _legacy_entry_matches(K, specs, seed=70 + K)


def _legacy_entry_matches(K, specs, seed):
    counts, dicts = _clients(K, specs, seed=seed)
    r = _Round(counts, dicts)
    rc, out, sumsq = r.run()
    assert rc == 0
    lib = r.lib
    cptrs = np.ascontiguousarray(r.ptrs[:, r.key_index])
    w_dev = torch.tensor(r.w64, dtype=torch.float32, device=DEV)
    out2 = torch.full((r.g.P,), float("nan"), device=DEV)
    partials = torch.empty(max(1, lib.fedavg_reduce_sqdist_segments_partials(K)), dtype=torch.float64, device=DEV)
    sums2 = torch.empty(K, dtype=torch.float64, device=DEV)
    need = lib.fedavg_segments_workspace(K, r.n)
    ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    ws_d = torch.empty(need, dtype=torch.uint8, device=DEV)
    rc2 = lib.fedavg_reduce_sqdist_segments_f32(cptrs.ctypes.data, r.numel.ctypes.data, r.offset.ctypes.data,
                                                r.kind.ctypes.data, r.n, K, w_dev.data_ptr(), out2.data_ptr(),
                                                partials.data_ptr(), partials.numel(), sums2.data_ptr(),
                                                ws_h.data_ptr(), ws_d.data_ptr(), need, None)
    torch.cuda.synchronize()
    assert rc2 == 0
    assert_bits(out2.cpu(), out.cpu(), f"legacy fused entry K={K}")
    assert np.allclose(sums2.cpu().numpy(), sumsq.cpu().numpy(), rtol=1e-12, atol=0.0)


def test_drop_in_device_round_all_empty_keys():
    """A model whose fp32 keys are all empty (numel 0): no native call, the
    reference's loop result (empty tensors) and zero :291 distances."""
    K = 4
    dicts = [OrderedDict(a=torch.zeros(0, device=DEV), b=torch.zeros((3, 0), device=DEV)) for _ in range(K)]
    counts = [3, 1, 4, 1]
    agg = mfl_amd.DeviceAggregator(DEV)
    wl = [(n, OrderedDict(sd)) for n, sd in zip(counts, dicts)]
    glob = agg.aggregate(wl)
    assert glob["a"].shape == (0,) and glob["b"].shape == (3, 0)
    assert glob["a"].device.type == "cuda"
    d = agg.client_distances(wl, glob)
    assert np.array_equal(d, np.zeros(K))


def test_device_round_resnet56_doubling_property():
    """resnet56 x 100 (350 keys, 58 int64 buffers) through the zero-copy
    tiles (the LDS-address form): against the reference's torch loop bit for
    bit, then every client doubled in place -- powers of two commute with
    every rounding step, so the average must come out exactly 2x and each
    client's fp64 sum of squares exactly 4x (the sums' order is the same
    grid, so the property is bit-exact)."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "scripts"))
    from model_shapes import CONFIGS

    K, shapes = CONFIGS["resnet56"]
    specs = [(s, torch.int64 if n.endswith("num_batches_tracked") else torch.float32) for n, s in shapes]
    counts, dicts = _clients(K, specs, seed=56)
    r = _Round(counts, dicts)
    rc, out, sumsq = r.run()
    assert rc == 0
    assert_bits(out.cpu(), _expected(counts, dicts, r.g), "resnet56 device round")
    for sd in dicts:
        for t in sd.values():
            t.mul_(2)
    rc2, out2, sumsq2 = r.run()
    assert rc2 == 0
    assert torch.equal(out2.view(torch.int32), (out * 2.0).view(torch.int32))
    assert torch.equal(sumsq2, sumsq * 4.0)


def test_device_round_many_keys_window_plan():
    """A model of 2,100 keys at 20 clients on the one-wave windows (48-row
    instance): its descriptor table (2,101 x 48 entries) is larger than the
    room the workspace reserves when a 128-row table would not fit, so the
    round takes the pointer form -- same bits, exact sums (round 5 fix: the
    table was written past the workspace before)."""
    specs = [((4500,), torch.float32)] * 2100
    counts, dicts = _clients(20, specs, seed=21)
    r = _Round(counts, dicts)
    rc, out, sumsq = r.run()
    assert rc == 0
    exp = _expected(counts, dicts, r.g)
    assert_bits(out.cpu(), exp, "2,100-key device round")
    ref = _exact_sums(dicts, r.g, exp)
    assert np.allclose(sumsq.cpu().numpy(), ref, rtol=1e-11, atol=0.0)
