"""Device-resident clients: state_dicts whose tensors already live in HBM.

The reference's ``aggregate`` (fedavg_trainer.py:441-458) runs its torch ops
on whatever device the clients' tensors are on; client.py:96 moves them to the
host (``net.cpu().state_dict()``), and a GPU-side deployment drops that copy.
Then the drop-in packs the rows with one kernel (``fedavg_pack_rows_device``)
and returns device tensors.  Parity bar as everywhere: bit-exact against the
reference's golden vectors and the torch oracle; the packing kernel is checked
byte for byte against the host packer (``fedavg_pack_rows``).
"""
import copy
from collections import OrderedDict

import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd
from golden_io import case_names, load_case
from test_gpu_parity import assert_bits

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield


def _to_dev(w_locals):
    return [(n, OrderedDict((k, v.to(DEV)) for k, v in sd.items())) for n, sd in w_locals]


_CASES = [c for c in case_names() if c not in ("empty_w_locals", "no_keys_k2")]


@pytest.mark.parametrize("rows", [False, True], ids=["zero_copy", "rows"])
@pytest.mark.parametrize("name", _CASES)
def test_device_clients_match_reference_golden(name, rows, monkeypatch):
    _, w_locals, expected = load_case(name)
    dl = _to_dev(w_locals)
    first = dl[0][1]
    others = [dict(sd) for _, sd in dl[1:]]
    monkeypatch.setattr(mfl_amd.DeviceAggregator, "DEVICE_SEGMENTS", not rows)
    out = mfl_amd.aggregate(dl)  # the device is taken from the clients' tensors
    assert out is first
    assert list(out.keys()) == list(expected.keys())
    for k, exp in expected.items():
        assert out[k].device == DEV
        assert_bits(out[k], exp, f"{name}/{k}")
    for d, (_, sd) in zip(others, dl[1:]):
        assert all(d[k] is sd[k] for k in d)


@pytest.mark.parametrize("name", ["mnist_lr_k100", "resnet_like_bn_k5", "int_dtypes_k3", "float64_key_k3",
                                  "bfloat16_key_k3", "float16_key_k3", "ieee_specials_k4", "single_client_k1",
                                  "int64_nbt_example"])
def test_device_clients_streaming_session(name):
    _, w_locals, expected = load_case(name)
    dl = _to_dev(w_locals)
    agg = mfl_amd.DeviceAggregator(DEV)
    sess = agg.begin_round(dl[0][1], len(dl) + 2)
    for n, sd in dl:
        sess.add(n, sd)
    out = sess.finish(dl)
    assert out is dl[0][1]
    for k, exp in expected.items():
        assert out[k].device == DEV
        assert_bits(out[k], exp, f"{name}/{k}")


def test_device_clients_random_rounds_bit_exact():
    """20 seeded random rounds (1-40 clients, 1-12 keys of random shapes and
    dtypes incl. int64/int32/int16/int8/uint8/bool buffers and fp64/fp16/bf16
    keys) through one aggregator, device in, device out, against the torch
    oracle on the host copies."""
    rng = np.random.default_rng(91)
    agg = mfl_amd.DeviceAggregator(DEV)
    extra = [torch.float64, torch.float16, torch.bfloat16, torch.int16, torch.int8, torch.uint8]
    for case in range(20):
        K = int(rng.integers(1, 41))
        keys = []
        for j in range(int(rng.integers(1, 13))):
            shape = tuple(int(d) for d in rng.integers(1, 40, size=int(rng.integers(0, 5))))
            r = rng.random()
            dt = (torch.float32 if r < 0.6 else torch.int64 if r < 0.7 else torch.int32 if r < 0.75
                  else torch.bool if r < 0.8 else extra[int(rng.integers(0, len(extra)))])
            keys.append((f"k{j}", shape, dt))
        g = torch.Generator().manual_seed(1000 + case)
        w_locals = []
        for i in range(K):
            sd = OrderedDict()
            for name, shape, dt in keys:
                if dt == torch.bool:
                    sd[name] = torch.rand(shape, generator=g) > 0.5
                elif dt == torch.uint8:
                    sd[name] = torch.randint(0, 256, shape, generator=g).to(dt)
                elif not dt.is_floating_point:
                    sd[name] = torch.randint(-100, 100, shape, generator=g).to(dt)
                else:
                    sd[name] = (torch.randn(shape, generator=g) * 0.05).to(dt)
            w_locals.append((int(rng.integers(1, 10**6)), sd))
        ref = O.aggregate_torch(copy.deepcopy(w_locals))
        out = agg.aggregate(_to_dev(w_locals))
        for k in ref:
            assert out[k].device == DEV
            assert_bits(out[k], ref[k], f"case {case} key {k}")


def test_pack_kernel_matches_host_packer():
    """fedavg_pack_rows_device vs fedavg_pack_rows on the same item list:
    every kind, empty items, items spanning many 16K-element chunks, odd
    offsets; compared byte for byte (padding included)."""
    lib = mfl_amd._lib.load()
    g = torch.Generator().manual_seed(5)
    kinds = {0: torch.float32, 1: torch.int64, 2: torch.int32, 3: torch.int16, 4: torch.int8, 5: torch.uint8,
             6: torch.bool}
    sizes = [0, 1, 3, 63, 64, 65, 16_383, 16_384, 16_385, 100_003, 1_000_000, 7]
    srcs_h, items = [], []
    off = 5
    for j, n in enumerate(sizes):
        kind = j % 7
        dt = kinds[kind]
        if dt == torch.bool:
            t = torch.rand(n, generator=g) > 0.5
        elif dt == torch.float32:
            t = torch.randn(n, generator=g)
        elif dt == torch.uint8:
            t = torch.randint(0, 256, (n,), generator=g).to(dt)
        else:
            t = torch.randint(-(2**31), 2**31 - 1, (n,), generator=g).to(dt)
            if dt == torch.int64:
                t = t * 4099 + 3  # beyond 2^24: the int64 -> fp32 rounding matters
        srcs_h.append(t)
        items.append((kind, off, n))
        off += n + (j % 3)
    total = off + 11
    srcs_d = [t.to(DEV) for t in srcs_h]
    it_h = np.array([[t.data_ptr(), n, o, k] for t, (k, o, n) in zip(srcs_h, items)], dtype=np.int64)
    it_d = np.array([[t.data_ptr(), n, o, k] for t, (k, o, n) in zip(srcs_d, items)], dtype=np.int64)
    host = torch.full((total,), -7.0, dtype=torch.float32)
    mfl_amd._lib.check(lib.fedavg_pack_rows(it_h.ctypes.data, len(items), host.data_ptr(), 4, 4), "pack")
    dev = torch.full((total,), -7.0, dtype=torch.float32, device=DEV)
    need = lib.fedavg_pack_rows_device_workspace(len(items))
    ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    ws_d = torch.empty(need, dtype=torch.uint8, device=DEV)
    s = torch.cuda.current_stream(DEV)
    mfl_amd._lib.check(lib.fedavg_pack_rows_device(it_d.ctypes.data, len(items), dev.data_ptr(), 4, ws_h.data_ptr(),
                                                   ws_d.data_ptr(), need, s.cuda_stream), "pack_device")
    s.synchronize()
    assert dev.cpu().view(torch.int32).numpy().tobytes() == host.view(torch.int32).numpy().tobytes()


@pytest.mark.parametrize("es", [4, 8, 2])
def test_pack_kernel_many_tiny_items(es):
    """Thousands of 1-40 element items (BatchNorm's scalar num_batches_tracked
    over every client): fedavg_pack_rows_device takes its thread-per-item
    kernel (average <= 64 elements); byte for byte against the host packer,
    every kind for fp32 rows, raw items for 8- and 2-byte rows."""
    lib = mfl_amd._lib.load()
    rng = np.random.default_rng(es)
    g = torch.Generator().manual_seed(es)
    kinds = {0: {4: torch.float32, 8: torch.float64, 2: torch.float16}[es], 1: torch.int64, 2: torch.int32,
             3: torch.int16, 4: torch.int8, 5: torch.uint8, 6: torch.bool}
    srcs_h, items, off = [], [], 3
    for j in range(3000):
        kind = int(rng.integers(0, 7)) if es == 4 else 0
        n = int(rng.integers(0, 41)) if j % 5 else 1
        dt = kinds[kind]
        if dt == torch.bool:
            t = torch.rand(n, generator=g) > 0.5
        elif dt.is_floating_point:
            t = torch.randn(n, generator=g).to(dt)
        elif dt == torch.uint8:
            t = torch.randint(0, 256, (n,), generator=g).to(dt)
        else:
            t = torch.randint(-(2**31), 2**31 - 1, (n,), generator=g).to(dt)
            if dt == torch.int64:
                t = t * 4099 + 3
        srcs_h.append(t)
        items.append((kind, off, n))
        off += n + int(rng.integers(0, 3))
    srcs_d = [t.to(DEV) for t in srcs_h]
    it_h = np.array([[t.data_ptr(), n, o, k] for t, (k, o, n) in zip(srcs_h, items)], dtype=np.int64)
    it_d = np.array([[t.data_ptr(), n, o, k] for t, (k, o, n) in zip(srcs_d, items)], dtype=np.int64)
    dt_row = kinds[0]
    host = torch.full((off + 5,), -7.0, dtype=dt_row)
    mfl_amd._lib.check(lib.fedavg_pack_rows(it_h.ctypes.data, len(items), host.data_ptr(), es, 4), "pack")
    dev = torch.full((off + 5,), -7.0, dtype=dt_row, device=DEV)
    need = lib.fedavg_pack_rows_device_workspace(len(items))
    ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    ws_d = torch.empty(need, dtype=torch.uint8, device=DEV)
    s = torch.cuda.current_stream(DEV)
    mfl_amd._lib.check(lib.fedavg_pack_rows_device(it_d.ctypes.data, len(items), dev.data_ptr(), es, ws_h.data_ptr(),
                                                   ws_d.data_ptr(), need, s.cuda_stream), "pack_device")
    s.synchronize()
    assert dev.cpu().view(torch.uint8).numpy().tobytes() == host.view(torch.uint8).numpy().tobytes()


@pytest.mark.parametrize("dtype", [torch.float64, torch.float16, torch.bfloat16])
def test_pack_kernel_raw_other_widths(dtype):
    lib = mfl_amd._lib.load()
    esize = torch.empty(0, dtype=dtype).element_size()
    g = torch.Generator().manual_seed(esize)
    srcs = [(torch.randn(n, generator=g) * 3).to(dtype).to(DEV) for n in (1, 40_000, 16_384 * 4 + 1, 0, 9)]
    off, rows = 3, []
    for t in srcs:
        rows.append([t.data_ptr(), t.numel(), off, 0])
        off += t.numel() + 1
    it = np.array(rows, dtype=np.int64)
    dev = torch.zeros(off + 2, dtype=dtype, device=DEV)
    need = lib.fedavg_pack_rows_device_workspace(len(rows))
    ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    ws_d = torch.empty(need, dtype=torch.uint8, device=DEV)
    mfl_amd._lib.check(lib.fedavg_pack_rows_device(it.ctypes.data, len(rows), dev.data_ptr(), esize, ws_h.data_ptr(),
                                                   ws_d.data_ptr(), need, None), "pack_device")
    torch.cuda.synchronize()
    exp = torch.zeros(off + 2, dtype=dtype)
    for t, r in zip(srcs, rows):
        exp[r[2]:r[2] + r[1]] = t.cpu()
    assert torch.equal(dev.cpu().view(torch.uint8), exp.view(torch.uint8))


def test_pack_kernel_rejects_host_sources_and_bad_items():
    lib = mfl_amd._lib.load()
    host_src = torch.ones(100)
    dev = torch.zeros(200, device=DEV)
    need = lib.fedavg_pack_rows_device_workspace(1)
    ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    ws_d = torch.empty(need, dtype=torch.uint8, device=DEV)
    it = np.array([[host_src.data_ptr(), 100, 0, 0]], dtype=np.int64)
    rc = lib.fedavg_pack_rows_device(it.ctypes.data, 1, dev.data_ptr(), 4, ws_h.data_ptr(), ws_d.data_ptr(), need, None)
    assert rc == -10001  # a host source would fault the kernel: refused before launch
    d_src = torch.ones(100, device=DEV)
    bad = np.array([[d_src.data_ptr(), 100, 0, 9]], dtype=np.int64)  # unknown kind
    rc = lib.fedavg_pack_rows_device(bad.ctypes.data, 1, dev.data_ptr(), 4, ws_h.data_ptr(), ws_d.data_ptr(), need, None)
    assert rc == -10001
    pageable = torch.empty(need, dtype=torch.uint8)
    ok = np.array([[d_src.data_ptr(), 100, 0, 0]], dtype=np.int64)
    rc = lib.fedavg_pack_rows_device(ok.ctypes.data, 1, dev.data_ptr(), 4, pageable.data_ptr(), ws_d.data_ptr(), need,
                                     None)
    assert rc == -10001
    rc = lib.fedavg_pack_rows_device(ok.ctypes.data, 1, dev.data_ptr(), 4, ws_h.data_ptr(), ws_d.data_ptr(), need - 1,
                                     None)
    assert rc == -10001
    torch.cuda.synchronize()
    assert float(dev.sum()) == 0.0  # nothing was launched


def test_mixed_devices_rejected():
    _, w_locals, _ = load_case("mnist_lr_k10")
    dl = _to_dev(w_locals)
    dl[3] = w_locals[3]  # one client left on the host
    with pytest.raises(TypeError):
        mfl_amd.DeviceAggregator(DEV).aggregate(dl)
    dl = _to_dev(w_locals)
    dl[0][1]["linear.bias"] = dl[0][1]["linear.bias"].cpu()  # one key of client 0 on the host
    with pytest.raises(TypeError):
        mfl_amd.DeviceAggregator(DEV).aggregate(dl)


def test_device_clients_distances_cached_and_uncached():
    _, w_locals, _ = load_case("mnist_lr_k100")
    ref_locals = copy.deepcopy(w_locals)
    ref_glob = O.aggregate_torch(ref_locals)
    exact = O.client_distances_exact(ref_locals, ref_glob)
    dl = _to_dev(w_locals)
    agg = mfl_amd.DeviceAggregator(DEV)
    w_glob = agg.aggregate(dl)
    norms = agg.client_distances(dl, w_glob)  # rows left in HBM by the aggregate
    assert norms[0] == 0.0
    assert np.all(np.abs(norms - exact) <= np.spacing(exact.astype(np.float32)).astype(np.float64))
    again = mfl_amd.DeviceAggregator(DEV).client_distances(dl, w_glob)  # packed on the device afresh
    assert np.array_equal(again, norms)
    host_glob = OrderedDict((k, v.cpu()) for k, v in w_glob.items())
    with pytest.raises(TypeError):  # w - w_glob across devices
        mfl_amd.DeviceAggregator(DEV).client_distances(dl[1:], host_glob)


@pytest.mark.parametrize("name", ["resnet_like_bn_k5", "mnist_lr_k10"])  # pipelined / one-call host rounds
def test_device_and_host_rounds_alternate_on_one_aggregator(name):
    """A device round returns before its kernels ran; the host round right
    after it (no synchronization in between) must not disturb it through the
    shared staging (weights, rows), and both must be exact."""
    _, _, expected = load_case(name)
    agg = mfl_amd.DeviceAggregator(DEV)
    outs = []
    for r in range(4):
        _, wl, _ = load_case(name)
        if r % 2 == 0:  # different weights each round: a stale weight vector would show
            wl = [(n * (r + 1) if i == 0 else n, sd) for i, (n, sd) in enumerate(wl)]
        outs.append((r, copy.deepcopy(wl) if r % 2 == 0 else None, agg.aggregate(_to_dev(wl) if r % 2 == 0 else wl)))
    torch.cuda.synchronize()
    for r, ref_in, out in outs:
        exp = O.aggregate_torch(ref_in) if ref_in is not None else expected
        for k in exp:
            assert out[k].device.type == ("cuda" if r % 2 == 0 else "cpu")
            assert_bits(out[k], exp[k], f"{name} round {r} {k}")


def _segment_case(K, specs, seed, offset_base=3):
    """K clients whose keys are views into one flat device buffer per client at
    odd fp32 offsets (4-B aligned, not 16-B), of the given (shape, dtype)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    dicts = []
    for i in range(K):
        sizes = [int(np.prod(shape)) for shape, _ in specs]
        flat = torch.empty(sum(sizes) + 4 * len(specs) + offset_base, device=DEV)
        sd, off = OrderedDict(), offset_base + i % 3
        for j, ((shape, dt), n) in enumerate(zip(specs, sizes)):
            if dt == torch.float32:
                sd[f"k{j}"] = (torch.randn(n, generator=g, device=DEV) * 0.05).view(shape)
                flat[off:off + n] = sd[f"k{j}"].reshape(-1)
                sd[f"k{j}"] = flat[off:off + n].view(shape)
                off += n + 1
            elif dt == torch.bool:
                sd[f"k{j}"] = torch.rand(shape, generator=g, device=DEV) > 0.5
            else:
                sd[f"k{j}"] = torch.randint(-3000, 3000, shape, generator=g, device=DEV).to(dt)
        dicts.append(sd)
    counts = [int(c) for c in np.random.default_rng(seed).integers(1, 1000, size=K)]
    return [(n, sd) for n, sd in zip(counts, dicts)]


_SEG_SPECS = [((8192,), torch.float32), ((8191,), torch.float32), ((8193,), torch.float32), ((0,), torch.float32),
              ((4096,), torch.float32), ((4095,), torch.float32), ((4097,), torch.float32),
              ((3, 5), torch.float32), ((), torch.int64), ((7,), torch.int32), ((1,), torch.float32),
              ((40_001,), torch.float32), ((5, 2), torch.bool), ((16_384 * 3 + 2,), torch.float32)]


@pytest.mark.parametrize("K", [1, 2, 5, 33])
def test_segments_reduce_bit_identical_to_rows(K):
    """Zero-copy reduce (fedavg_reduce_segments_f32, views at odd offsets,
    key tails around the 8,192-column unit, integer/bool keys) against the
    packed-rows reduce of the same clients and the torch oracle."""
    wl = _segment_case(K, _SEG_SPECS, seed=K)
    ref = O.aggregate_torch([(n, OrderedDict((k, v.cpu()) for k, v in sd.items())) for n, sd in wl])
    seg = mfl_amd.DeviceAggregator(DEV)
    rows = mfl_amd.DeviceAggregator(DEV)
    rows.DEVICE_SEGMENTS = False
    out_seg = seg.aggregate([(n, OrderedDict(sd)) for n, sd in wl])
    assert seg._last["dev"][torch.float32][0] is None  # no rows were packed
    out_rows = rows.aggregate([(n, OrderedDict(sd)) for n, sd in wl])
    for k in ref:
        assert_bits(out_seg[k], ref[k], f"segments K={K} {k}")
        assert_bits(out_rows[k], out_seg[k].cpu(), f"rows vs segments K={K} {k}")


def test_segments_distances_match_rows_path():
    wl = _segment_case(9, [s for s in _SEG_SPECS if s[1] != torch.bool], seed=11)
    seg = mfl_amd.DeviceAggregator(DEV)
    rows = mfl_amd.DeviceAggregator(DEV)
    rows.DEVICE_SEGMENTS = False
    wa = [(n, OrderedDict(sd)) for n, sd in wl]
    wb = [(n, OrderedDict(sd)) for n, sd in wl]
    ga, gb = seg.aggregate(wa), rows.aggregate(wb)
    na = seg.client_distances(wa, ga)  # zero-copy sums of squares
    nb = rows.client_distances(wb, gb)  # packed rows
    ref_locals = [(n, OrderedDict((k, v.cpu()) for k, v in sd.items())) for n, sd in wl]
    ref_glob = O.aggregate_torch(copy.deepcopy(ref_locals))
    ref_locals[0] = (ref_locals[0][0], ref_glob)
    exact = O.client_distances_exact(ref_locals, ref_glob)
    assert na[0] == 0.0 and nb[0] == 0.0
    assert np.all(np.abs(na - exact) <= np.spacing(exact.astype(np.float32)).astype(np.float64))
    assert np.all(np.abs(na - nb) <= np.spacing(exact.astype(np.float32)).astype(np.float64))


def test_segments_rows_materialized_for_fpf_record_round():
    """After a zero-copy round the rows are packed on demand (client 0 from its
    own tensors, not the average its dict now holds)."""
    _, w_locals, _ = load_case("mnist_lr_k10")
    dl = _to_dev(w_locals)
    client0 = OrderedDict((k, v.clone()) for k, v in dl[0][1].items())
    agg = mfl_amd.DeviceAggregator(DEV)
    agg.aggregate(dl)
    rows = agg.materialize_rows()
    assert rows is not None and rows.shape[0] == 10
    P = sum(v.numel() for v in client0.values())
    exp0 = torch.cat([v.reshape(-1) for v in client0.values()])
    exp3 = torch.cat([v.reshape(-1) for v in dl[3][1].values()])
    assert torch.equal(rows[0, :P], exp0) and torch.equal(rows[3, :P], exp3)
    assert agg.materialize_rows() is rows or torch.equal(agg.materialize_rows(), rows)


def test_segments_rejects_host_sources():
    lib = mfl_amd._lib.load()
    host = torch.ones(100)
    out = torch.zeros(100, device=DEV)
    w = torch.ones(1, device=DEV)
    need = lib.fedavg_segments_workspace(1, 1)
    ws_h = torch.empty(need, dtype=torch.uint8, pin_memory=True)
    ws_d = torch.empty(need, dtype=torch.uint8, device=DEV)
    ptrs = np.array([[host.data_ptr()]], dtype=np.int64)
    meta = [np.array([v], dtype=np.int64) for v in (100, 0, 0)]
    rc = lib.fedavg_reduce_segments_f32(ptrs.ctypes.data, meta[0].ctypes.data, meta[1].ctypes.data,
                                        meta[2].ctypes.data, 1, 1, w.data_ptr(), out.data_ptr(), ws_h.data_ptr(),
                                        ws_d.data_ptr(), need, None)
    assert rc == -10001
    dsrc = torch.ones(101, device=DEV)
    odd = np.array([[dsrc.data_ptr() + 2]], dtype=np.int64)  # not fp32-aligned
    rc = lib.fedavg_reduce_segments_f32(odd.ctypes.data, meta[0].ctypes.data, meta[1].ctypes.data,
                                        meta[2].ctypes.data, 1, 1, w.data_ptr(), out.data_ptr(), ws_h.data_ptr(),
                                        ws_d.data_ptr(), need, None)
    assert rc == -10001
    torch.cuda.synchronize()
    assert float(out.sum()) == 0.0


_SEG_VARIANTS = [(4, 8, 3), (4, 8, 0), (8, 4, 3), (2, 8, 6), (4, 4, 3), (8, 2, 6), (16, 2, 3), (2, 16, 3), (1, 16, 1)]


@pytest.mark.parametrize("K", [1, 6, 19])
def test_segments_variants_bit_identical(K):
    """Every schedule of the tuning hook fedavg_reduce_segments_f32_variant
    (units of 1,024 x C columns, so the key tails fall differently) gives the
    production zero-copy reduce's bits, integer/bool keys included."""
    kinds = {torch.float32: 0, torch.int64: 1, torch.int32: 2, torch.bool: 6}
    wl = _segment_case(K, _SEG_SPECS, seed=100 + K)
    keys = list(wl[0][1].keys())
    numel = np.array([wl[0][1][k].numel() for k in keys], dtype=np.int64)
    offset = np.concatenate([[0], np.cumsum(numel)[:-1]]).astype(np.int64)
    kind = np.array([kinds[wl[0][1][k].dtype] for k in keys], dtype=np.int64)
    ptrs = np.array([[sd[k].data_ptr() for k in keys] for _, sd in wl], dtype=np.int64)
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights([n for n, _ in wl]), torch.float32, DEV)
    lib = mfl_amd._lib.load_probe()
    need = lib.fedavg_segments_workspace(K, len(keys))
    P = int(numel.sum())
    args = (ptrs.ctypes.data, numel.ctypes.data, offset.ctypes.data, kind.ctypes.data, len(keys), K, w.data_ptr())
    ref = torch.full((P,), float("nan"), device=DEV)
    ws = [(torch.empty(need, dtype=torch.uint8, pin_memory=True), torch.empty(need, dtype=torch.uint8, device=DEV))
          for _ in range(len(_SEG_VARIANTS) + 1)]
    mfl_amd._lib.check(lib.fedavg_reduce_segments_f32(*args, ref.data_ptr(), ws[0][0].data_ptr(),
                                                      ws[0][1].data_ptr(), need, None), "production")
    outs = []
    for i, (u, c, b) in enumerate(_SEG_VARIANTS):
        out = torch.full((P,), float("nan"), device=DEV)
        mfl_amd._lib.check(lib.fedavg_reduce_segments_f32_variant(*args, out.data_ptr(), ws[i + 1][0].data_ptr(),
                                                                  ws[i + 1][1].data_ptr(), need, u, c, b, None),
                           f"U{u}C{c}b{b}")
        outs.append(out)
    torch.cuda.synchronize()
    exp = O.aggregate_torch([(n, OrderedDict((k, v.cpu()) for k, v in sd.items())) for n, sd in wl])
    assert_bits(ref.cpu(), torch.cat([exp[k].reshape(-1).float() for k in keys]), f"production K={K}")
    for (u, c, b), out in zip(_SEG_VARIANTS, outs):
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), f"U{u}C{c}b{b} K={K}"
    bad = lib.fedavg_reduce_segments_f32_variant(*args, ref.data_ptr(), ws[0][0].data_ptr(), ws[0][1].data_ptr(),
                                                 need, 3, 8, 3, None)
    assert bad == -10003


def test_client_arena_rounds_use_the_row_kernel_bit_exact():
    """client_arena dicts (views into one [K, ld] buffer in the packed layout)
    are reduced by the row kernel straight from that buffer: bit-exact vs the
    reference's loop, :291 from the same rows, and a layout that is NOT the
    packed one (keys in another order) takes the segments path, same bits."""
    import copy
    from collections import OrderedDict
    for name in ["mnist_lr_k10", "mnist_lr_k100", "flat_k10_p65", "thirds_k3"]:
        meta, w_locals, expected = load_case(name)
        if not all(t.dtype == torch.float32 for t in w_locals[0][1].values()):
            continue
        ref_locals = copy.deepcopy(w_locals)
        ref_glob = O.aggregate_torch(ref_locals)
        rows, adicts = mfl_amd.client_arena(w_locals[0][1], len(w_locals), DEV)
        for a, (_, sd) in zip(adicts, w_locals):
            for k, v in sd.items():
                a[k].copy_(v)
        agg = mfl_amd.DeviceAggregator(DEV)
        agg.ARENA_MIN_BYTES = 0  # golden cases are small
        wl = [(n, OrderedDict(a)) for (n, _), a in zip(w_locals, adicts)]
        out = agg.aggregate(wl)
        assert agg.arena_rounds == 1, name
        assert out is wl[0][1]
        for k, exp in expected.items():
            assert out[k].is_cuda
            assert torch.equal(out[k].cpu().reshape(-1).view(torch.int32), exp.reshape(-1).view(torch.int32)), (name, k)
        # the arena itself is untouched (client 0's row still holds its update)
        first = next(iter(w_locals[0][1]))
        assert torch.equal(adicts[0][first].cpu(), w_locals[0][1][first])
        norms = agg.client_distances(wl, out)
        exact = O.client_distances_exact(ref_locals, ref_glob)
        assert norms[0] == 0.0
        assert np.allclose(norms, exact, rtol=1.2e-7, atol=0), (name, norms, exact)
        # keys in another order than the buffer's: not the packed layout -> segments path
        if len(adicts[0]) > 1:
            agg2 = mfl_amd.DeviceAggregator(DEV)
            agg2.ARENA_MIN_BYTES = 0
            wl2 = [(n, OrderedDict(reversed(list(a.items())))) for (n, _), a in zip(w_locals, adicts)]
            out2 = agg2.aggregate(wl2)
            assert agg2.arena_rounds == 0
            for k, exp in expected.items():
                assert torch.equal(out2[k].cpu().reshape(-1).view(torch.int32), exp.reshape(-1).view(torch.int32))
