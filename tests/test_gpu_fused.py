"""GPU parity of the fused aggregate + :291 pass (fedavg_reduce_sqdist_f32).

The averaged model must carry the oracle's bits (fedavg_trainer.py:450-457,
the same bar as fedavg_reduce_f32); the sums of squares follow :291's rule
(fp32 difference, squared and summed in fp64), checked against fp64 sums of
the same fp32 differences at 1e-12 relative and for run-to-run determinism.
"""
import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield


def _rows(K, P, seed, pad=float("nan")):
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.full((K, ld), pad, device=DEV)
    x[:, :P] = torch.randn((K, P), generator=g, device=DEV) * 0.05 + torch.randn((K, 1), generator=g, device=DEV) * 1e-3
    counts = torch.randint(1, 1000, (K,), generator=torch.Generator().manual_seed(seed)).tolist()
    weights = mfl_amd.sample_weights(counts)
    return x, ld, weights


def _sumsq_ref(x, out, P):
    return torch.stack([((x[k, :P] - out[:P]).double() ** 2).sum() for k in range(x.shape[0])])


@pytest.mark.parametrize("K,P", [(1, 1), (1, 129), (2, 3), (3, 127), (3, 128), (5, 1001), (7, 4096 * 3 + 5),
                                 (13, 300_007), (64, 65_536), (100, 100_003), (127, 20_000), (128, 20_001)])
def test_fused_small_vs_oracle(K, P):
    x, ld, weights = _rows(K, P, K * 1000 + P)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, sumsq = mfl_amd.reduce_with_sqdist(x, w, P)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
    assert out.cpu().numpy().view(np.uint32).tobytes() == exp.view(np.uint32).tobytes()
    ref = _sumsq_ref(x, out, P)
    rel = ((sumsq - ref).abs() / ref.clamp_min(1e-300)).max().item()
    assert rel < 1e-12, rel
    _, again = mfl_amd.reduce_with_sqdist(x, w, P)
    assert torch.equal(sumsq, again)  # deterministic


@pytest.mark.parametrize("K,P", [(129, 5003), (256, 777), (257, 2049), (300, 70_001), (301, 33_333), (500, 1001),
                                 (512, 4099), (400, 300_001)])
def test_fused_many_clients_vs_oracle(K, P):
    """K > 128: register-staged tiles of 64 / 32 columns (16 / 10 / 16 slots
    per thread), up to 512 clients -- the reduce's bits."""
    x, ld, weights = _rows(K, P, K * 7 + P)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, sumsq = mfl_amd.reduce_with_sqdist(x, w, P)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), weights)
    assert out.cpu().numpy().view(np.uint32).tobytes() == exp.view(np.uint32).tobytes()
    ref = _sumsq_ref(x, out, P)
    rel = ((sumsq - ref).abs() / ref.clamp_min(1e-300)).max().item()
    assert rel < 1e-12, rel


@pytest.mark.parametrize("K,P", [(1025, 5003), (1300, 2001)])
def test_fused_large_k_takes_two_passes(K, P):
    """K > 1024: the same entry runs the two production passes; same bits."""
    x, ld, weights = _rows(K, P, K + P)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, sumsq = mfl_amd.reduce_with_sqdist(x, w, P)
    assert torch.equal(out.view(torch.int32), mfl_amd.reduce_packed(x, w, P).view(torch.int32))
    assert torch.equal(sumsq, mfl_amd.client_sqdist(x, out, P))


@pytest.mark.parametrize("K", [16, 17, 32, 33, 64, 65, 128, 129, 192, 193, 320, 321, 368, 369, 512, 513, 1024])
def test_fused_plan_boundaries_bit_exact(K):
    """Both sides of every switch of fused_plan (register-staged 256 / 128
    columns, LDS-DMA 128 / 64, register-staged 64 / 32 columns with 16 / 10 /
    16 slots, split-row windows of up to 8 / 16 waves): the reduce's bits,
    sums within 1e-12 of the two-pass sums, on a ragged P (NaN padding) and a
    P that leaves some workgroups no tile."""
    for P in (64 * 1000 + 3, 12_345):
        x, ld, weights = _rows(K, P, K * 31 + P)
        w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
        out, sumsq = mfl_amd.reduce_with_sqdist(x, w, P)
        ref_out = mfl_amd.reduce_packed(x, w, P)
        assert torch.equal(out.view(torch.int32), ref_out.view(torch.int32)), (K, P)
        ref = mfl_amd.client_sqdist(x, ref_out, P)
        rel = ((sumsq - ref).abs() / ref).max().item()
        assert rel < 1e-12, (K, P, rel)


def test_fused_rejects_unaligned_rows():
    """Unaligned rows: fedavg_reduce_sqdist_f32 refuses them up front (its
    distance pass reads 16-B slices) and the drop-in never sends them there."""
    K, P = 5, 1001
    x, ld, weights = _rows(K, P + 8, 9)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    lib = mfl_amd._lib.load()
    view = x[:, 1:]  # 4-B aligned rows
    out = torch.empty(P, device=DEV)
    s = torch.empty(K, dtype=torch.float64, device=DEV)
    ws = torch.empty(max(1, lib.fedavg_reduce_sqdist_workspace(K, P)), dtype=torch.float64, device=DEV)
    rc = lib.fedavg_reduce_sqdist_f32(view.data_ptr(), K, P, ld, w.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                      ws.numel(), s.data_ptr(), None)
    assert rc == mfl_amd._lib.FEDAVG_EALIGN
    from mfl_amd.aggregate import fuse_eligible

    assert not fuse_eligible(view) and fuse_eligible(x)


def test_fused_target_size_matches_two_pass():
    """100 x 25M (the north-star round): the reduce's bits on every column,
    sums within 1e-12 of the two-pass sums."""
    K, P = 100, 25_000_000 + 3
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn((K, ld), generator=g, device=DEV) * 0.05
    w = mfl_amd.weights_tensor(mfl_amd.sample_weights(list(range(1, K + 1))), torch.float32, DEV)
    out, sumsq = mfl_amd.reduce_with_sqdist(x, w, P)
    ref_out = mfl_amd.reduce_packed(x, w, P)
    assert torch.equal(out.view(torch.int32), ref_out.view(torch.int32))
    ref = mfl_amd.client_sqdist(x, ref_out, P)
    rel = ((sumsq - ref).abs() / ref).max().item()
    assert rel < 1e-12, rel
    del x


def test_fused_variants_same_bits():
    lib = mfl_amd._lib.load_probe()
    K, P = 100, 600_372
    x, ld, weights = _rows(K, P, 3)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out0, s0 = mfl_amd.reduce_with_sqdist(x, w, P)
    n_ws = K * 256 * 8
    work = torch.empty(n_ws, dtype=torch.float64, device=DEV)
    # tile width (+1000 double-buffered, +10000 rows per wave), workgroups per CU
    # register-staged (200000 + S, 1800000 + S: 16 slots), two tiles in flight
    # (+ 10000000), XCD / CU-contiguous sweeps (2200064, 4200064)
    for cols, bpc in [(64, 0), (128, 0), (128, 1), (64, 2), (256, 0), (1064, 0), (10064, 0), (10128, 0), (11128, 0),
                      (200064, 0), (200032, 0), (1800064, 0), (1800032, 0), (10200064, 0), (2200064, 0), (4200064, 0),
                      (200064, 3)]:
        out = torch.empty(P, device=DEV)
        s = torch.empty(K, dtype=torch.float64, device=DEV)
        mfl_amd._lib.check(lib.fedavg_reduce_sqdist_f32_variant(x.data_ptr(), K, P, ld, w.data_ptr(), out.data_ptr(),
                                                                work.data_ptr(), n_ws, s.data_ptr(), cols, bpc,
                                                                None), f"cols {cols} bpc {bpc}", lib)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), out0.view(torch.int32)), (cols, bpc)
        rel = ((s - s0).abs() / s0).max().item()
        assert rel < 1e-12, (cols, bpc, rel)
    # two 256-column tiles of 100 rows (201 KB) exceed the CU's 160 KB of LDS
    rc = lib.fedavg_reduce_sqdist_f32_variant(x.data_ptr(), K, P, ld, w.data_ptr(), out.data_ptr(), work.data_ptr(),
                                              n_ws, s.data_ptr(), 1256, 0, None)
    assert rc == mfl_amd._lib.FEDAVG_EMODE


def test_fused_nonfinite_rows():
    """NaN/inf inside the model propagate as the reference's ops propagate
    them; NaN in the row padding never reaches the sums."""
    K, P = 4, 1030
    x, ld, weights = _rows(K, P, 9)
    x[1, 17] = float("inf")
    x[2, 500] = float("nan")
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, sumsq = mfl_amd.reduce_with_sqdist(x, w, P)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
    got = out.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    assert np.array_equal(got[~np.isnan(got)], exp[~np.isnan(exp)])
    ref = _sumsq_ref(x, out, P)
    assert torch.equal(torch.isnan(sumsq), torch.isnan(ref))


def _host_round(K, shapes, seed):
    g = torch.Generator().manual_seed(seed)
    w_locals = []
    for i in range(K):
        sd = {}
        for name, shp in shapes.items():
            if name.endswith("num_batches_tracked"):
                sd[name] = torch.tensor(10 + i, dtype=torch.int64)
            else:
                sd[name] = torch.randn(shp, generator=g) * 0.05
        w_locals.append((int(torch.randint(1, 500, (1,), generator=g)), sd))
    return w_locals


@pytest.mark.parametrize("K", [1, 9, 100, 128, 300, 512, 513, 1025])
def test_dropin_distances_from_the_fused_pass(K):
    """aggregate (host state_dicts) leaves the fused :291 sums; client_distances
    returns the reference's norms (torch.norm of the fp32 differences) from
    them -- client 0 (aliased to w_glob, :449) gets 0.  K = 1025 takes the
    two-pass route and gives the same norms."""
    import copy

    shapes = {"conv.weight": (32, 3, 5, 5), "conv.bias": (32,), "bn.num_batches_tracked": (),
              "fc.weight": (10, 3000), "fc.bias": (10,)}
    w_locals = _host_round(K, shapes, K)
    ref_locals = copy.deepcopy(w_locals)
    agg = mfl_amd.DeviceAggregator(DEV)
    agg.SMALL_ROUND_BYTES = 0  # the pipelined host path even for a few clients (small rounds: one native call)
    w_glob = agg.aggregate(w_locals)
    fused = agg._last.get("sumsq", {})
    assert (torch.float32 in fused) == (K <= 1024)
    norms = agg.client_distances(w_locals, w_glob)
    keys = list(shapes)
    exp = []
    for i, (_, sd) in enumerate(ref_locals):
        if i == 0:
            exp.append(0.0)
            continue
        d = torch.cat([(sd[k].reshape(-1) - w_glob[k].reshape(-1)).double() for k in keys])
        exp.append(float(torch.sqrt((d * d).sum()).float()))
    np.testing.assert_allclose(norms, np.array(exp), rtol=2e-7, atol=0)
    # the same round through the two passes (rows re-read): same fp32 norms up to one ulp
    agg2 = mfl_amd.DeviceAggregator(DEV)
    w_glob2 = agg2.aggregate(copy.deepcopy(ref_locals))
    agg2._last.pop("sumsq", None)
    locals2 = copy.deepcopy(ref_locals)
    locals2[0] = (locals2[0][0], w_glob2)
    norms2 = agg2.client_distances(locals2, w_glob2)
    np.testing.assert_allclose(norms, norms2, rtol=2e-7, atol=0)


def _device_round(K, shapes, seed, misalign=False):
    g = torch.Generator(device=DEV).manual_seed(seed)
    w_locals = []
    for i in range(K):
        sd = {}
        for name, shp in shapes.items():
            if name.endswith("num_batches_tracked"):
                sd[name] = torch.tensor(10 + i, dtype=torch.int64, device=DEV)
            else:
                t = torch.randn(shp, generator=g, device=DEV) * 0.05
                if misalign and i == K - 1 and name == "fc.weight":
                    buf = torch.empty(t.numel() + 1, device=DEV)  # a view one float into its storage
                    buf[1:].copy_(t.reshape(-1))
                    t = buf[1:].view(shp)
                sd[name] = t
        w_locals.append((int(torch.randint(1, 500, (1,), generator=torch.Generator().manual_seed(seed + i))), sd))
    return w_locals


@pytest.mark.parametrize("K,misalign", [(1, False), (7, False), (100, False), (129, False), (256, False), (12, True),
                                       (257, False), (600, False), (1025, False)])
def test_device_round_fused_segments(K, misalign):
    """Device-resident clients (separate tensors, an int64 buffer, ragged key
    sizes): the zero-copy round's average keeps the oracle's bits and the
    fused :291 sums give the reference's norms (tiles to 256 clients, split-row
    windows to 1024).  A misaligned client tensor or K > 1024 takes the
    two-pass route with the same results."""
    import copy

    shapes = {"conv.weight": (16, 3, 3, 3), "conv.bias": (16,), "bn.num_batches_tracked": (),
              "fc.weight": (10, 3001), "fc.bias": (10,), "head.weight": (257,)}
    w_locals = _device_round(K, shapes, 5 * K + misalign, misalign)
    host_locals = [(n, {k: v.cpu() for k, v in sd.items()}) for n, sd in w_locals]
    ref = O.aggregate_torch(copy.deepcopy(host_locals))
    agg = mfl_amd.DeviceAggregator(DEV)
    w_glob = agg.aggregate(w_locals)
    for k in shapes:
        got, exp = w_glob[k].cpu(), ref[k]
        assert got.dtype == exp.dtype, k
        assert torch.equal(got.reshape(-1).view(torch.int32), exp.reshape(-1).view(torch.int32)), k
    assert (torch.float32 in agg._last.get("sumsq", {})) == (K <= 1024 and not misalign)
    norms = agg.client_distances(w_locals, w_glob)
    keys = list(shapes)
    # :291's fp32 differences (int64 buffers promote to fp32), squared and summed exactly
    exp = [0.0] + [float(torch.sqrt(torch.cat([(sd[k].reshape(-1).float() - ref[k].reshape(-1)).double()
                                               for k in keys]).pow(2).sum()).float())
                   for _, sd in host_locals[1:]]
    np.testing.assert_allclose(norms, np.array(exp), rtol=2e-7, atol=0)


@pytest.mark.parametrize("P", [10_000_003, 11_227_812, 5_000_001, 25_000_003])
def test_client_sqdist_round_fill_schedules(P):
    """The :291 pass's 16- / 8- / 4-slice choice (round fill of the launch):
    every schedule within 1e-12 of fp64 sums of the fp32 differences."""
    K = 3
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(P)
    x = torch.full((K, ld), float("nan"), device=DEV)
    x[:, :P] = torch.randn((K, P), generator=g, device=DEV) * 0.05
    glob = torch.randn(ld, generator=g, device=DEV) * 0.05
    got = mfl_amd.client_sqdist(x, glob, P)
    ref = torch.stack([((x[k, :P] - glob[:P]).double() ** 2).sum() for k in range(K)])
    rel = ((got - ref).abs() / ref).max().item()
    assert rel < 1e-12, rel
    assert torch.equal(got, mfl_amd.client_sqdist(x, glob, P))
