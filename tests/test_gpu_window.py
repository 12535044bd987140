"""GPU parity of the wave-owned window kernels (reduce_sqdist_win_kernel):
the fused aggregate + :291 pass for 17-128 clients on long rows.

Every instance (KMAX rows x VEC columns per lane) is driven through the probe
entry at small shapes -- one window, ragged windows, K below KMAX (padding
rows weighted -0.0), NaN row padding -- and must give the oracle's bits
(fedavg_trainer.py:450-457) and :291 sums (fp32 difference, fp64 squares) of
the same fp32 differences within 1e-12; the production plan is then checked
on both sides of each K band at a length that selects the windows.
"""
import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
INSTANCES = [(16, 4), (32, 4), (48, 4), (64, 2), (80, 2), (100, 2), (128, 1)]
KIND_WIN = 3
KIND_WINN = 4


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
    return x, ld, mfl_amd.sample_weights(counts)


def _sumsq_ref(x, out, P):
    return torch.stack([((x[k, :P] - out[:P]).double() ** 2).sum() for k in range(x.shape[0])])


def _win(x, K, P, ld, w, kmax, vec, code=None):
    lib = mfl_amd._lib.load_probe()
    n_ws = K * 4 * 2048
    work = torch.empty(n_ws, dtype=torch.float64, device=DEV)
    out = torch.empty(P, device=DEV)
    s = torch.empty(K, dtype=torch.float64, device=DEV)
    code = code or 70000000 + kmax * 100 + 40 + vec
    mfl_amd._lib.check(lib.fedavg_reduce_sqdist_f32_variant(x.data_ptr(), K, P, ld, w.data_ptr(), out.data_ptr(),
                                                            work.data_ptr(), n_ws, s.data_ptr(), code, 0, None),
                       f"window {kmax}x{vec}", lib)
    return out, s


@pytest.mark.parametrize("kmax,vec", INSTANCES)
def test_window_instances_vs_oracle(kmax, vec):
    for K in sorted({1, 2, kmax // 2 + 1, kmax - 1, kmax}):
        for P in (1, 3, 64 * vec + 5, 100_003):
            x, ld, weights = _rows(K, P, kmax * 7919 + K * 131 + P)
            w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
            out, s = _win(x, K, P, ld, w, kmax, vec)
            exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
            assert out.cpu().numpy().view(np.uint32).tobytes() == exp.view(np.uint32).tobytes(), (kmax, vec, K, P)
            ref = _sumsq_ref(x, out, P)
            rel = ((s - ref).abs() / ref.clamp_min(1e-300)).max().item()
            assert rel < 1e-12, (kmax, vec, K, P, rel)
            _, again = _win(x, K, P, ld, w, kmax, vec)
            assert torch.equal(s, again)  # deterministic


def test_window_lds_rows_vs_oracle():
    """The 81-100 band's production form (rows 0..23 of the next window staged
    in LDS by LDS-DMA, weights read with v_readlane): oracle bits and sums at
    K = 25 .. 100, including a K whose padding rows start inside a batch."""
    lib = mfl_amd._lib.load_probe()
    for K in (25, 81, 97, 100):
        for P in (3, 133, 100_003):
            x, ld, weights = _rows(K, P, K * 7 + P)
            w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
            out, s = _win(x, K, P, ld, w, 100, 2, code=124000042)
            exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
            assert out.cpu().numpy().view(np.uint32).tobytes() == exp.view(np.uint32).tobytes(), (K, P)
            ref = _sumsq_ref(x, out, P)
            rel = ((s - ref).abs() / ref.clamp_min(1e-300)).max().item()
            assert rel < 1e-12, (K, P, rel)
    x, ld, weights = _rows(24, 1000, 1)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    work = torch.empty(24 * 8192, dtype=torch.float64, device=DEV)
    out = torch.empty(1000, device=DEV)
    s = torch.empty(24, dtype=torch.float64, device=DEV)
    rc = lib.fedavg_reduce_sqdist_f32_variant(x.data_ptr(), 24, 1000, ld, w.data_ptr(), out.data_ptr(), work.data_ptr(),
                                              work.numel(), s.data_ptr(), 124000042, 0, None)
    assert rc == mfl_amd._lib.FEDAVG_EMODE  # K <= 24: the LDS rows would hold padding rows


@pytest.mark.parametrize("kmax,vec", [(48, 4), (100, 2), (128, 1)])
def test_window_negative_zero_and_nonfinite(kmax, vec):
    """-0.0 everywhere keeps -0.0 through the padding rows' (+0 x -0.0) terms;
    inf / NaN inside the model propagate as the reference's ops do."""
    K, P = kmax - 3, 64 * vec * 3 + 1
    x, ld, weights = _rows(K, P, 5)
    x[:, :P] = -0.0
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, s = _win(x, K, P, ld, w, kmax, vec)
    assert torch.all(out.view(torch.int32) == torch.tensor(-0.0).view(torch.int32).item())
    assert torch.all(s == 0)
    x, ld, weights = _rows(K, P, 6)
    x[1, 17] = float("inf")
    x[2, P - 1] = float("nan")
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, s = _win(x, K, P, ld, w, kmax, vec)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
    got = out.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    assert np.array_equal(got[~np.isnan(got)], exp[~np.isnan(exp)])
    ref = _sumsq_ref(x, out, P)
    assert torch.equal(torch.isnan(s), torch.isnan(ref))


@pytest.mark.parametrize("K", [369, 400, 448, 512, 513, 640, 1024])
def test_split_windows_vs_oracle(K):
    """369-1024 clients take the split-row windows (ceil(K / 64) waves per
    64-column window, the chain handed from wave to wave): the average bit for
    bit against the oracle and the row reduce, the sums within 1e-12 of plain
    torch in fp64, deterministic -- one window, a ragged last window, more
    windows than workgroups."""
    lib = mfl_amd._lib.load_probe()
    for P in (1, 3, 64 + 5, 50_003):
        plan = lib.fedavg_fused_plan_of(K, P)
        assert plan // 1000000 == KIND_WINN and plan % 100 == (8 if K <= 512 else 16), plan
        x, ld, weights = _rows(K, P, K * 13 + P)
        w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
        out, s = mfl_amd.reduce_with_sqdist(x, w, P)
        exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
        assert out.cpu().numpy().tobytes() == exp.tobytes(), (K, P)
        assert torch.equal(out.view(torch.int32), mfl_amd.reduce_packed(x, w, P).view(torch.int32))
        ref = _sumsq_ref(x, out, P)
        rel = ((s - ref).abs() / ref.clamp_min(1e-300)).max().item()
        assert rel < 1e-12, (K, P, rel)
        _, again = mfl_amd.reduce_with_sqdist(x, w, P)
        assert torch.equal(s, again)


@pytest.mark.parametrize("K", [160, 192, 256, 270, 289, 320, 368])
def test_split_windows_low_band(K):
    """160-368 clients on long rows take the split-row windows too
    (prefetching the next window's first 8 rows per wave): sampled windows of
    the average bit-exact against the oracle, the whole average equal to the
    row reduce's bits, the sums within 1e-12 of plain torch in fp64."""
    lib = mfl_amd._lib.load_probe()
    P = 1_700_003
    plan = lib.fedavg_fused_plan_of(K, P)
    assert plan == KIND_WINN * 1000000 + 64 * 100 + 8, plan
    x, ld, weights = _rows(K, P, K * 7)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, s = mfl_amd.reduce_with_sqdist(x, w, P)
    _oracle_windows(x, out, weights, P, seed=K)
    assert torch.equal(out.view(torch.int32), mfl_amd.reduce_packed(x, w, P).view(torch.int32))
    ref = _sumsq_torch64(x, out, P)
    assert ((s - ref).abs() / ref).max().item() < 1e-12
    _, again = mfl_amd.reduce_with_sqdist(x, w, P)
    assert torch.equal(s, again)
    del x


def test_split_windows_cfg4_shard_and_nonfinite():
    """cfg4's per-rank shape at N = 8 (500 x 1.4M): sampled windows against
    the oracle, sums against torch fp64; then -0.0 and inf / NaN through the
    split windows as through the one-wave windows."""
    K, P = 500, 1_403_477
    x, ld, weights = _rows(K, P, 4)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, s = mfl_amd.reduce_with_sqdist(x, w, P)
    _oracle_windows(x, out, weights, P, seed=4)
    ref = _sumsq_torch64(x, out, P)
    assert ((s - ref).abs() / ref).max().item() < 1e-12
    del x
    K, P = 400, 64 * 3 + 1
    x, ld, weights = _rows(K, P, 5)
    x[:, :P] = -0.0
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, s = mfl_amd.reduce_with_sqdist(x, w, P)
    assert torch.all(out.view(torch.int32) == torch.tensor(-0.0).view(torch.int32).item())
    assert torch.all(s == 0)
    x, ld, weights = _rows(K, P, 6)
    x[1, 17] = float("inf")
    x[300, P - 1] = float("nan")
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, s = mfl_amd.reduce_with_sqdist(x, w, P)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
    got = out.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    assert np.array_equal(got[~np.isnan(got)], exp[~np.isnan(exp)])
    assert torch.equal(torch.isnan(s), torch.isnan(_sumsq_ref(x, out, P)))


@pytest.mark.parametrize("nsmax,pf,Ks", [(8, 8, (2, 63, 64, 65, 200, 511, 512)), (16, 16, (513, 777, 1024)),
                                          (16, 8, (70, 640)), (8, 16, (129, 448))])
def test_split_windows_handoff_kernel_vs_oracle(nsmax, pf, Ks):
    """reduce_sqdist_winf_kernel (the production split windows: LDS flags
    instead of barriers, broadcast weights, PF prefetched rows) through the
    probe entry at every wave count it serves, K below a multiple of 64
    (padding rows weighted -0.0), one window, a ragged last window and more
    windows than workgroups: the oracle's bits, sums within 1e-12 of torch
    fp64, deterministic."""
    code = 91000000 + pf * 100 + nsmax
    for K in Ks:
        for P in (1, 67, 64 * 7 + 3, 2_000_003 if K in (Ks[0], Ks[-1]) else 40_001):
            x, ld, weights = _rows(K, P, K * 31 + P)
            w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
            out, s = _win(x, K, P, ld, w, 0, 0, code=code)
            if P <= 64 * 7 + 3:
                exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
                assert out.cpu().numpy().view(np.uint32).tobytes() == exp.view(np.uint32).tobytes(), (K, P)
            else:
                _oracle_windows(x, out, weights, P, n=3, width=min(2053, P // 4), seed=K)
            assert torch.equal(out.view(torch.int32), mfl_amd.reduce_packed(x, w, P).view(torch.int32)), (K, P)
            ref = _sumsq_torch64(x, out, P)
            rel = ((s - ref).abs() / ref.clamp_min(1e-300)).max().item()
            assert rel < 1e-12, (K, P, rel)
            _, again = _win(x, K, P, ld, w, 0, 0, code=code)
            assert torch.equal(s, again)
            del x


def test_split_windows_handoff_kernel_bounds():
    """The hand-off kernel refuses K past its waves and K < 2 (EMODE; the
    probe entry itself refuses K > 1024 first, EINVAL)."""
    lib = mfl_amd._lib.load_probe()
    for K, code in ((513, 91000808), (1, 91000808), (1025, 91001616)):
        x, ld, weights = _rows(K, 100, 1)
        w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
        work = torch.empty(K * 8192, dtype=torch.float64, device=DEV)
        out = torch.empty(100, device=DEV)
        s = torch.empty(K, dtype=torch.float64, device=DEV)
        rc = lib.fedavg_reduce_sqdist_f32_variant(x.data_ptr(), K, 100, ld, w.data_ptr(), out.data_ptr(), work.data_ptr(),
                                                  work.numel(), s.data_ptr(), code, 0, None)
        assert rc == (mfl_amd._lib.FEDAVG_EINVAL if K > 1024 else mfl_amd._lib.FEDAVG_EMODE), (K, code, rc)


def _oracle_windows(x, out, weights, P, n=6, width=2053, seed=0):
    """Sampled column windows of the fused output, bit for bit against the
    oracle (fedavg_trainer.py:450-457 restated) on host copies of the same
    columns: the first, the last and random ones."""
    rng = np.random.default_rng(seed)
    w32 = np.array([np.float32(v) for v in weights], dtype=np.float32)
    for s in sorted({0, P - width, *[int(v) for v in rng.integers(0, P - width, size=n)]}):
        exp = O.reduce_f32(x[:, s:s + width].cpu().numpy(), w32)
        got = out[s:s + width].cpu().numpy()
        assert got.tobytes() == exp.tobytes(), f"window at column {s}"


def _sumsq_torch64(x, out, P, step=1 << 20):
    """:291's sums of squares by plain torch: the fp32 difference as the
    reference forms it, squared and summed in fp64 (column chunks)."""
    tot = torch.zeros(x.shape[0], dtype=torch.float64, device=DEV)
    for c0 in range(0, P, step):
        c1 = min(P, c0 + step)
        tot += ((x[:, c0:c1] - out[None, c0:c1]).double() ** 2).sum(1)
    return tot


@pytest.mark.parametrize("K", [17, 48, 49, 64, 65, 80, 81, 100, 101, 128])
def test_window_plan_bands_bit_exact(K):
    """Long rows: the production plan takes the window instance of K's band;
    sampled windows of its average bit-exact against the oracle, its :291 sums
    within 1e-12 of a plain-torch fp64 reference, and the whole average equal
    to the production row reduce's bits."""
    lib = mfl_amd._lib.load_probe()
    P = 8_400_000 + 3
    plan = lib.fedavg_fused_plan_of(K, P)
    assert plan // 1000000 == KIND_WIN, plan
    kmax, vec = (plan // 100) % 10000, plan % 100
    assert K <= kmax and (kmax, vec) in INSTANCES
    x, ld, weights = _rows(K, P, K * 31)
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, sumsq = mfl_amd.reduce_with_sqdist(x, w, P)
    _oracle_windows(x, out, weights, P, seed=K)
    ref = _sumsq_torch64(x, out, P)
    rel = ((sumsq - ref).abs() / ref).max().item()
    assert rel < 1e-12, (K, rel)
    ref_out = mfl_amd.reduce_packed(x, w, P)
    assert torch.equal(out.view(torch.int32), ref_out.view(torch.int32)), K
    del x


def test_window_target_sampled_oracle():
    """The north-star round, 100 clients x 25M (the drop-in's fused window
    pass, reduce_sqdist_win_kernel<100, 2>): clients generated on the device by
    mfl_amd.synthetic, every sampled window of the average bit-exact against the
    oracle applied to the same columns regenerated on the host by numpy, the
    :291 sums within 1e-12 of plain torch in fp64."""
    from mfl_amd import synthetic

    K, P = 100, 25_000_000
    ld = (P + 63) // 64 * 64
    rows = torch.empty((K, ld), device=DEV)
    synthetic.fill_rows(rows, [(0, 0, P)])
    weights = mfl_amd.sample_weights(synthetic.sample_counts(K))
    w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
    out, sumsq = mfl_amd.reduce_with_sqdist(rows, w, P)
    torch.cuda.synchronize()
    rng = np.random.default_rng(11)
    for s in [0, P - 4099, *[int(v) for v in rng.integers(0, P - 4099, size=10)]]:
        exp = O.reduce_f32(synthetic.client_columns_numpy(K, s, 4099), weights)
        assert out[s:s + 4099].cpu().numpy().tobytes() == exp.tobytes(), f"window at column {s}"
    ref = _sumsq_torch64(rows, out, P)
    assert ((sumsq - ref).abs() / ref).max().item() < 1e-12
    del rows
    torch.cuda.empty_cache()


def test_window_plan_short_rows_and_other_k():
    """Short rows keep the tile kernels (resnet56 x 100, 100 x 3M); K <= 16 and
    K > 128 never take the windows; the target (100 x 25M) does."""
    lib = mfl_amd._lib.load_probe()
    assert lib.fedavg_fused_plan_of(100, 600_372) // 1000000 != KIND_WIN
    assert lib.fedavg_fused_plan_of(100, 3_125_000) // 1000000 != KIND_WIN
    assert lib.fedavg_fused_plan_of(100, 25_000_000) == KIND_WIN * 1000000 + 100 * 100 + 2
    for K in (1, 16, 129, 300, 512):
        assert lib.fedavg_fused_plan_of(K, 25_000_000) // 1000000 != KIND_WIN
    # split-row windows from 369 rows: up to 8 waves per group to 512, 16 to 1024; then two passes
    assert lib.fedavg_fused_plan_of(369, 25_000_000) == KIND_WINN * 1000000 + 64 * 100 + 8
    assert lib.fedavg_fused_plan_of(369, 1_000) == KIND_WINN * 1000000 + 64 * 100 + 8
    # ... and (the hand-off kernel, round 6) 160-368 rows when each workgroup gets >= 8 windows
    for K in (160, 161, 200, 256, 257, 288, 289, 320, 368):
        assert lib.fedavg_fused_plan_of(K, 25_000_000) == KIND_WINN * 1000000 + 64 * 100 + 8, K
        assert lib.fedavg_fused_plan_of(K, 100_000) // 1000000 == 2, K  # < 8 windows per workgroup
    for K in (129, 159):
        assert lib.fedavg_fused_plan_of(K, 25_000_000) // 1000000 == 2, K
    assert lib.fedavg_fused_plan_of(512, 25_000_000) == KIND_WINN * 1000000 + 64 * 100 + 8
    assert lib.fedavg_fused_plan_of(513, 25_000_000) == KIND_WINN * 1000000 + 64 * 100 + 16
    assert lib.fedavg_fused_plan_of(1024, 1_000) == KIND_WINN * 1000000 + 64 * 100 + 16
    assert lib.fedavg_fused_plan_of(1025, 25_000_000) == 0
    # the LDS-DMA tiles' weak band (65-96 rows) keeps the windows down to 400K columns
    assert lib.fedavg_fused_plan_of(70, 600_000) == KIND_WIN * 1000000 + 80 * 100 + 2
    assert lib.fedavg_fused_plan_of(90, 400_000) == KIND_WIN * 1000000 + 100 * 100 + 2
    assert lib.fedavg_fused_plan_of(96, 1_500_000) == KIND_WIN * 1000000 + 100 * 100 + 2
    assert lib.fedavg_fused_plan_of(90, 399_999) // 1000000 != KIND_WIN
    assert lib.fedavg_fused_plan_of(97, 1_500_000) // 1000000 != KIND_WIN
    assert lib.fedavg_fused_plan_of(64, 1_500_000) // 1000000 != KIND_WIN


WIN_DEVICE_SHAPES = [("layer.weight", (8_400_017,)), ("layer.bias", (1001,)), ("tiny", (3,)),
                     ("proj.weight", (800, 1000)), ("proj.bias", (640,))]


@pytest.mark.parametrize("K,int_keys", [(20, False), (64, False), (81, True), (100, False), (100, True),
                                         (128, False), (128, True)])
def test_window_device_clients_bit_exact(K, int_keys):
    """Device-resident clients of a model long enough for the zero-copy
    windows (reduce_sqdist_segwin_kernel; 81-100 clients on its 100 x 2
    instance since round 4): ragged key ends at every window width, keys
    shorter than a window, and (int_keys) BatchNorm-style int64
    num_batches_tracked buffers (above 2^24) plus an int32 key, converted to
    fp32 on the device so the fp32 window kernel takes the round; the
    aggregate's bits against the reference loop on host copies, the fused :291
    distances within one fp32 unit of the exact restatement."""
    from collections import OrderedDict

    from test_gpu_model_shapes import _check_distances, _oracle

    torch.cuda.empty_cache()
    g = torch.Generator(device=DEV).manual_seed(K)
    base = {k: torch.randn(s, generator=g, device=DEV) * 0.05 for k, s in WIN_DEVICE_SHAPES}
    w_locals = []
    for i in range(K):
        sd = OrderedDict()
        for j, (k, s) in enumerate(WIN_DEVICE_SHAPES):
            sd[k] = base[k] + torch.randn(s, generator=g, device=DEV) * 1e-3
            if int_keys and j in (0, 2):
                sd[f"bn{j}.num_batches_tracked"] = torch.tensor((1 << 25) + 7 * i + j, dtype=torch.int64, device=DEV)
        if int_keys:
            sd["counts32"] = torch.arange(i, i + 37, dtype=torch.int32, device=DEV)
        w_locals.append((int(np.random.default_rng(i).integers(1, 1000)), sd))
    expected = _oracle(w_locals)
    out = mfl_amd.aggregate(w_locals, device=DEV)
    for k, e in expected.items():
        assert torch.equal(out[k].cpu().reshape(-1).view(torch.int32), e.reshape(-1).view(torch.int32)), k
    if int_keys:
        agg = mfl_amd.default_aggregator(DEV)
        assert agg._last.get("sumsq"), "the fused pass took the round"
    _check_distances(w_locals, out, max_checked=16)
    del w_locals, out, expected, base
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kh,vec", [(50, 2), (40, 2), (32, 2), (25, 4), (60, 2), (50, 4)])
def test_split_row_windows_vs_oracle(kh, vec):
    """The split-row probe (reduce_sqdist_win2_kernel: two waves per window,
    the chain handed from rows 0..KH-1 to KH..2KH-1 over LDS): oracle bits and
    sums with K inside the first wave, across the split and at 2 KH."""
    for K in sorted({1, kh - 1, kh, kh + 1, 2 * kh - 3, 2 * kh}):
        for P in (1, 3, 64 * vec + 5, 100_003):
            x, ld, weights = _rows(K, P, kh * 7127 + K * 31 + P)
            w = mfl_amd.weights_tensor(weights, torch.float32, DEV)
            out, s = _win(x, K, P, ld, w, kh, vec, code=80000000 + kh * 100 + vec)
            exp = O.reduce_f32(x[:, :P].cpu().numpy(), np.array([np.float32(v) for v in weights], dtype=np.float32))
            assert out.cpu().numpy().view(np.uint32).tobytes() == exp.view(np.uint32).tobytes(), (kh, vec, K, P)
            ref = _sumsq_ref(x, out, P)
            rel = ((s - ref).abs() / ref.clamp_min(1e-300)).max().item()
            assert rel < 1e-12, (kh, vec, K, P, rel)
