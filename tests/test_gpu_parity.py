"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden vectors.  Run on the MI355X box: ``pytest -m gpu``.

Bar: bit-exact for the fp32/fp64/fp16/bf16 exact kernels (NaN positions must
match; NaN payload bits are not compared -- x86 and gfx950 produce different
default-NaN patterns and IEEE 754 leaves them unspecified).  The split-client
fp32 variant is tolerance-gated: norm-wise relative error <= 1e-6 (the
north-star tolerance) and identical bits run to run.
"""
import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd
from golden_io import case_names, load_case

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def assert_bits(got: torch.Tensor, exp: torch.Tensor, what=""):
    got = got.detach().cpu()
    exp = exp.detach().cpu()
    assert got.dtype == exp.dtype, (what, got.dtype, exp.dtype)
    assert tuple(got.shape) == tuple(exp.shape), (what, got.shape, exp.shape)
    if got.dtype == torch.bool:
        assert torch.equal(got, exp), what
        return
    g = got.reshape(-1)
    e = exp.reshape(-1)
    if got.is_floating_point():
        gn, en = torch.isnan(g), torch.isnan(e)
        assert torch.equal(gn, en), f"{what}: NaN positions differ"
        g = g[~gn]
        e = e[~en]
    gb = g.contiguous().view(torch.uint8).numpy()
    eb = e.contiguous().view(torch.uint8).numpy()
    if gb.tobytes() != eb.tobytes():
        gv, ev = g.numpy(), e.numpy()
        diff = np.nonzero(gv.astype(np.float64) != ev.astype(np.float64))[0]
        raise AssertionError(f"{what}: {len(diff)} mismatching elements, first {diff[:5]}: "
                             f"{gv[diff[:5]]} vs {ev[diff[:5]]}")


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield


def _w(weights, dtype=torch.float32):
    return mfl_amd.weights_tensor(weights, dtype, DEV)


# ---------------------------------------------------------------------------
# golden vectors through the drop-in (host state_dicts in, host state_dict out)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", [c for c in case_names() if c != "empty_w_locals"])
def test_dropin_matches_reference_golden(name):
    meta, w_locals, expected = load_case(name)
    first = w_locals[0][1] if w_locals else None
    others = [dict(sd) for _, sd in w_locals[1:]]
    out = mfl_amd.aggregate(w_locals)
    assert out is first  # fedavg_trainer.py:449 aliasing
    assert list(out.keys()) == list(expected.keys())
    for k, exp in expected.items():
        assert out[k].device.type == "cpu"
        assert_bits(out[k], exp, f"{name}/{k}")
    for d, (_, sd) in zip(others, w_locals[1:]):  # other clients untouched
        assert all(d[k] is sd[k] for k in d)


def test_dropin_repeated_rounds_reuse_staging():
    agg = mfl_amd.DeviceAggregator(DEV)
    for name in ["mnist_lr_k10", "mnist_lr_k100", "mnist_lr_k10", "resnet_like_bn_k5"]:
        _, w_locals, expected = load_case(name)
        out = agg.aggregate(w_locals)
        for k in expected:
            assert_bits(out[k], expected[k], name)


@pytest.mark.parametrize("small_bytes", [0, 1 << 30])
def test_small_round_native_path_and_pipelined_path_agree(small_bytes):
    """fedavg_round_f32 (one native call) and the pipelined torch-stream path
    give the reference's bits; both leave the round's rows in HBM for :291."""
    for name in ["mnist_lr_k10", "mnist_lr_k100", "resnet_like_bn_k5", "int_dtypes_k3", "adversarial_k10",
                 "flat_k10_p65"]:
        meta, w_locals, expected = load_case(name)
        agg = mfl_amd.DeviceAggregator(DEV)
        agg.SMALL_ROUND_BYTES = small_bytes
        out = agg.aggregate(w_locals)
        for k, exp in expected.items():
            assert_bits(out[k], exp, f"{name}/{k} small_bytes={small_bytes}")
        has_bool = any(t.dtype == torch.bool for _, sd in w_locals[1:] for t in sd.values())
        if torch.float32 in agg._last.get("dev", {}) and not has_bool:  # :291 raises on bool buffers
            norms = agg.client_distances(w_locals, out)
            assert norms.shape == (len(w_locals),) and norms[0] == 0.0


def test_dropin_femnist_cnn_shape():
    # FEMNIST + CNN_DropOut (P = 1,206,590; 8 keys), K = 10
    shapes = [("conv2d_1.weight", (32, 1, 3, 3)), ("conv2d_1.bias", (32,)), ("conv2d_2.weight", (64, 32, 3, 3)),
              ("conv2d_2.bias", (64,)), ("linear_1.weight", (128, 9216)), ("linear_1.bias", (128,)),
              ("linear_2.weight", (62, 128)), ("linear_2.bias", (62,))]
    g = torch.Generator().manual_seed(3)
    base = {k: torch.randn(s, generator=g) * 0.05 for k, s in shapes}
    w_locals = []
    for i in range(10):
        sd = {k: base[k] + torch.randn(s, generator=g) * 1e-3 for k, s in shapes}
        w_locals.append((int(torch.randint(1, 1000, (1,), generator=g)), sd))
    import copy
    ref = O.aggregate_torch(copy.deepcopy(w_locals))
    out = mfl_amd.aggregate(w_locals)
    assert sum(t.numel() for t in out.values()) == 1_206_590
    for k in ref:
        assert_bits(out[k], ref[k], k)


# ---------------------------------------------------------------------------
# device-resident kernels vs the oracle
# ---------------------------------------------------------------------------
def _clients(K, P, ld=None, seed=0, dtype=torch.float32):
    ld = ld or max((P + 63) // 64 * 64, 64)
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn((K, ld), generator=g, device=DEV, dtype=torch.float32) * 0.05
    return x.to(dtype)


def _weights(K, seed=1234):
    n = np.random.default_rng(seed).integers(1, 1001, size=K)
    return O.sample_weights([int(v) for v in n])


@pytest.mark.parametrize("K", [1, 2, 3, 7, 8, 9, 16, 17, 33, 100, 257])
@pytest.mark.parametrize("P", [1, 3, 4, 5, 63, 64, 65, 1000, 4097])
def test_reduce_f32_exact(K, P):
    x = _clients(K, P, seed=K * 1000 + P)
    w = _weights(K, seed=K + P)
    out = mfl_amd.reduce_packed(x, _w(w), P)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), w)
    assert_bits(out, torch.from_numpy(exp), f"K={K} P={P}")


@pytest.mark.parametrize("K,P", [(10, 1 << 20), (100, 600_372), (37, 3_000_001)])
def test_reduce_f32_exact_large(K, P):
    x = _clients(K, P, seed=P)
    w = _weights(K, seed=K)
    out = mfl_amd.reduce_packed(x, _w(w), P)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), w)
    assert_bits(out, torch.from_numpy(exp), f"K={K} P={P}")


def _schedule_boundary_cases():
    """(K, P) on both sides of every production-schedule switch: the slice
    count per thread steps at 2 x CUs x 256 threads x {2, 4, 8} float4
    columns and at 2 x CUs x 256 x 16 (the buffer-descriptor U2 x C16
    kernel), the Infinity-Cache band spans 64-240 MiB of client rows, and
    K <= 4 takes the single-launch path."""
    full = 2 * torch.cuda.get_device_properties(DEV).multi_processor_count
    cases = []
    for c in (2, 4, 8):
        t = full * 256 * c * 4  # elements at the switch
        cases += [(5, t - 4), (5, t - 1), (5, t), (5, t + 3)]
    t = full * 256 * 16 * 4  # fp32 only: U2 x C16 buffer-descriptor kernel from here
    cases += [(5, t - 4), (5, t), (5, t + 3)]
    # K >= 64: 4 slices per thread in the short-row bands (from full/4 x 256 x 4 float4 columns)
    for t in (full // 4 * 256 * 4 * 4, full * 256 * 2 * 4):
        cases += [(64, t - 4), (64, t + 1), (63, t + 1), (100, t - 1)]
    # one block per CU at 6 slices (K >= 64) or 3 slices (K >= 256) per thread
    cus = full // 2
    for c, K in ((6, 100), (3, 256)):
        lo, hi = cus * 3 // 4 * 256 * c * 4, cus * 256 * c * 4
        cases += [(K, lo - 4), (K, lo + 1), (K, hi - 1), (K, hi + 4), (K - 1, lo + 1)]
    # 5 <= K < 64: buffer-descriptor U8 x C2 in the 4-slice band, U8 x C1 for
    # 8 <= K <= 32 from full/2 x 256 float4 columns
    for t in (full * 256 * 4 * 4, full * 256 * 8 * 4):
        cases += [(5, t - 1), (5, t + 1), (63, t - 4), (63, t + 3), (64, t + 3)]
    t = full * 256 // 2 * 4
    cases += [(8, t - 4), (8, t + 1), (32, t + 3), (33, t + 3), (7, t + 5), (10, 1_206_590)]
    mib = 1 << 20
    cases += [(20, 64 * mib // 80 - 3), (20, 64 * mib // 80 + 5), (20, 240 * mib // 80 - 1), (20, 240 * mib // 80 + 7)]
    cases += [(4, 1_000_003), (5, 1_000_003), (1, 65), (2, 7)]
    return cases


def test_dropin_random_state_dicts_bit_exact():
    """30 seeded random rounds through the drop-in: 1-40 clients, 1-12 keys of
    random shapes (0-d to 4-d), fp32 with int64 / int32 / bool buffers and
    now and then an fp64, fp16 or bf16 key, sample counts 1..10^6; one
    aggregator across rounds (staging reuse, key-table reuse and rebuild)."""
    import copy
    from collections import OrderedDict
    rng = np.random.default_rng(77)
    agg = mfl_amd.DeviceAggregator(DEV)
    extra = [torch.float64, torch.float16, torch.bfloat16]
    for case in range(30):
        K = int(rng.integers(1, 41))
        keys = []
        for j in range(int(rng.integers(1, 13))):
            shape = tuple(int(d) for d in rng.integers(1, 40, size=int(rng.integers(0, 5))))
            r = rng.random()
            dt = (torch.float32 if r < 0.7 else torch.int64 if r < 0.8 else torch.int32 if r < 0.85
                  else torch.bool if r < 0.9 else extra[int(rng.integers(0, 3))])
            keys.append((f"k{j}", shape, dt))
        g = torch.Generator().manual_seed(case)
        w_locals = []
        for i in range(K):
            sd = OrderedDict()
            for name, shape, dt in keys:
                if dt == torch.bool:
                    sd[name] = torch.rand(shape, generator=g) > 0.5
                elif not dt.is_floating_point:
                    sd[name] = torch.randint(-1000, 1000, shape, generator=g).to(dt)
                else:
                    sd[name] = (torch.randn(shape, generator=g) * 0.05).to(dt)
            w_locals.append((int(rng.integers(1, 10**6)), sd))
        ref = O.aggregate_torch(copy.deepcopy(w_locals))
        out = agg.aggregate(w_locals)
        assert out is w_locals[0][1]
        for k in ref:
            assert_bits(out[k], ref[k], f"case {case} key {k}")


def test_random_shapes_strides_and_offsets_bit_exact():
    """60 seeded random problems: K in [1, 300], P in [1, 300K], row stride
    ld >= P with NaN in the padding (it must never leak into a result), the
    buffer start at a 4/8/12-byte offset now and then (scalar path), and an
    output written into a larger NaN-filled buffer (nothing outside [0, P))."""
    rng = np.random.default_rng(2024)
    for case in range(60):
        K = int(rng.integers(1, 301))
        P = int(rng.integers(1, 300_001)) if case % 3 else int(rng.integers(1, 5000))
        pad = int(rng.choice([0, 1, 3, 4, 60, 64, 1000]))
        off = int(rng.choice([0, 0, 0, 1, 2, 3]))
        ld = P + pad + off
        store = torch.full((K * ld + 8,), float("nan"), device=DEV)
        x = store[off:off + K * ld].view(K, ld)
        x[:, :P] = torch.randn((K, P), device=DEV, generator=torch.Generator(device=DEV).manual_seed(case)) * 0.05
        w = _weights(K, seed=case)
        big = torch.full((P + 16,), float("nan"), device=DEV)
        out = mfl_amd.reduce_packed(x, _w(w), P, out=big[4:4 + P])
        exp = O.reduce_f32(x[:, :P].cpu().numpy(), w)
        assert_bits(out, torch.from_numpy(exp), f"case {case}: K={K} P={P} ld={ld} off={off}")
        assert torch.isnan(big[:4]).all() and torch.isnan(big[4 + P:]).all(), f"case {case}: wrote outside out"


def test_chunk_of_wider_shard_streams_and_is_bit_exact():
    """A column chunk of a wider row buffer (ld > P, the N > 1 pipeline) does
    not take the Infinity-Cache schedule; the result is bit-exact either way."""
    from mfl_amd import _lib
    K, S, C = 100, 390_656, 3
    assert _lib.f32_schedule(K, S)["nontemporal"] == 0          # alone: cache-resident band
    assert _lib.f32_schedule(K, S, S * C)["nontemporal"] == 1   # chunk of a 3x wider shard: streamed
    x = _clients(K, S * C, seed=3)
    w = _weights(K, seed=4)
    for j in range(C):
        out = mfl_amd.reduce_packed(x[:, j * S:(j + 1) * S], _w(w), S)
        exp = O.reduce_f32(x[:, j * S:(j + 1) * S].cpu().numpy(), w)
        assert_bits(out, torch.from_numpy(exp), f"chunk {j}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float64])
def test_chunk_of_wider_shard_other_dtypes(dtype):
    """fp16/bf16/fp64 chunks of a wider row buffer (streamed schedule) give
    the oracle's bits (O.reduce_f64 / O.reduce_half on the same columns) and
    those of the same columns reduced from a contiguous copy."""
    K, S, C = 100, 390_656, 3
    x = _clients(K, S * C, seed=5, dtype=dtype)
    wl = _weights(K, seed=6)
    w = _w(wl, torch.float64 if dtype == torch.float64 else torch.float32)
    iv = torch.int64 if dtype == torch.float64 else torch.int16
    for j in (0, C - 1):
        view = x[:, j * S:(j + 1) * S]
        got = mfl_amd.reduce_packed(view, w, S)
        ref = mfl_amd.reduce_packed(view.contiguous(), w, S)
        assert torch.equal(got.view(iv), ref.view(iv)), (dtype, j)
        host = view.cpu()
        if dtype == torch.float64:
            exp = torch.from_numpy(O.reduce_f64(host.numpy(), wl))
        elif dtype == torch.float16:
            exp = torch.from_numpy(O.reduce_half(host.numpy(), wl, "float16"))
        else:
            bits = O.reduce_half(host.view(torch.int16).numpy(), wl, "bfloat16")
            exp = torch.from_numpy(bits.view(np.int16).copy()).view(torch.bfloat16)
        assert_bits(got, exp, f"{dtype} chunk {j} vs oracle")


def test_schedule_switch_boundaries_bit_exact():
    for K, P in _schedule_boundary_cases():
        x = _clients(K, P, seed=K * 7 + P)
        w = _weights(K, seed=P)
        out = mfl_amd.reduce_packed(x, _w(w), P)
        exp = O.reduce_f32(x[:, :P].cpu().numpy(), w)
        assert_bits(out, torch.from_numpy(exp), f"K={K} P={P} schedule={mfl_amd._lib.f32_schedule(K, P)}")


@pytest.mark.parametrize("unroll", [4, 8, 16])
@pytest.mark.parametrize("nt", [0, 1])
def test_tuned_variants_bit_identical(unroll, nt):
    K, P = 45, 123_457
    x = _clients(K, P, seed=5)
    w = _w(_weights(K))
    base = mfl_amd.reduce_packed(x, w, P)
    got = mfl_amd.reduce_packed(x, w, P, tuned=(unroll, nt))
    assert_bits(got, base, f"unroll={unroll} nt={nt}")


def _all_variants():
    out = []
    for U in (1, 2, 4, 8, 16):
        for C in (1, 2, 4, 8, 16):
            if (C == 8 and U > 8) or (C == 16 and U > 2):
                continue
            for nt in (0, 1):
                for pipe in (0, 1, 2, 3, 4, 5):
                    if pipe in (1, 3) and U * C > 32:
                        continue
                    if pipe == 2 and U * C > 16:
                        continue
                    out.append((U, nt, C, pipe, 0))
    out += [(32, nt, C, pipe, 0) for nt in (0, 1) for C in (1, 2) for pipe in (0, 4)]
    return out + [(8, 1, 4, 0, 2048), (4, 1, 1, 2, 300), (16, 0, 2, 1, 7), (4, 1, 8, 3, 5), (2, 1, 8, 3, 333),
                  (4, 1, 8, 4, 3), (8, 1, 4, 4, 17), (8, 0, 1, 4, 1), (4, 1, 8, 5, 7), (8, 1, 8, 5, 256),
                  (2, 1, 16, 5, 1), (8, 1, 4, 5, 1000)]


def test_schedule_variants_bit_identical():
    """Every schedule of the exact kernel (register batches, double-buffered,
    LDS-DMA staging, multi-column, capped grid) gives the default's bits,
    including a ragged last column group and a P % 4 tail."""
    for K, P in [(37, 123_457), (1, 4099), (9, 1_000_003), (3, 64 * 64 * 3 + 5), (5, 190)]:
        x = _clients(K, P, seed=K + P)
        w = _w(_weights(K))
        base = mfl_amd.reduce_packed(x, w, P)
        exp = O.reduce_f32(x[:, :P].cpu().numpy(), _weights(K))
        assert_bits(base, torch.from_numpy(exp), f"default K={K} P={P}")
        for v in _all_variants():
            got = mfl_amd.reduce_packed(x, w, P, tuned=v)
            assert torch.equal(got.view(torch.int32), base.view(torch.int32)), (K, P, v)


@pytest.mark.parametrize("K,P", [(37, 123_457), (1, 4099), (9, 1_000_003), (3, 64 * 64 * 3 + 5), (5, 190),
                                 (100, 600_372)])
def test_buffer_descriptor_reduce_bit_identical(K, P):
    """fedavg_reduce_f32_buf (per-row buffer descriptors, 32-bit lane offsets)
    gives the production kernel's bits for every (U, C) and grid cap, with a
    ragged last column group and a P % 4 tail."""
    lib = mfl_amd._lib.load_probe()
    x = _clients(K, P, seed=K + 7 * P)
    w = _w(_weights(K))
    base = mfl_amd.reduce_packed(x, w, P)
    for u, c, bs, b in [(4, 8, 256, 0), (4, 8, 256, 3), (8, 4, 256, 0), (4, 4, 256, 5), (2, 8, 256, 0),
                        (2, 16, 256, 0), (1, 16, 256, 7), (8, 8, 256, 0), (16, 1, 256, 0), (16, 4, 256, 0),
                        (16, 1, 64, 0), (16, 2, 64, 11), (8, 4, 64, 0), (32, 1, 64, 0), (16, 1, 128, 0),
                        (8, 2, 128, 3), (4, 8, 128, 0)]:
        out = torch.full((P,), float("nan"), device=DEV)
        mfl_amd._lib.check(lib.fedavg_reduce_f32_buf(x.data_ptr(), K, P, x.shape[1], w.data_ptr(), out.data_ptr(),
                                                     u, c, bs, b, None), f"U{u}C{c}B{bs}b{b}", lib)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), base.view(torch.int32)), (K, P, u, c, bs, b)


def test_misaligned_clients_take_scalar_path():
    K, P = 6, 1001
    big = _clients(K, P + 1, ld=1088, seed=9)
    x = big[:, 1:]  # 4-byte offset: not 16-B aligned, ld stays 1088
    w = _weights(K)
    out = mfl_amd.reduce_packed(x, _w(w), P)
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), w)
    assert_bits(out, torch.from_numpy(exp))


def test_odd_ld_and_misaligned_out():
    K, P = 5, 999
    x = _clients(K, P, ld=1001, seed=10)
    w = _weights(K)
    out_big = torch.empty(P + 1, device=DEV)
    out = mfl_amd.reduce_packed(x, _w(w), P, out=out_big[1:])
    exp = O.reduce_f32(x[:, :P].cpu().numpy(), w)
    assert_bits(out[:P], torch.from_numpy(exp))


def test_ptrs_variant_mixed_alignment():
    K, P = 9, 10_003
    store = _clients(K, P + 4, seed=12)
    clients = [store[i, (i % 4):(i % 4) + P] for i in range(K)]  # 0/4/8/12-byte offsets
    w = _weights(K)
    out = mfl_amd.reduce_tensors(clients, _w(w))
    exp = O.reduce_f32(np.stack([c.cpu().numpy() for c in clients]), w)
    assert_bits(out, torch.from_numpy(exp))


# units of 4,096 columns: below one unit, exact units, one past, the U4 batch
# remainder (K - 1) % 4 in 0..3, and more units than one launch (3 x CUs)
@pytest.mark.parametrize("K,P", [(1, 3), (2, 4096), (4, 4097), (5, 8192 + 5), (8, 12_288), (13, 777),
                                 (100, 3_200_003)])
def test_ptrs_variant_units(K, P):
    clients = [_clients(1, P, seed=500 + i)[0, :P].clone() for i in range(K)]
    w = _weights(K)
    out_big = torch.empty(P + 1, device=DEV)
    out = mfl_amd.reduce_tensors(clients, _w(w), out=out_big[1:])  # dword-aligned output
    exp = O.reduce_f32(torch.stack(clients).cpu().numpy(), w)
    assert_bits(out, torch.from_numpy(exp))


@pytest.mark.parametrize("K,P", [(3, 33), (10, 4099), (64, 100_000)])
def test_reduce_f64_exact(K, P):
    x = _clients(K, P, seed=P, dtype=torch.float64)
    w = _weights(K)
    out = mfl_amd.reduce_packed(x, _w(w, torch.float64), P)
    exp = O.reduce_f64(x[:, :P].cpu().numpy(), w)
    assert_bits(out, torch.from_numpy(exp))


@pytest.mark.parametrize("kind", ["float16", "bfloat16"])
@pytest.mark.parametrize("K,P", [(3, 70), (10, 4099), (50, 65_536)])
def test_reduce_half_exact(kind, K, P):
    dt = torch.float16 if kind == "float16" else torch.bfloat16
    x = _clients(K, P, seed=P + K, dtype=dt)
    w = _weights(K)
    out = mfl_amd.reduce_packed(x, _w(w), P)
    xs = x[:, :P].cpu()
    if kind == "float16":
        exp = torch.from_numpy(O.reduce_half(xs.numpy(), w, kind))
    else:
        bits = O.reduce_half(xs.view(torch.int16).numpy(), w, kind)
        exp = torch.from_numpy(bits.view(np.int16).copy()).view(torch.bfloat16)
    assert_bits(out, exp, kind)


@pytest.mark.parametrize("kind", ["float16", "bfloat16"])
@pytest.mark.parametrize("K,P", [(7, 4099), (40, 70_001)])
def test_reduce_half_adversarial_bit_patterns(kind, K, P):
    """Random 16-bit patterns: subnormals, near-overflow, +-inf, NaNs of every
    payload and sign.  Bit-exact vs the oracle; NaN positions must match, and
    for bf16 every NaN is c10's canonical 0x7FC0 (the packed kernel
    canonicalises at the store)."""
    dt = torch.float16 if kind == "float16" else torch.bfloat16
    rng = np.random.default_rng(P + K)
    ld = (P + 63) // 64 * 64
    bits = rng.integers(0, 1 << 16, size=(K, ld), dtype=np.uint16)
    # keep most lanes finite so that not every column ends up NaN
    expo_mask = np.uint16(0x7C00 if kind == "float16" else 0x7F80)
    special = rng.random((K, ld)) < 0.9
    bits[special & ((bits & expo_mask) == expo_mask)] ^= np.uint16(0x4000)
    x = torch.from_numpy(bits.view(np.int16)).view(dt).to(DEV)
    w = _weights(K)
    out = mfl_amd.reduce_packed(x, _w(w), P)
    xs = x[:, :P].cpu()
    if kind == "float16":
        exp = torch.from_numpy(O.reduce_half(xs.numpy(), w, kind))
    else:
        eb = O.reduce_half(xs.view(torch.int16).numpy(), w, kind)
        exp = torch.from_numpy(eb.view(np.int16).copy()).view(torch.bfloat16)
        got_bits = out.cpu().view(torch.int16).numpy().view(np.uint16)
        nan = np.isnan(O.bf16_bits_to_f32(got_bits))
        assert nan.any() and (got_bits[nan] == 0x7FC0).all()
    assert_bits(out, exp, kind)


def test_cvt16_hardware_rounding_equals_c10_all_fp32_inputs():
    """The packed kernels round with v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32.
    Over all 2^32 fp32 bit patterns: bf16 equals c10's integer
    round_to_nearest_even and fp16 the scalar v_cvt_f16_f32, for every
    non-NaN input (subnormals and overflow included); NaN stays NaN."""
    lib = mfl_amd._lib.load_probe()
    n = 1 << 28
    a = torch.empty(n, dtype=torch.int16, device=DEV)
    b = torch.empty(n, dtype=torch.int16, device=DEV)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    for chunk in range(16):
        inp = torch.arange(chunk * n, (chunk + 1) * n, dtype=torch.int64, device=DEV).to(torch.int32)
        nan_in = ((inp & 0x7F800000) == 0x7F800000) & ((inp & 0x7FFFFF) != 0)
        for hw, ref, expo, mant in [(0, 1, 0x7F80, 0x7F), (2, 3, 0x7C00, 0x3FF)]:
            mfl_amd._lib.check(lib.fedavg_probe_cvt16(inp.data_ptr(), n, hw, a.data_ptr(), stream), "probe")
            mfl_amd._lib.check(lib.fedavg_probe_cvt16(inp.data_ptr(), n, ref, b.data_ptr(), stream), "probe")
            same = (a == b) | nan_in
            assert bool(same.all()), (chunk, hw, int((~same).sum()))
            ai = a.to(torch.int32)
            nan_out = ((ai & expo) == expo) & ((ai & mant) != 0)
            assert bool((nan_out == nan_in).all()), (chunk, hw)


@pytest.mark.parametrize("splits", [2, 4, 8])
@pytest.mark.parametrize("K,P", [(3, 1000), (10, 7850), (100, 600_372), (500, 65_536)])
def test_splitk_within_tolerance_and_deterministic(splits, K, P):
    x = _clients(K, P, seed=P) * 0.02 + _clients(1, P, seed=P + 1)  # model-like: base + per-client noise
    w = _weights(K)
    a = mfl_amd.reduce_packed(x, _w(w), P, splits=splits)
    b = mfl_amd.reduce_packed(x, _w(w), P, splits=splits)
    assert_bits(a, b, "run-to-run")
    exp = torch.from_numpy(O.reduce_f32(x[:, :P].cpu().numpy(), w)).double()
    err = (a.cpu().double() - exp).norm() / exp.norm()
    assert err <= 1e-6, float(err)


# ---------------------------------------------------------------------------
# BASELINE.json full size (K = 100, P = 25M): sampled-column parity + properties
# ---------------------------------------------------------------------------
def test_target_size_sampled_parity():
    K, P = 100, 25_000_000
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(0)
    base = torch.randn(ld, generator=g, device=DEV) * 0.05
    x = torch.empty((K, ld), device=DEV)
    for k in range(K):
        gk = torch.Generator(device=DEV).manual_seed(1000 + k)
        x[k] = base + torch.randn(ld, generator=gk, device=DEV) * 1e-3
    w = _weights(K)
    out = mfl_amd.reduce_packed(x, _w(w), P)
    rng = np.random.default_rng(0)
    starts = list(rng.integers(0, P - 8192, size=16)) + [0, P - 4099]
    for s in starts:
        s = int(s)
        e = min(s + 4099, P)
        exp = O.reduce_f32(x[:, s:e].cpu().numpy(), w)
        assert_bits(out[s:e], torch.from_numpy(exp), f"window {s}")
    # every variant gives the same bits at full size (idempotence across launches)
    for tuned in [(4, 0), (16, 1)]:
        again = mfl_amd.reduce_packed(x, _w(w), P, tuned=tuned)
        assert torch.equal(again.view(torch.int32), out.view(torch.int32))
    # linearity sanity in fp64: |out - sum w_i x_i| small relative to the norm
    ref64 = torch.zeros(P, dtype=torch.float64, device=DEV)
    for k in range(K):
        ref64 += x[k, :P].double() * float(np.float32(w[k]))
    rel = (out.double() - ref64).norm() / ref64.norm()
    assert rel < 1e-6
    # the fused aggregate + :291 pass at full size: the same average bits, and
    # an exact scaling property of the whole vector -- doubling every client
    # doubles every product, sum and fp32 difference exactly (powers of two
    # commute with rounding away from overflow / subnormals), so the average
    # must come out exactly 2x and every client's fp64 sum of squares 4x
    out_f, sums = mfl_amd.reduce_with_sqdist(x, _w(w), P)
    assert torch.equal(out_f.view(torch.int32), out.view(torch.int32))
    x.mul_(2.0)
    out2, sums2 = mfl_amd.reduce_with_sqdist(x, _w(w), P)
    assert torch.equal(out2.view(torch.int32), (out * 2.0).view(torch.int32))
    assert torch.equal(sums2, sums * 4.0)
    del x


def test_sharded_reducer_single_rank_chunks():
    from mfl_amd.distributed import ShardedReducer
    K, P = 12, 100_003
    host = torch.randn((K, P)) * 0.05
    w = _weights(K)
    red = ShardedReducer(K, P, chunks=3, device=DEV)
    red.load_from_host(host)
    assert red.step(_w(w)) is None  # world size 1: no gather
    exp = O.reduce_f32(host.numpy(), w)
    got = torch.cat([v for v, _ in red.local_model_columns()])
    assert_bits(got, torch.from_numpy(exp))


def test_sharded_reducer_host_out():
    """SURVEY 8e host-consumer form: chunks D2H'd into pinned host memory, no collective."""
    from mfl_amd.distributed import ShardedReducer
    K, P = 9, 250_001
    host = torch.randn((K, P)) * 0.05
    w = _weights(K)
    out = torch.full((P,), float("nan"), pin_memory=True)
    red = ShardedReducer(K, P, chunks=4, device=DEV, host_out=out)
    red.load_from_host(host)
    for _ in range(2):  # second step rewrites the same host buffer
        got = red.step(_w(w))
        assert got.data_ptr() == out.data_ptr()
        assert_bits(got.clone(), torch.from_numpy(O.reduce_f32(host.numpy(), w)))
    with pytest.raises(ValueError):
        ShardedReducer(K, P, device=DEV, host_out=torch.empty(P))  # not pinned


@pytest.mark.parametrize("ws,chunks,K", [(1, 3, 7), (2, 1, 7), (3, 4, 7), (8, 8, 7), (3, 2, 1)])
def test_upload_segments_strided_dma(ws, chunks, K):
    """SURVEY 8e input distribution: every rank's column segments of a pinned
    host [K, P] buffer land in its device rows via one strided DMA each."""
    from mfl_amd.distributed import plan_shards, upload_segments
    P = 300_007
    host = torch.randn((K, P)).pin_memory()
    seen = torch.zeros(P, dtype=torch.int32)
    for r in range(ws):
        plan = plan_shards(P, ws, r, chunks)
        dst = torch.full((K, plan.local_cols), float("nan"), device=DEV)
        segs = plan.local_segments()
        upload_segments(dst, host, segs)
        torch.cuda.synchronize()
        got = dst.cpu()
        for l, g, n in segs:
            assert torch.equal(got[:, l:l + n], host[:, g:g + n]), (r, l, g, n)
            seen[g:g + n] += 1
    assert bool((seen == 1).all())  # the ranks' segments partition the columns


def test_upload_shard_rejects_pageable_source():
    lib = mfl_amd._lib.load()
    dst = torch.empty(64, device=DEV)
    src = torch.zeros(64)  # pageable
    assert lib.fedavg_upload_shard(dst.data_ptr(), 256, src.data_ptr(), 256, 256, 1, None) == -10001


def test_sharded_reducer_load_from_pinned_host_zero_padding():
    from mfl_amd.distributed import ShardedReducer
    K, P = 10, 1_000_003
    host = (torch.randn((K, P)) * 0.05).pin_memory()
    w = _weights(K)
    red = ShardedReducer(K, P, chunks=5, device=DEV)
    red.clients.fill_(float("nan"))
    red.load_from_host(host)
    red.step(_w(w))
    got = torch.cat([v for v, _ in red.local_model_columns()])
    assert_bits(got, torch.from_numpy(O.reduce_f32(host.numpy(), w)))
    valid = sum(n for _, _, n in red.plan.local_segments())
    assert not torch.isnan(red.clients).any()  # padding columns were zeroed
    assert valid == P


@pytest.mark.parametrize("P", [4_194_304 + 3, 17_000_021])
def test_aggregate_chunked_fetch_bit_exact(P):
    """P >= 2 x D2H_CHUNK_MIN_COLS: the reduce runs in column chunks with the
    D2H of chunk c overlapping the reduce of chunk c+1 (aggregate and session)."""
    from collections import OrderedDict

    K = 3
    g = torch.Generator().manual_seed(P)
    base = torch.randn(P, generator=g) * 0.05
    dicts = [OrderedDict(a=(base[:1000] + 1e-3 * torch.randn(1000, generator=g)).reshape(10, 100),
                         b=base[1000:] + 1e-3 * torch.randn(P - 1000, generator=g)) for _ in range(K)]
    counts = [17, 400, 3]
    w = O.sample_weights(counts)
    flat = np.stack([torch.cat([d["a"].reshape(-1), d["b"]]).numpy() for d in dicts])
    exp = torch.from_numpy(O.reduce_f32(flat, w))
    agg = mfl_amd.DeviceAggregator(DEV)
    wl = [(n, OrderedDict(d)) for n, d in zip(counts, dicts)]
    out = agg.aggregate(wl)
    assert_bits(torch.cat([out["a"].reshape(-1), out["b"]]), exp)
    sess = agg.begin_round(dicts[0], K)
    wl2 = [(n, OrderedDict(d)) for n, d in zip(counts, dicts)]
    for n, d in wl2:
        sess.add(n, d)
    out2 = sess.finish(wl2)
    assert_bits(torch.cat([out2["a"].reshape(-1), out2["b"]]), exp)


@pytest.mark.parametrize("nbytes", [16, 100, 4096 + 12, 50_000_016])
def test_copy_to_host_zero_copy(nbytes):
    lib = mfl_amd._lib.load()
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=DEV)
    dst = torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True)
    s = torch.cuda.current_stream(DEV)
    for blocks in (1, 64, 0):
        dst.zero_()
        mfl_amd._lib.check(lib.fedavg_copy_to_host(src.data_ptr(), dst.data_ptr(), nbytes, blocks, s.cuda_stream),
                           "copy")
        s.synchronize()
        assert torch.equal(dst, src.cpu())


def test_copy_to_host_rejects_pageable_memory():
    lib = mfl_amd._lib.load()
    src = torch.zeros(64, dtype=torch.uint8, device=DEV)
    dst = torch.zeros(64, dtype=torch.uint8)  # pageable
    rc = lib.fedavg_copy_to_host(src.data_ptr(), dst.data_ptr(), 64, 8, None)
    assert rc == -10001


@pytest.mark.parametrize("small_bytes", [None, 0])  # one-call finish for small fp32 rounds / chunked path
def test_round_session_streaming_matches_golden(small_bytes):
    small_seen = 0
    for name in ["mnist_lr_k100", "mnist_lr_k10", "resnet_like_bn_k5", "int_dtypes_k3", "float64_key_k3",
                 "bfloat16_key_k3", "flat_k10_p65", "single_client_k1", "ieee_specials_k4", "subnormal_products_k3",
                 "adversarial_k10", "float_counts_k4"]:
        meta, w_locals, expected = load_case(name)
        agg = mfl_amd.DeviceAggregator(DEV)
        if small_bytes is not None:
            agg.SMALL_ROUND_BYTES = small_bytes
        sess = agg.begin_round(w_locals[0][1], len(w_locals) + 3)
        groups = sess.table.groups
        assert sess._small == (small_bytes is None and list(groups) == [torch.float32])
        small_seen += sess._small
        for n, sd in w_locals:
            sess.add(n, sd)
        out = sess.finish(w_locals)
        assert out is w_locals[0][1]
        for k, exp in expected.items():
            assert_bits(out[k], exp, f"{name}/{k}")
    assert small_seen >= (4 if small_bytes is None else 0)


@pytest.mark.parametrize("small_bytes", [None, 0])
def test_round_session_finish_under_side_stream(small_bytes):
    """begin_round on the default stream, finish() under another one: the
    weights must be uploaded on the stream the reduce runs on (a previous
    round's weights, or the warm-up's 1/K, would otherwise be read).  Several
    rounds with different sample counts on one aggregator, the weight copy
    held back by a busy side stream."""
    _, w_locals, expected = load_case("mnist_lr_k10")
    for big in (False, True):
        agg = mfl_amd.DeviceAggregator(DEV)
        if small_bytes is not None:
            agg.SMALL_ROUND_BYTES = small_bytes
        if big:  # a multi-chunk row (reduce_and_fetch path): one 4.2M-column key
            g = torch.Generator().manual_seed(5)
            base = torch.randn(4_194_304 + 5, generator=g) * 0.05
            rounds = []
            for r in range(3):
                counts = [int(c) for c in torch.randint(1, 1000, (4,), generator=g)]
                dl = [(n, {"w": base + 1e-3 * torch.randn(base.numel(), generator=g)}) for n in counts]
                exp = torch.from_numpy(O.reduce_f32(np.stack([d["w"].numpy() for _, d in dl]),
                                                    O.sample_weights(counts)))
                rounds.append((dl, {"w": exp}))
        else:
            rounds = []
            for r in range(3):  # same rows, permuted sample counts: different weights per round
                perm = np.random.default_rng(r).permutation(len(w_locals))
                dl = [(w_locals[int(p)][0], {k: v.clone() for k, v in w_locals[i][1].items()})
                      for i, p in enumerate(perm)]
                counts = [n for n, _ in dl]
                flat_keys = list(expected)
                rows = np.stack([np.concatenate([d[k].reshape(-1).numpy().astype(np.float32) for k in flat_keys])
                                 for _, d in dl])
                ref = O.reduce_f32(rows, O.sample_weights(counts))
                exp, off = {}, 0
                for k in flat_keys:
                    n = expected[k].numel()
                    exp[k] = torch.from_numpy(ref[off:off + n].copy()).reshape(expected[k].shape)
                    off += n
                rounds.append((dl, exp))
        side = torch.cuda.Stream(DEV)
        for dl, exp in rounds:
            sess = agg.begin_round(dl[0][1], len(dl))
            for n, sd in dl:
                sess.add(n, sd)
            with torch.cuda.stream(side):
                torch.cuda._sleep(2_000_000)  # the side stream is busy when finish() enqueues on it
                out = sess.finish(dl)
            torch.cuda.synchronize(DEV)
            for k, e in exp.items():
                assert_bits(out[k], e, f"side-stream finish {k}")


def test_round_session_checks_w_locals():
    _, w_locals, _ = load_case("mnist_lr_k10")
    agg = mfl_amd.DeviceAggregator(DEV)
    sess = agg.begin_round(w_locals[0][1], 10)
    for n, sd in w_locals[:5]:
        sess.add(n, sd)
    with pytest.raises(ValueError):
        sess.finish(w_locals)


# ---------------------------------------------------------------------------
# post-aggregate client distances (fedavg_trainer.py:291) and delta (:293)
# ---------------------------------------------------------------------------
def _fp32_ulp(x):
    return np.spacing(np.float32(abs(x))).astype(np.float64)


@pytest.mark.parametrize("name", ["mnist_lr_k10", "mnist_lr_k100", "resnet_like_bn_k5", "adversarial_k10",
                                  "flat_k10_p65", "thirds_k3", "single_client_k1"])
def test_client_distances_after_aggregate(name):
    import copy
    _, w_locals, _ = load_case(name)
    ref_locals = copy.deepcopy(w_locals)
    ref_glob = O.aggregate_torch(ref_locals)  # reference order: :217 aggregate ...
    agg = mfl_amd.DeviceAggregator(DEV)
    w_glob = agg.aggregate(w_locals)
    norms = agg.client_distances(w_locals, w_glob)  # ... then :291 (cached device rows)
    exact = O.client_distances_exact(ref_locals, ref_glob)
    torch_ref = O.client_distances_torch(ref_locals, ref_glob)
    assert norms[0] == 0.0 and exact[0] == 0.0 and torch_ref[0] == 0.0  # aliasing quirk: w_locals[0][1] is w_glob
    for a, e, t in zip(norms, exact, torch_ref):
        assert abs(a - e) <= _fp32_ulp(e), (name, a, e)
        assert abs(a - t) <= 1e-5 * max(abs(t), 1e-30) + 1e-30, (name, a, t)
    # the uncached path (fresh upload) agrees with the cached one
    again = mfl_amd.DeviceAggregator(DEV).client_distances(w_locals, w_glob)
    assert np.array_equal(again, norms)
    lr = 0.03
    d = mfl_amd.estimate_delta(w_locals, w_glob, lr, device=DEV)
    d_ref = O.delta_from_norms([n for n, _ in ref_locals], torch_ref, lr)
    assert abs(d - d_ref) <= 1e-5 * abs(d_ref) + 1e-30


@pytest.mark.parametrize("name", ["float64_key_k3", "float16_key_k3", "bfloat16_key_k3", "resnet_like_bn_k5"])
def test_client_distances_other_dtypes(name):
    """:291 with fp64 / fp16 / bf16 keys (the reference's torch.cat dtype
    promotion): every group's pass, summed, rooted and rounded to the cat
    dtype, against the oracle's accurate restatement (within one unit of
    that dtype; fp64 within 1e-12) and ATen's own norm (two units)."""
    import copy
    _, w_locals, _ = load_case(name)
    orig = copy.deepcopy(w_locals)  # the aggregates below alias and overwrite client 0's dict (:449)
    ref_locals = copy.deepcopy(w_locals)
    ref_glob = O.aggregate_torch(ref_locals)
    cat = torch.cat([ref_locals[-1][1][k].reshape(-1) - ref_glob[k].reshape(-1) for k in ref_glob]).dtype
    eps = 1e-12 if cat == torch.float64 else torch.finfo(cat).eps
    exact = O.client_distances_exact(ref_locals, ref_glob)
    torch_ref = O.client_distances_torch(ref_locals, ref_glob)
    agg = mfl_amd.DeviceAggregator(DEV)
    w_glob = agg.aggregate(w_locals)
    for norms in (agg.client_distances(w_locals, w_glob),  # cached rows
                  mfl_amd.DeviceAggregator(DEV).client_distances(w_locals, w_glob)):  # fresh upload
        assert norms[0] == 0.0
        assert np.allclose(norms, exact, rtol=eps, atol=0), (name, norms, exact)
        assert np.allclose(norms, torch_ref, rtol=2 * max(eps, 1e-6), atol=0), (name, norms, torch_ref)
    # device-resident clients: the same groups packed in HBM
    dl = [(n, {k: v.to(DEV) for k, v in sd.items()}) for n, sd in orig]
    dev_agg = mfl_amd.DeviceAggregator(DEV)
    dglob = dev_agg.aggregate(dl)
    norms = dev_agg.client_distances(dl, dglob)
    assert np.allclose(norms, exact, rtol=eps, atol=0), (name, norms, exact)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("K,P", [(3, 1), (5, 7), (7, 4099), (100, 1_000_003)])
def test_client_sqdist_other_dtypes_vs_torch(dtype, K, P):
    """The fp64 / fp16 / bf16 pass against torch on the device: differences in
    the rows' dtype (torch's own rounding), squares summed in fp64."""
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(P + K)
    x = (torch.randn((K, ld), generator=g, device=DEV) * 0.05).to(dtype)
    glob = (torch.randn(ld, generator=g, device=DEV) * 0.05).to(dtype)
    x[:, P:] = float("nan")  # padding never contributes
    got = mfl_amd.client_sqdist(x, glob, P)
    ref = torch.stack([((x[k, :P] - glob[:P]).double() ** 2).sum() for k in range(K)])
    rel = ((got - ref).abs() / ref.clamp_min(1e-300)).max().item()
    assert rel < 1e-12, rel
    assert torch.equal(got, mfl_amd.client_sqdist(x, glob, P))  # deterministic


def test_client_sqdist_large_vs_fp64():
    K, P = 100, 25_000_000 + 3
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn((K, ld), generator=g, device=DEV) * 0.05
    glob = torch.randn(ld, generator=g, device=DEV) * 0.05
    got = mfl_amd.client_sqdist(x, glob, P)
    ref = torch.stack([((x[k, :P] - glob[:P]).double() ** 2).sum() for k in range(K)])
    rel = ((got - ref).abs() / ref).max().item()
    assert rel < 1e-12, rel
    again = mfl_amd.client_sqdist(x, glob, P)
    assert torch.equal(got, again)  # deterministic
    del x


@pytest.mark.parametrize("K,P", [(7, 1001), (3, 4096 * 16 + 5), (13, 300_007), (100, 600_372), (2, 3)])
def test_client_sqdist_buffer_descriptor_variants(K, P):
    """fedavg_client_sqdist_buf (hardware range check instead of predicated
    loads; NaN in the row padding past P) matches the fp64 reference for every
    schedule, deterministically."""
    lib = mfl_amd._lib.load_probe()
    ld = (P + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(K + P)
    x = torch.full((K, ld), float("nan"), device=DEV)
    x[:, :P] = torch.randn((K, P), generator=g, device=DEV) * 0.05
    glob = torch.full((ld,), float("nan"), device=DEV)
    glob[:P] = torch.randn(P, generator=g, device=DEV) * 0.05
    ref = torch.stack([((x[k, :P] - glob[:P]).double() ** 2).sum() for k in range(K)])
    n_ws = lib.fedavg_client_sqdist_workspace(K, P)
    work = torch.empty(n_ws, dtype=torch.float64, device=DEV)
    for u, c, mb in [(4, 8, 0), (2, 16, 0), (2, 16, 3), (8, 4, 5), (2, 8, 0), (8, 8, 1)]:
        outs = []
        for _ in range(2):
            o = torch.empty(K, dtype=torch.float64, device=DEV)
            mfl_amd._lib.check(lib.fedavg_client_sqdist_buf(x.data_ptr(), K, P, ld, glob.data_ptr(), work.data_ptr(),
                                                            n_ws, o.data_ptr(), u, c, mb, None), f"U{u}C{c}mb{mb}")
            outs.append(o)
        torch.cuda.synchronize()
        rel = ((outs[0] - ref).abs() / ref).max().item()
        assert rel < 1e-12, (u, c, mb, rel)
        assert torch.equal(outs[0], outs[1]), (u, c, mb)


def test_client_sqdist_padding_nan_ignored():
    K, P = 3, 1001  # P % 4 == 1: the last float4 holds 3 padding lanes
    x = torch.full((K, 1024), float("nan"), device=DEV)
    x[:, :P] = torch.arange(P, device=DEV, dtype=torch.float32) * 1e-3
    glob = torch.full((1024,), float("nan"), device=DEV)
    glob[:P] = 0.0
    got = mfl_amd.client_sqdist(x, glob, P)
    assert torch.isfinite(got).all()
    assert abs(got[0].item() - float(((torch.arange(P, device=DEV, dtype=torch.float32) * 1e-3).double() ** 2).sum())) < 1e-9


def test_client_distances_bool_buffer_raises():
    _, w_locals, _ = load_case("int_dtypes_k3")
    w_glob = mfl_amd.aggregate(w_locals)
    with pytest.raises(RuntimeError):
        mfl_amd.client_distances(w_locals, w_glob)


def test_client_distances_after_streaming_round():
    import copy
    _, w_locals, _ = load_case("mnist_lr_k100")
    ref_locals = copy.deepcopy(w_locals)
    ref_glob = O.aggregate_torch(ref_locals)
    agg = mfl_amd.DeviceAggregator(DEV)
    sess = agg.begin_round(w_locals[0][1], len(w_locals))
    for n, sd in w_locals:
        sess.add(n, sd)
    w_glob = sess.finish(w_locals)
    norms = agg.client_distances(w_locals, w_glob)
    exact = O.client_distances_exact(ref_locals, ref_glob)
    assert norms[0] == 0.0
    assert np.all(np.abs(norms - exact) <= np.spacing(exact.astype(np.float32)).astype(np.float64))


def test_plain_c_consumer_runs():
    import subprocess
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    subprocess.run(["make", "-s", "-C", str(root / "examples"), "c_abi_demo"], check=True, timeout=120)
    proc = subprocess.run([str(root / "examples" / "c_abi_demo"), "37", "1000003"], capture_output=True,
                          text=True, timeout=120)
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert "C ABI demo OK" in proc.stdout


def test_int64_indexing_beyond_2_31_elements():
    """A row longer than 2^31 elements (8.6 GB): every offset in the kernels is
    64-bit.  Sampled windows at the start, around 2^31 and at the ragged end."""
    K = 2
    P = (1 << 31) + 4099
    ld = (P + 63) // 64 * 64
    x = torch.empty((K, ld), device=DEV)
    for k in range(K):
        g = torch.Generator(device=DEV).manual_seed(70 + k)
        x[k].normal_(0.0, 0.05, generator=g)
    w = _weights(K)
    out = mfl_amd.reduce_packed(x, _w(w), P)
    for s in (0, (1 << 31) - 2048, (1 << 31) - 3, P - 4099):
        e = min(s + 4099, P)
        exp = O.reduce_f32(x[:, s:e].cpu().numpy(), w)
        assert_bits(out[s:e], torch.from_numpy(exp), f"window {s}")
    sq = mfl_amd.client_sqdist(x, out, P)
    ref = torch.stack([((x[k, :P] - out[:P]).double() ** 2).sum() for k in range(K)])
    assert ((sq - ref).abs() / ref).max().item() < 1e-12
    del x, out


@pytest.mark.parametrize("dtype,K,P", [(torch.float64, 8, 10_000_003), (torch.float16, 6, 40_000_005),
                                       (torch.bfloat16, 5, 40_000_001), (torch.float64, 600, 200_001),
                                       (torch.bfloat16, 3, 1_000_003),
                                       # fp64 on both sides of its switch to the buffer-descriptor kernel
                                       (torch.float64, 5, 4_194_301), (torch.float64, 5, 4_194_307)])
def test_reduce_vec_dtypes_multilaunch(dtype, K, P):
    """fp64/fp16/bf16 production schedule (round-split, multi-slice, nt) is
    bit-exact on sampled windows incl. launch boundaries and the ragged tail."""
    from mfl_amd import _lib
    x = _clients(K, P, seed=P % 1000 + K, dtype=dtype)
    w = _weights(K, seed=K)
    out = mfl_amd.reduce_packed(x, _w(w, torch.float64 if dtype == torch.float64 else torch.float32), P)
    lanes = 16 // x.element_size()
    f32_equiv = P * (16 // lanes) // 4
    launches = _lib.f32_schedule(K, f32_equiv)["launches"]
    starts = [0, P // 2, P - 4099] + [int(P * i / max(launches, 1)) - 2048 for i in range(1, launches)]
    for s in starts:
        s = max(0, min(s, P - 4099))
        xs = x[:, s:s + 4099].cpu()
        if dtype == torch.float64:
            exp = torch.from_numpy(O.reduce_f64(xs.numpy(), w))
        elif dtype == torch.float16:
            exp = torch.from_numpy(O.reduce_half(xs.numpy(), w, "float16"))
        else:
            bits = O.reduce_half(xs.view(torch.int16).numpy(), w, "bfloat16")
            exp = torch.from_numpy(bits.view(np.int16).copy()).view(torch.bfloat16)
        assert_bits(out[s:s + 4099], exp, f"{dtype} window {s}")
    del x


@pytest.mark.parametrize("dtype,K,P", [(torch.bfloat16, 7, 300_011), (torch.float16, 13, 4096 * 8 * 3 + 5),
                                       (torch.float64, 5, 100_003), (torch.bfloat16, 1, 77)])
def test_vec_buffer_descriptor_bit_identical(dtype, K, P):
    """fedavg_reduce_vec_buf gives the production fp16/bf16/fp64 kernel's bits
    for every schedule, ragged last group and P tail included."""
    lib = mfl_amd._lib.load_probe()
    x = _clients(K, P, seed=K + P, dtype=dtype)
    wdt = torch.float64 if dtype == torch.float64 else torch.float32
    w = _w(_weights(K), wdt)
    base = mfl_amd.reduce_packed(x, w, P)
    iv = torch.int64 if dtype == torch.float64 else torch.int16
    code = {torch.float16: 0, torch.bfloat16: 1, torch.float64: 2}[dtype]
    for u, c, b in [(8, 4, 0), (4, 8, 3), (2, 16, 0), (4, 4, 1), (2, 8, 0)]:
        out = torch.empty(P, dtype=dtype, device=DEV)
        mfl_amd._lib.check(lib.fedavg_reduce_vec_buf(code, x.data_ptr(), K, P, x.shape[1], w.data_ptr(),
                                                     out.data_ptr(), u, c, b, None), f"U{u}C{c}b{b}")
        torch.cuda.synchronize()
        assert torch.equal(out.view(iv), base.view(iv)), (dtype, K, P, u, c, b)


def test_open_session_blocks_aggregate():
    _, w_locals, _ = load_case("mnist_lr_k10")
    agg = mfl_amd.DeviceAggregator(DEV)
    sess = agg.begin_round(w_locals[0][1], 10)
    sess.add(*w_locals[0])
    with pytest.raises(RuntimeError):
        agg.aggregate(w_locals)
    with pytest.raises(RuntimeError):
        agg.begin_round(w_locals[0][1], 10)
    for n, sd in w_locals[1:]:
        sess.add(n, sd)
    sess.finish(w_locals)
    agg.begin_round(w_locals[0][1], 10)  # allowed again


# ---------------------------------------------------------------------------
# small rounds: the one-call native host side (fedavg_collect_ext.small_round)
# ---------------------------------------------------------------------------
def test_small_round_native_path_rounds_bit_exact_and_fall_back():
    """After one small fp32 round, the next rounds with the same key table run
    their whole host side in one native call.  Every round is bit-exact vs the
    reference's loop and returns w_locals[0][1]; the :291 cache stays valid;
    and every input the native walk refuses falls back to the general path,
    which raises the reference's exception (nothing written before)."""
    import copy
    for name in ["mnist_lr_k10", "mnist_lr_k100", "resnet_like_bn_k5", "flat_k10_p65"]:
        meta, w_locals, expected = load_case(name)
        agg = mfl_amd.DeviceAggregator(DEV)
        for r in range(4):
            wl = copy.deepcopy(w_locals)
            out = agg.aggregate(wl)
            assert out is wl[0][1]
            for k, exp in expected.items():
                assert_bits(out[k], exp, f"{name}/{k} round {r}")
            assert list(out.keys()) == list(expected.keys())
            if not any(t.dtype == torch.bool for _, sd in wl for t in sd.values()):
                norms = agg.client_distances(wl, out)  # rows the native round left in HBM
                assert norms[0] == 0.0 and np.all(np.isfinite(norms))
        assert agg.fast_rounds == 3, name
    # fallbacks: the general path sees (and raises for) what the walk refused
    meta, w_locals, expected = load_case("mnist_lr_k10")
    agg = mfl_amd.DeviceAggregator(DEV)
    agg.aggregate(copy.deepcopy(w_locals))
    wl = copy.deepcopy(w_locals)
    wl = [(0, sd) for _, sd in wl]
    with pytest.raises(ZeroDivisionError):
        agg.aggregate(wl)
    wl = copy.deepcopy(w_locals)
    del wl[3][1][next(iter(wl[3][1]))]
    with pytest.raises(KeyError):
        agg.aggregate(wl)
    wl = copy.deepcopy(w_locals)
    wl = [(float(n), sd) for n, sd in wl]  # float counts: the general path (Python true division)
    ref = O.aggregate_torch(copy.deepcopy(wl))
    out = agg.aggregate(wl)
    for k in ref:
        assert_bits(out[k], ref[k], f"float counts {k}")
    before = agg.fast_rounds
    wl = copy.deepcopy(w_locals)
    out = agg.aggregate(wl)  # back on the native path after the general one
    for k, exp in expected.items():
        assert_bits(out[k], exp, f"after fallback {k}")
    assert agg.fast_rounds == before + 1


@pytest.mark.parametrize("K,P", [(10, 1_206_590), (100, 781_312), (3, 4099), (100, 25_000_000)])
def test_timed_reduce_same_bits_and_kernel_time(K, P):
    """fedavg_reduce_f32_timed (launch-attached events, bench.py's timing
    hook) gives fedavg_reduce_f32's bits, and its event pair brackets the
    reduce's launches (a positive time, below the host-side wall time)."""
    import time
    x = _clients(K, P, seed=P + 1)
    w = _w(_weights(K))
    base = mfl_amd.reduce_packed(x, w, P)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()
    torch.cuda.synchronize()
    out = torch.full((P,), float("nan"), device=DEV)
    t0 = time.perf_counter()
    mfl_amd.reduce_packed(x, w, P, out, events=(e0, e1))
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3
    assert torch.equal(out.view(torch.int32), base.view(torch.int32))
    ms = e0.elapsed_time(e1)
    assert 0.0 < ms <= wall_ms
    fresh = torch.cuda.Event(enable_timing=True)
    with pytest.raises(ValueError):  # never recorded: no HIP event behind it yet
        mfl_amd.reduce_packed(x, w, P, out, events=(fresh, e1))
