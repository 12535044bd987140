"""Host-side logic of the drop-in (no GPU): the reference's early returns and
errors, key tables, packing/unpacking and dtype promotion rules."""
import copy
from collections import OrderedDict

import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd
from mfl_amd.aggregate import _Prepared, prepare
from mfl_amd.layout import KeyTable, result_dtype
from golden_io import bits_equal, case_names, load_case


def test_empty_w_locals_returns_global_copy():
    torch.manual_seed(0)
    glob = torch.nn.Linear(5, 3)
    _, _, expected = load_case("empty_w_locals")
    out = mfl_amd.aggregate([], model_global=glob)
    assert list(out.keys()) == list(expected.keys())
    for k in expected:
        assert bits_equal(out[k], expected[k])
    # a copy, not the live parameters
    out["weight"].add_(1.0)
    assert not torch.equal(out["weight"], glob.weight.detach())


def test_mixin_empty_path_uses_model_global():
    class Trainer(mfl_amd.FedAvgAggregateMixin):
        def __init__(self):
            torch.manual_seed(0)
            self.model_global = torch.nn.Linear(5, 3)

    out = Trainer().aggregate([])
    _, _, expected = load_case("empty_w_locals")
    assert all(bits_equal(out[k], expected[k]) for k in expected)


def test_install_patches_class():
    class RefLike:
        def aggregate(self, w_locals):
            raise AssertionError("reference path must not run")

    mfl_amd.install(RefLike)
    t = RefLike()
    t.model_global = torch.nn.Linear(2, 2)
    out = t.aggregate([])
    assert set(out.keys()) == {"weight", "bias"}
    assert RefLike.aggregate.__wrapped_reference__ is not None


def test_no_keys_returns_first_dict():
    meta, w_locals, expected = load_case("no_keys_k2")
    first = w_locals[0][1]
    out = mfl_amd.aggregate(w_locals)
    assert out is first and len(out) == 0


def test_zero_total_raises_zero_division():
    sd = OrderedDict(w=torch.ones(3))
    with pytest.raises(ZeroDivisionError):
        prepare([(0, sd), (0, copy.deepcopy(sd))])


def test_missing_key_raises_key_error():
    a = OrderedDict(w=torch.ones(3), b=torch.ones(2))
    b = OrderedDict(w=torch.ones(3))
    with pytest.raises(KeyError):
        prepare([(1, a), (1, b)])


def test_extra_keys_in_later_clients_ignored():
    a = OrderedDict(w=torch.ones(3))
    b = OrderedDict(w=torch.ones(3), extra=torch.ones(7))
    prep = prepare([(1, a), (2, b)])
    assert isinstance(prep, _Prepared)
    assert [e.name for e in prep[1].entries] == ["w"]


def test_shape_mismatch_raises():
    a = OrderedDict(w=torch.ones(3))
    b = OrderedDict(w=torch.ones(1))  # the reference would silently broadcast
    with pytest.raises(mfl_amd.ShapeMismatchError):
        prepare([(1, a), (1, b)])
    with pytest.raises(RuntimeError):  # same exception family as the reference's broadcast error
        prepare([(1, OrderedDict(w=torch.ones(2, 3))), (1, OrderedDict(w=torch.ones(3, 2)))])


def test_dtype_mismatch_raises():
    with pytest.raises(TypeError):
        prepare([(1, OrderedDict(w=torch.ones(3))), (1, OrderedDict(w=torch.ones(3, dtype=torch.float64)))])


def test_same_dict_twice_refused():
    sd = OrderedDict(w=torch.ones(3))
    with pytest.raises(ValueError):
        prepare([(1, sd), (1, sd)])


@pytest.mark.parametrize("src,res", [
    (torch.float32, torch.float32), (torch.float64, torch.float64), (torch.float16, torch.float16),
    (torch.bfloat16, torch.bfloat16), (torch.int64, torch.float32), (torch.int32, torch.float32),
    (torch.uint8, torch.float32), (torch.bool, torch.float32),
])
def test_result_dtype_matches_aten_promotion(src, res):
    assert result_dtype(src) == res
    assert (torch.ones(2, dtype=src) * 0.5).dtype == res


def test_key_table_groups_and_alignment():
    _, w_locals, _ = load_case("resnet_like_bn_k5")
    table = KeyTable(w_locals[0][1])
    assert list(table.groups) == [torch.float32]  # int64 buffers join the fp32 group
    g = table.groups[torch.float32]
    assert g.P == sum(t.numel() for t in w_locals[0][1].values())
    assert g.ld % mfl_amd.ALIGN_ELEMS == 0 and g.ld >= g.P
    offs = [e.offset for e in g.keys]
    assert offs == sorted(offs) and offs[0] == 0


@pytest.mark.parametrize("name", ["resnet_like_bn_k5", "int_dtypes_k3", "float64_key_k3", "mnist_lr_k10",
                                  "bfloat16_key_k3", "scalar_key_k3"])
def test_pack_then_cpu_oracle_reproduces_reference(name):
    """Packing is lossless w.r.t. the reference's promotion: the oracle run on
    the packed rows reproduces the golden output bit for bit."""
    meta, w_locals, expected = load_case(name)
    table = KeyTable(w_locals[0][1])
    dicts = [sd for _, sd in w_locals]
    table.validate(dicts)
    weights = O.sample_weights([n for n, _ in w_locals])
    for g in table.groups.values():
        buf = torch.zeros((len(dicts), g.ld), dtype=g.dtype)
        table.pack_into(g, buf, dicts)
        if g.dtype == torch.float32:
            flat = torch.from_numpy(O.reduce_f32(buf[:, :g.P].numpy(), weights))
        elif g.dtype == torch.float64:
            flat = torch.from_numpy(O.reduce_f64(buf[:, :g.P].numpy(), weights))
        elif g.dtype == torch.bfloat16:
            bits = O.reduce_half(buf[:, :g.P].view(torch.int16).numpy(), weights, "bfloat16")
            flat = torch.from_numpy(bits.view(np.int16).copy()).view(torch.bfloat16)
        else:
            flat = torch.from_numpy(O.reduce_half(buf[:, :g.P].numpy(), weights, "float16"))
        for k, t in table.unpack(g, flat).items():
            assert bits_equal(t, expected[k]), k


def test_int64_to_fp32_rounding_matches_reference_cast():
    _, w_locals, expected = load_case("int_dtypes_k3")
    big = w_locals[0][1]["big"]
    assert (big > 2**24).all()  # values that do not fit fp32 exactly
    buf = torch.zeros((1, 64))
    table = KeyTable(OrderedDict(big=big))
    table.pack_into(table.groups[torch.float32], buf, [OrderedDict(big=big)])
    assert torch.equal(buf[0, :40], big.to(torch.float32))


def test_launch_patches_reference_module_before_script_runs(tmp_path):
    """mfl_amd.launch: the script's own `from fedavg_trainer import FedAvgTrainer`
    (main_fedavg.py:16) must bind the patched class."""
    import subprocess
    import sys
    from pathlib import Path

    (tmp_path / "fedavg_trainer.py").write_text(
        "class FedAvgTrainer:\n"
        "    def aggregate(self, w_locals):\n"
        "        return 'reference'\n")
    (tmp_path / "main_fedavg.py").write_text(
        "import sys, torch\n"
        "from fedavg_trainer import FedAvgTrainer\n"
        "t = FedAvgTrainer(); t.model_global = torch.nn.Linear(2, 2)\n"
        "out = t.aggregate([])\n"
        "print('PATCHED' if isinstance(out, dict) and set(out) == {'weight', 'bias'} else 'NOT', sys.argv[1:])\n")
    repo = Path(__file__).resolve().parents[1]
    env = dict(__import__("os").environ, PYTHONPATH=str(repo))
    proc = subprocess.run([sys.executable, "-m", "mfl_amd.launch", str(tmp_path / "main_fedavg.py"), "--gpu", "0"],
                          cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert proc.returncode == 0, proc.stderr
    assert "PATCHED ['--gpu', '0']" in proc.stdout


def _python_collect(table, dicts, monkeypatch):
    from mfl_amd import layout
    monkeypatch.setattr(layout, "_COLLECT", [None])
    try:
        return table.collect(dicts)
    finally:
        monkeypatch.setattr(layout, "_COLLECT", [])


def test_native_collect_matches_python_walk(monkeypatch):
    from mfl_amd.layout import _collect_ext
    if _collect_ext() is None:
        pytest.skip("collect extension not built")
    for name in ["resnet_like_bn_k5", "int_dtypes_k3", "mnist_lr_k100", "float64_key_k3", "bfloat16_key_k3"]:
        _, w_locals, _ = load_case(name)
        dicts = [sd for _, sd in w_locals]
        table = KeyTable(dicts[0])
        native, keep = table.collect(dicts)
        assert keep == []
        py, _ = _python_collect(table, dicts, monkeypatch)
        assert (native == py).all(), name


@pytest.mark.parametrize("case", ["missing", "shape", "dtype", "noncontig", "notensor"])
def test_native_collect_falls_back_for_unusual_clients(case):
    a = OrderedDict(w=torch.arange(6, dtype=torch.float32).reshape(2, 3), b=torch.ones(2))
    if case == "missing":
        b = OrderedDict(w=torch.ones(2, 3))
        err = KeyError
    elif case == "shape":
        b = OrderedDict(w=torch.ones(3, 2), b=torch.ones(2))
        err = mfl_amd.ShapeMismatchError
    elif case == "dtype":
        b = OrderedDict(w=torch.ones(2, 3, dtype=torch.float64), b=torch.ones(2))
        err = TypeError
    elif case == "notensor":
        b = OrderedDict(w=[[1.0] * 3] * 2, b=torch.ones(2))
        err = AttributeError
    else:
        b = OrderedDict(w=torch.ones(3, 2).t(), b=torch.ones(2))  # non-contiguous: handled, not an error
        err = None
    table = KeyTable(a)
    if err is None:
        ptrs, keep = table.collect([a, b])
        assert len(keep) == 1 and ptrs[1, 0] == keep[0][0].data_ptr()
        assert torch.equal(keep[0][0], b["w"])
    else:
        with pytest.raises(err):
            table.collect([a, b])


def test_prepare_reuses_table_hint_only_when_client0_matches():
    """DeviceAggregator reuses the previous round's KeyTable (prepare's
    table_hint) only when client 0 has exactly its keys, in order, with the
    same shapes and dtypes; otherwise it builds a fresh table, and a bad later
    client still raises the reference's exception."""
    from mfl_amd.layout import _collect_ext
    a = OrderedDict(w=torch.ones(2, 3), b=torch.zeros(2))
    b = OrderedDict(w=torch.ones(2, 3) * 2, b=torch.ones(2))
    table = prepare([(1, a), (2, b)])[1]
    p = prepare([(1, OrderedDict(a)), (2, b)], table_hint=table)
    assert (p[1] is table) == (_collect_ext() is not None)
    assert (p[4] == prepare([(1, OrderedDict(a)), (2, b)])[4]).all()
    cases = [
        OrderedDict(w=torch.ones(3, 3), b=torch.zeros(2)),                      # other shape
        OrderedDict(w=torch.ones(2, 3), b=torch.zeros(2), c=torch.ones(1)),     # extra key in client 0
        OrderedDict(b=torch.zeros(2), w=torch.ones(2, 3)),                      # other key order
        OrderedDict(w=torch.ones(2, 3, dtype=torch.float64), b=torch.zeros(2)),  # other dtype
    ]
    for c in cases:
        other = OrderedDict((k, v.clone()) for k, v in c.items())
        p = prepare([(1, c), (2, other)], table_hint=table)
        assert p[1] is not table
        assert [e.name for e in p[1].entries] == list(c.keys())
        assert [e.shape for e in p[1].entries] == [tuple(v.shape) for v in c.values()]
    with pytest.raises(KeyError):
        prepare([(1, OrderedDict(a)), (2, OrderedDict(w=torch.ones(2, 3)))], table_hint=table)
    with pytest.raises(mfl_amd.ShapeMismatchError):
        prepare([(1, OrderedDict(a)), (2, OrderedDict(w=torch.ones(3, 2), b=torch.ones(2)))], table_hint=table)


def test_functional_aggregate_trivial_cases_need_no_gpu():
    class M:
        def cpu(self):
            return self

        def state_dict(self):
            return OrderedDict(w=torch.arange(3.0))

    out = mfl_amd.aggregate([], model_global=M())
    assert torch.equal(out["w"], torch.arange(3.0))
    empty = OrderedDict()
    assert mfl_amd.aggregate([(1, empty), (2, OrderedDict())]) is empty


def test_fpf_tracker_without_gpu_fails_loudly():
    import mfl_amd

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(mfl_amd.FedAvgLibraryError):
        mfl_amd.FPFTracker(4, {"w": torch.zeros(3)}, 2)


def test_client_device_and_mixed_device_rejection():
    """Where the clients live is read from client 0's first key; collect then
    requires every tensor of every client there (host clients, or all on one
    HIP device -- checked here with meta tensors standing in for a device)."""
    _, w_locals, _ = load_case("mnist_lr_k10")
    dicts = [sd for _, sd in w_locals]
    table = KeyTable(dicts[0])
    assert table.client_device(dicts) == torch.device("cpu")
    ptrs, _ = table.collect(dicts)
    assert ptrs.shape == (10, 2)
    mixed = [OrderedDict(sd) for sd in dicts]
    mixed[4]["linear.bias"] = mixed[4]["linear.bias"].to("meta")
    with pytest.raises(TypeError, match="client 4"):
        table.collect(mixed)
    with pytest.raises(TypeError):
        prepare([(n, sd) for (n, _), sd in zip(w_locals, mixed)])
    meta0 = [OrderedDict((k, v.to("meta")) for k, v in dicts[0].items())] + dicts[1:]
    with pytest.raises(TypeError, match="not supported"):
        KeyTable(meta0[0]).client_device(meta0)
    # a retained table never accepts clients on another device than it was asked for
    assert table.try_collect(mixed) is None


def test_try_collect_needs_client0_exactly_the_table():
    """A table kept from an earlier round is reused only when client 0 is a
    dict holding exactly its keys in order (the native walk's strict0 check);
    other clients may hold their keys in any order or extra keys, as the
    reference only reads client 0's keys from them (fedavg_trainer.py:450-457)."""
    _, w_locals, _ = load_case("resnet_like_bn_k5")
    dicts = [OrderedDict(sd) for _, sd in w_locals]
    table = KeyTable(dicts[0])
    got = table.try_collect(dicts)
    assert got is not None and np.array_equal(got[0], table.collect(dicts)[0])
    names = list(dicts[0])
    reordered = OrderedDict((k, dicts[0][k]) for k in reversed(names))
    assert table.try_collect([reordered] + dicts[1:]) is None
    extra = OrderedDict(dicts[0])
    extra["extra.key"] = torch.zeros(3)
    assert table.try_collect([extra] + dicts[1:]) is None
    missing = OrderedDict((k, v) for k, v in dicts[0].items() if k != names[-1])
    assert table.try_collect([missing] + dicts[1:]) is None
    assert table.try_collect([dict(dicts[0])] + dicts[1:]) is not None  # a plain dict in the same order
    later = [dicts[0]] + [OrderedDict((k, sd[k]) for k in reversed(names)) for sd in dicts[1:]]
    got = table.try_collect(later)
    assert got is not None and np.array_equal(got[0], table.collect(dicts)[0])
    assert table.try_collect([{names[1]: dicts[0][names[1]]}]) is None  # first key missing: no KeyError


def test_synthetic_inputs_torch_and_numpy_bit_identical():
    """bench.py's device-generated clients (mfl_amd.synthetic) are reproduced
    bit for bit by the numpy form the parity checks regenerate them with."""
    from mfl_amd import synthetic

    for g0, n, K in [(0, 1000, 3), (123_456_789, 4_099, 5), (2**40 + 7, 65, 2)]:
        g = torch.arange(g0, g0 + n, dtype=torch.int64)
        dev = torch.stack([synthetic.client_columns_torch(k, g) for k in range(K)]).numpy()
        host = synthetic.client_columns_numpy(K, g0, n)
        assert dev.tobytes() == host.tobytes()
    x = synthetic.client_columns_numpy(2, 0, 200_000)
    assert abs(float(x[0].std()) - 0.05) < 1e-3 and abs(float(x[0].mean())) < 1e-3
    assert abs(float((x[1] - x[0]).std()) - 1e-3 * 2 ** 0.5) < 1e-4
    rows = torch.empty(3, 300)
    synthetic.fill_rows(rows, [(0, 7, 100), (128, 1000, 150)])
    assert rows[:, 0:100].numpy().tobytes() == synthetic.client_columns_numpy(3, 7, 100).tobytes()
    assert rows[:, 128:278].numpy().tobytes() == synthetic.client_columns_numpy(3, 1000, 150).tobytes()
    assert float(rows[:, 100:128].abs().sum()) == 0.0 and float(rows[:, 278:].abs().sum()) == 0.0


def test_client_arena_layout_is_detected_on_host_pointers():
    """DeviceAggregator._arena_rows (host-side pointer arithmetic, no GPU):
    client_arena dicts are recognised as the packed [K, ld] layout and viewed
    as [K, P] with stride ld; reordered keys or a gap between clients are not."""
    from collections import OrderedDict

    from mfl_amd.aggregate import DeviceAggregator

    for name in ["mnist_lr_k10", "flat_k10_p65", "flat_k1_p1"]:
        _, wl, _ = load_case(name)
        rows, adicts = mfl_amd.client_arena(wl[0][1], len(wl), "cpu")
        t = KeyTable(adicts[0])
        ptrs, _ = t.collect(adicts)
        g = t.groups[torch.float32]
        v = DeviceAggregator._arena_rows(g, ptrs, adicts)
        assert v is not None and v.shape == (len(wl), g.P) and (len(wl) == 1 or v.stride(0) == g.ld)
        assert v.data_ptr() == rows.data_ptr()
        if len(adicts[0]) > 1:
            rev = [OrderedDict(reversed(list(a.items()))) for a in adicts]
            t2 = KeyTable(rev[0])
            p2, _ = t2.collect(rev)
            assert DeviceAggregator._arena_rows(t2.groups[torch.float32], p2, rev) is None
        if len(adicts) > 2:  # every other client: a non-uniform pitch
            sub = adicts[:1] + adicts[2:]
            p3, _ = t.collect(sub)
            assert DeviceAggregator._arena_rows(g, p3, sub) is None


def test_fused_distance_eligibility(monkeypatch):
    """Which row reductions also form the :291 sums (fedavg_reduce_sqdist_f32):
    16-B aligned fp32 rows of 1..1024 clients, with FEDAVG_FUSE_DISTANCES on
    (the default)."""
    import sys

    A = sys.modules[mfl_amd.DeviceAggregator.__module__]
    assert A.FUSE_DISTANCES and A.FUSED_MAX_K == 1024 and A.FUSED_SEGMENTS_MAX_K == 1024
    assert A.fuse_eligible(torch.empty((1, 64)))
    assert A.fuse_eligible(torch.empty((1024, 64)))
    assert not A.fuse_eligible(torch.empty((1025, 64)))
    rows = torch.empty((10, 72))
    assert A.fuse_eligible(rows[:, :64]) and not A.fuse_eligible(rows[:, 1:65])  # unaligned start
    assert not A.fuse_eligible(torch.empty((10, 66))[:, :64])  # row stride 66 floats
    assert not A.fuse_eligible(torch.empty((0, 64)))
    for dt in (torch.float64, torch.float16, torch.bfloat16):
        assert not A.fuse_eligible(torch.empty((10, 64), dtype=dt))
    monkeypatch.setattr(A, "FUSE_DISTANCES", False)
    assert not A.fuse_eligible(torch.empty((10, 64)))
