"""The drop-in over several GPUs from one process (multi.ShardedAggregator,
SURVEY.md 8e's host-consumer form): each device takes a column shard of the
packed host rows over its own link, reduces it and copies it to its global
positions -- no collective, the same bits as one GPU.  Rehearsed here with N
shards mapped to cuda:0 (every shard has its own buffers and streams, so the
split, the strided uploads and the scatter of the results are what runs on
the driver's 8-GPU node)."""
import copy
import sys
from collections import OrderedDict
from pathlib import Path

import numpy as np
import pytest
import torch

import fedavg_oracle as O
import mfl_amd
from golden_io import GOLDEN_DIR, load_case
from test_gpu_parity import DEV, assert_bits

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "scripts"))
from model_shapes import CONFIGS  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield


def _sharded(n):
    agg = mfl_amd.ShardedAggregator([DEV.index or 0] * n)
    agg.SMALL_ROUND_BYTES = 0  # shard even the golden cases (the product keeps rounds <= 4 MB on one device)
    return agg


CASES = sorted(p.stem for p in GOLDEN_DIR.glob("*.npz") if p.stem != "empty_w_locals")


@pytest.mark.parametrize("n", [2, 8])
def test_golden_cases_bit_exact_over_shards(n):
    agg = _sharded(n)
    for name in CASES:
        _, w_locals, expected = load_case(name)
        if not w_locals or not len(w_locals[0][1]):
            continue
        wl = copy.deepcopy(w_locals)
        out = agg.aggregate(wl)
        assert out is wl[0][1]  # fedavg_trainer.py:449: the result IS client 0's dict
        assert list(out.keys()) == list(expected.keys())
        for k, e in expected.items():
            assert_bits(out[k], e, f"{name} n={n} {k}")
    assert agg.rounds_sharded > 0


def _resnet56_host(seed=3):
    K, shapes = CONFIGS["resnet56"]
    g = torch.Generator(device=DEV).manual_seed(seed)
    base = {k: torch.randn(s, generator=g, device=DEV) * 0.05 for k, s in shapes}
    out = []
    for i in range(K):
        sd = OrderedDict()
        for k, s in shapes:
            if k.endswith("num_batches_tracked"):
                sd[k] = torch.tensor(1000 + 3 * i, dtype=torch.int64)
            else:
                sd[k] = (base[k] + torch.randn(s, generator=g, device=DEV) * 1e-3).cpu()
        out.append(sd)
    counts = [int(c) for c in np.random.default_rng(seed).integers(1, 1000, size=K)]
    return list(zip(counts, out))


@pytest.mark.parametrize("n", [2, 8])
def test_resnet56_x100_over_shards_bit_exact_and_distances(n):
    w_locals = _resnet56_host()
    exp = O.aggregate_torch(copy.deepcopy(w_locals))
    agg = _sharded(n)
    agg.SMALL_ROUND_BYTES = None  # the product rule: 240 MB of rows is sharded
    wl = [(c, OrderedDict(sd)) for c, sd in w_locals]
    out = agg.aggregate(wl)
    assert agg.rounds_sharded == 1 and agg.last_profile["shards"] == n
    for k, e in exp.items():
        assert_bits(out[k], e, f"resnet56 n={n} {k}")
    # :291 after the sharded round: the devices' fp64 sums added in device order
    got = np.asarray(agg.client_distances(wl, out), dtype=np.float64)
    idx = [0, 1, 50, 99]
    ref = O.client_distances_exact([wl[i] for i in idx], out)
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    assert got[0] == 0.0
    assert np.all(np.abs(got[idx] - ref) <= ulp)


def test_functional_routing_and_install(monkeypatch):
    """FEDAVG_DEVICES routes the functional drop-in; install(devices=...)
    routes the patched loop's plain path (streaming off here)."""
    from loop_replay import fresh_classes

    w_locals = _resnet56_host(seed=5)
    exp = O.aggregate_torch(copy.deepcopy(w_locals))
    monkeypatch.setenv("FEDAVG_DEVICES", ",".join([str(DEV.index or 0)] * 4))
    out = mfl_amd.aggregate([(c, OrderedDict(sd)) for c, sd in w_locals])
    for k, e in exp.items():
        assert_bits(out[k], e, k)
    assert mfl_amd.sharded_aggregator([DEV.index or 0] * 4).rounds_sharded >= 1
    monkeypatch.delenv("FEDAVG_DEVICES")
    T, C = fresh_classes()
    mfl_amd.install(T, client_cls=C, stream_clients=False, devices=[DEV.index or 0] * 3)
    rounds = [[(n, [sd]) for n, sd in w_locals]]
    tr = T(OrderedDict((k, torch.zeros_like(v)) for k, v in w_locals[0][1].items()), rounds)
    tr.train()
    for k, e in exp.items():
        assert_bits(tr.results[0][k], e, k)
    assert mfl_amd.sharded_aggregator([DEV.index or 0] * 3).rounds_sharded >= 1


def test_device_resident_and_small_rounds_are_delegated():
    _, w_locals, expected = load_case("mnist_lr_k10")
    agg = mfl_amd.ShardedAggregator([DEV.index or 0] * 4)
    out = agg.aggregate(copy.deepcopy(w_locals))  # 314 KB of rows: one native call on one device
    for k, e in expected.items():
        assert_bits(out[k], e, k)
    dev_wl = [(n, OrderedDict((k, v.to(DEV)) for k, v in sd.items())) for n, sd in copy.deepcopy(w_locals)]
    out = agg.aggregate(dev_wl)
    assert next(iter(out.values())).is_cuda  # reduced where the clients lie
    for k, e in expected.items():
        assert_bits(out[k].cpu(), e, k)
    assert agg.rounds_delegated == 2 and agg.rounds_sharded == 0


# -- streamed rounds over shards (install(devices=[...]), autostream's default path) ----------

STREAM_CASES = ["mnist_lr_k10", "resnet_like_bn_k5", "int_dtypes_k3", "float64_key_k3", "bfloat16_key_k3",
                "float16_key_k3", "adversarial_k10", "ieee_specials_k4", "mnist_lr_k100", "flat_k1_p1",
                "flat_k10_p65", "single_client_k1", "scalar_key_k3", "float_counts_k4", "subnormal_products_k3",
                "thirds_k3", "sixths_k3", "flat_k7_p1000"]


class _Keyless:
    def load_state_dict(self, sd):
        pass


def _stream_trainer(rounds, n, monkeypatch, **kw):
    from loop_replay import fresh_classes

    monkeypatch.setattr("mfl_amd.autostream.ClientFeed.SMALL_ROUND_BYTES", 0)  # stream the tiny goldens too
    sagg = mfl_amd.sharded_aggregator([DEV.index or 0] * n)
    monkeypatch.setattr(sagg, "SMALL_ROUND_BYTES", 0)  # and shard them
    T, C = fresh_classes()
    mfl_amd.install(T, client_cls=C, stream_clients=True, devices=[DEV.index or 0] * n)
    first = rounds[0][0][1][-1]
    return T(OrderedDict((k, torch.zeros_like(v)) for k, v in first.items()), rounds, **kw), sagg


@pytest.mark.parametrize("n", [2, 8])
def test_install_devices_streams_golden_rounds_over_shards_bit_exact(n, monkeypatch):
    from loop_replay import rounds_from_cases

    cases = [load_case(c) for c in STREAM_CASES]
    rounds = rounds_from_cases(cases, n_rounds=len(cases))
    tr, sagg = _stream_trainer(rounds, n, monkeypatch, n_clients=100)
    tr.model_global = _Keyless()  # key tables change from round to round here
    before = sagg.rounds_streamed
    tr.train()
    feed = tr.__dict__["_mfl_feed"]
    assert feed.stats["rounds_streamed"] == len(rounds), feed.stats
    assert sagg.rounds_streamed - before == len(rounds)  # every round streamed over the shards
    for r, res in enumerate(tr.results):
        _, _, expected = cases[r]
        assert list(res.keys()) == list(expected.keys())
        for k, e in expected.items():
            assert_bits(res[k], e, f"round {r} ({STREAM_CASES[r]}) n={n} {k}")


@pytest.mark.parametrize("n", [2, 8])
def test_install_devices_streams_resnet56_x100_bit_exact_and_distances(n, monkeypatch):
    """The product rule (no threshold changes): resnet56 x 100 (240 MB of rows)
    streams over n shards, every round; :291 after it reads the shards'
    fused fp64 sums (1 ulp of the exact norms)."""
    from loop_replay import fresh_classes

    w_locals = _resnet56_host(seed=7)
    exp = O.aggregate_torch(copy.deepcopy(w_locals))
    sagg = mfl_amd.sharded_aggregator([DEV.index or 0] * n)
    T, C = fresh_classes()
    mfl_amd.install(T, client_cls=C, devices=[DEV.index or 0] * n)  # streaming on by default
    rounds = [[(c, [sd]) for c, sd in w_locals]] * 2
    tr = T(OrderedDict((k, torch.zeros_like(v)) for k, v in w_locals[0][1].items()), rounds)
    before = sagg.rounds_streamed
    wl_seen = []
    tr.after_append = lambda r, wl: wl_seen.append(wl)
    tr.train()
    feed = tr.__dict__["_mfl_feed"]
    assert feed.stats["rounds_streamed"] == 2 and sagg.rounds_streamed - before == 2, feed.stats
    assert feed.stats["last_round"]["finish_profile"]["shards"] == n
    for res in tr.results:
        for k, e in exp.items():
            assert_bits(res[k], e, f"resnet56 streamed n={n} {k}")
    wl = wl_seen[-1]
    out = wl[0][1]  # the last round's w_glob (:449: client 0's dict)
    got = np.asarray(sagg.client_distances(wl, out), dtype=np.float64)
    idx = [0, 1, 50, 99]
    ref = O.client_distances_exact([wl[i] for i in idx], out)
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    assert got[0] == 0.0
    assert np.all(np.abs(got[idx] - ref) <= ulp), (got[idx], ref)


def test_streamed_shards_fall_back_on_in_place_edit(monkeypatch):
    """An in-place edit between :199 and :217 (the version counter) falls back to
    the plain sharded path, with the reference's bits for the edited round."""
    w_locals = _resnet56_host(seed=9)
    expect = []

    def edit(r, wl):
        if r == 1:
            wl[42][1]["layer2.0.conv1.weight"].view(-1)[17] += 1e-3
        expect.append(O.aggregate_torch(copy.deepcopy(wl)))

    tr, sagg = _stream_trainer([[(c, [sd]) for c, sd in w_locals]] * 2, 4, monkeypatch, after_append=edit)
    tr.train()
    stats = tr.__dict__["_mfl_feed"].stats
    assert stats["rounds_streamed"] == 1 and stats["rounds_fallback"] == 1, stats
    assert stats["last_verify"]["status"] == 8 and stats["last_verify"]["client"] == 42
    for res, e in zip(tr.results, expect):
        for k, v in e.items():
            assert_bits(res[k], v, k)


def test_session_blocks_plain_round_on_the_same_shards():
    sagg = mfl_amd.ShardedAggregator([DEV.index or 0] * 2)
    w_locals = _resnet56_host(seed=11)
    sess = sagg.begin_round(w_locals[0][1], len(w_locals))
    assert isinstance(sess, mfl_amd.ShardedRoundSession)
    for c, sd in w_locals[:3]:
        sess.add(c, sd)
    with pytest.raises(RuntimeError):
        sagg.aggregate(copy.deepcopy(w_locals))
    sess.abandon()
    out = sagg.aggregate([(c, OrderedDict(sd)) for c, sd in w_locals])  # the staging is free again
    exp = O.aggregate_torch(copy.deepcopy(w_locals))
    for k, e in exp.items():
        assert_bits(out[k], e, k)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="distinct devices need >= 2 visible GPUs")
def test_distinct_devices_stream_and_plain_bit_exact(monkeypatch):
    """Every visible GPU one shard: the pinned staging read by several devices'
    DMA engines, per-device streams, results to one pinned buffer."""
    devs = list(range(torch.cuda.device_count()))
    w_locals = _resnet56_host(seed=13)
    exp = O.aggregate_torch(copy.deepcopy(w_locals))
    out = mfl_amd.sharded_aggregator(devs).aggregate([(c, OrderedDict(sd)) for c, sd in w_locals])
    for k, e in exp.items():
        assert_bits(out[k], e, k)
    from loop_replay import fresh_classes

    T, C = fresh_classes()
    monkeypatch.setenv("FEDAVG_STREAM_DISTINCT_DEVICES", "1")  # streaming over distinct GPUs is opt-in
    mfl_amd.install(T, client_cls=C, devices=devs)
    tr = T(OrderedDict((k, torch.zeros_like(v)) for k, v in w_locals[0][1].items()),
           [[(c, [sd]) for c, sd in w_locals]])
    tr.train()
    assert tr.__dict__["_mfl_feed"].stats["rounds_streamed"] == 1
    for k, e in exp.items():
        assert_bits(tr.results[0][k], e, k)
