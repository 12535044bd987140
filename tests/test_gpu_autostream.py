"""Zero-edit streaming on the GPU: mfl_amd.install on the loop-replay harness
(tests/loop_replay.py, shaped like fedavg_trainer.py:172-219 and client.py)
streams each valid client's upload and must give the golden vectors' bits;
rounds whose w_locals is not what was streamed fall back to the plain path
with the reference's results."""
import copy
from collections import OrderedDict

import pytest
import torch

import fedavg_oracle as O
import mfl_amd
from golden_io import load_case
from loop_replay import fresh_classes, rounds_from_cases
from test_gpu_parity import DEV, assert_bits

pytestmark = pytest.mark.gpu

CASES = ["mnist_lr_k10", "resnet_like_bn_k5", "int_dtypes_k3", "float64_key_k3", "bfloat16_key_k3",
         "adversarial_k10", "ieee_specials_k4", "float16_key_k3", "mnist_lr_k100"]


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield


@pytest.fixture(autouse=True)
def _stream_small_rounds(request, monkeypatch):
    # the golden cases are small rounds, which the feed leaves to the plain
    # path by default; stream them here so the streamed path is what is checked
    if "default_threshold" not in request.keywords:
        monkeypatch.setattr("mfl_amd.autostream.ClientFeed.SMALL_ROUND_BYTES", 0)


def _trainer(rounds, **kw):
    T, C = fresh_classes()
    mfl_amd.install(T, device=DEV, client_cls=C, stream_clients=True)
    first = rounds[0][0][1][-1]
    return T(OrderedDict((k, torch.zeros_like(v)) for k, v in first.items()), rounds, **kw)


def test_install_streams_golden_rounds_bit_exact():
    cases = [load_case(n) for n in CASES]
    rounds = rounds_from_cases(cases, n_rounds=2 * len(cases))
    tr = _trainer(rounds, n_clients=100)
    tr.model_global = _Keyless()  # load_state_dict of changing key tables: the harness skips :219 here
    tr.train()
    feed = tr.__dict__["_mfl_feed"]
    assert feed.stats["rounds_streamed"] == len(rounds), feed.stats
    for r, res in enumerate(tr.results):
        _, _, expected = cases[r % len(cases)]
        assert list(res.keys()) == list(expected.keys())
        for k, e in expected.items():
            assert_bits(res[k], e, f"round {r} ({CASES[r % len(cases)]}) {k}")


class _Keyless:
    def load_state_dict(self, sd):
        pass


def test_retried_clients_still_stream():
    _, w_locals, expected = load_case("resnet_like_bn_k5")
    rounds = [[(n, [None, None, sd] if i % 2 else [sd]) for i, (n, sd) in enumerate(w_locals)]] * 2
    tr = _trainer(rounds)
    tr.train()
    assert tr.__dict__["_mfl_feed"].stats["rounds_streamed"] == 2
    for res in tr.results:
        for k, e in expected.items():
            assert_bits(res[k], e, k)


@pytest.mark.parametrize("where", ["sampled", "count"])
def test_changed_w_locals_falls_back_to_reference_bits(where):
    _, w_locals, _ = load_case("mnist_lr_k10")
    rounds = [[(n, [sd]) for n, sd in w_locals]] * 2
    expect = []

    def change(r, wl):
        if r == 1:
            if where == "sampled":
                wl[3][1]["linear.weight"].view(-1)[0] += 0.5  # first element of the largest key: a sampled position
            else:
                wl.append((wl[0][0], copy.deepcopy(wl[0][1])))
        expect.append(O.aggregate_torch(copy.deepcopy(wl)))

    tr = _trainer(rounds, after_append=change)
    tr.train()
    stats = tr.__dict__["_mfl_feed"].stats
    assert stats["rounds_streamed"] == 1 and stats["rounds_fallback"] == 1, stats
    for res, exp in zip(tr.results, expect):
        for k, e in exp.items():
            assert_bits(res[k], e, k)


def test_plain_round_after_streamed_round():
    """A plain aggregate between streamed rounds on the same aggregator, and
    the streamed round's rows left for client_distances (:291)."""
    _, w_locals, expected = load_case("mnist_lr_k100")
    tr = _trainer([[(n, [sd]) for n, sd in w_locals]])
    tr.train()
    assert tr.__dict__["_mfl_feed"].stats["rounds_streamed"] == 1
    out = mfl_amd.aggregate(copy.deepcopy(w_locals), device=DEV)  # plain path, same default aggregator
    for k, e in expected.items():
        assert_bits(out[k], e, k)
        assert_bits(tr.results[0][k], e, k)


@pytest.mark.default_threshold
def test_small_rounds_take_the_plain_path():
    _, w_locals, expected = load_case("mnist_lr_k10")
    tr = _trainer([[(n, [sd]) for n, sd in w_locals]] * 3, n_clients=100)
    tr.train()
    stats = tr.__dict__["_mfl_feed"].stats
    assert stats["rounds_small"] == 3 and stats["rounds_streamed"] == 0 and stats["rounds_fallback"] == 0, stats
    for res in tr.results:
        for k, e in expected.items():
            assert_bits(res[k], e, k)
