"""GPU parity of the FPF2 bookkeeping (fedavg_trainer.py:108-119, 210, 271-278, 314-327).

* Against the reference itself: the rounds captured from the reference's own
  ``train()`` loop (tests/golden/fpf, oracle/gen_golden_fpf.py) are replayed
  through ``mfl_amd.FPFTracker`` + the GPU aggregate; every per-round FPF2 row
  must match the reference's CSV row (zeros exactly, others to rtol 1e-5 --
  the index is a norm, accumulated in fp64 here and in fp32 lanes by ATen).
* Against the oracle on random rounds at the reference's real size
  (client_num_in_total = 1000 vehicles, MNIST-LR P = 7850): ``local_w_diffs``,
  ``G_mat``, ``local_itr_lst`` and ``LRU_itr_lst`` bit-identical; ``A_mat``
  (one fp32 mean per round) to rtol 1e-5.
"""
import copy
from collections import OrderedDict

import numpy as np
import pytest
import torch

import fedavg_oracle as O
import fpf_oracle as FO
import fpf_replay
import mfl_amd

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
RTOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    """A plain ``pytest`` on a GPU-less box skips this module like the other test_gpu_* modules."""
    yield


class _TrackerImpl:
    def __init__(self, meta, init, g2=FO.G2):
        self.t = mfl_amd.FPFTracker(meta["client_num_in_total"], init, meta["comm_round"], device=DEV,
                                    threshold=meta["threshold"], g2=g2)

    def begin_round(self, last_w):
        self.t.begin_round(last_w)

    def record_client(self, c, w, last_w):
        self.t.record_client(c, w)

    def record_round(self, idx, w_locals, w_glob):
        self.t.record_round(idx, w_locals, w_glob)

    def aggregate(self, w_locals, model_state):
        if not w_locals:
            return copy.deepcopy(model_state)  # fedavg_trainer.py:442-443
        return mfl_amd.aggregate(w_locals, device=DEV)

    def fpf_index(self):
        return self.t.fpf_index()

    def end_round(self, t, idx, itr, w_glob, last_w):
        self.t.end_round(t, idx, itr, w_glob)


class _DeviceTrackerImpl(_TrackerImpl):
    """The same loop with every state_dict on the GPU (client.py:96 without
    the .cpu()): last_w, the clients and the aggregate's result."""

    def __init__(self, meta, init):
        super().__init__(meta, init)
        self._dev = {}

    def _d(self, sd):
        if id(sd) not in self._dev:  # keeps sd alive, so the id is not reused
            self._dev[id(sd)] = (sd, OrderedDict((k, v.to(DEV)) for k, v in sd.items()))
        return self._dev[id(sd)][1]

    def begin_round(self, last_w):
        self.t.begin_round(self._d(last_w))

    def record_client(self, c, w, last_w):
        self.t.record_client(c, self._d(w))

    def record_round(self, idx, w_locals, w_glob):
        self.t.record_round(idx, [(n, self._d(sd)) for n, sd in w_locals], w_glob)

    def aggregate(self, w_locals, model_state):
        if not w_locals:
            return self._d(copy.deepcopy(model_state))
        out = mfl_amd.aggregate([(n, self._d(sd)) for n, sd in w_locals])
        assert all(v.device == DEV for v in out.values())
        return out


class _OracleImpl(_TrackerImpl):
    def __init__(self, meta, init, g2=FO.G2):
        weight_size = sum(v.numel() for v in init.values())
        self.o = FO.FPFOracle(meta["client_num_in_total"], weight_size, meta["comm_round"], meta["threshold"], g2=g2)

    def begin_round(self, last_w):
        pass

    def record_client(self, c, w, last_w):
        self.o.record_client(c, w, last_w)

    def aggregate(self, w_locals, model_state):
        if not w_locals:
            return copy.deepcopy(model_state)
        return O.aggregate_torch(w_locals)

    def fpf_index(self):
        return self.o.fpf_index()

    def end_round(self, t, idx, itr, w_glob, last_w):
        self.o.end_round(t, idx, itr, w_glob, last_w)


def assert_fpf_rows(got, exp):
    exp = np.asarray(exp, dtype=np.float64)
    got = np.asarray(got, dtype=np.float64)
    assert got.shape == exp.shape
    assert np.array_equal(got == 0, exp == 0), "zero (scrubbed) positions differ"
    np.testing.assert_allclose(got, exp, rtol=RTOL, atol=0)


@pytest.mark.parametrize("after", [False, True], ids=["record_client", "record_round"])
@pytest.mark.parametrize("name", fpf_replay.case_names())
def test_fpf_tracker_matches_reference_loop(name, after):
    case = fpf_replay.load_case(name)
    impl = _TrackerImpl(case.meta, case.init)
    got = fpf_replay.replay(case, impl, record_after_aggregate=after)
    assert_fpf_rows(got, case.fpf)


@pytest.mark.parametrize("after", [False, True], ids=["record_client", "record_round"])
@pytest.mark.parametrize("name", fpf_replay.case_names())
def test_fpf_tracker_device_resident_clients(name, after):
    case = fpf_replay.load_case(name)
    got = fpf_replay.replay(case, _DeviceTrackerImpl(case.meta, case.init), record_after_aggregate=after)
    assert_fpf_rows(got, case.fpf)
    host = fpf_replay.replay(case, _TrackerImpl(case.meta, case.init), record_after_aggregate=after)
    assert np.array_equal(got.view(np.uint32), host.view(np.uint32))  # same bits as the host-client loop


def _random_case(n_total, P, rounds, seed, threshold=FO.THRESHOLD_WEIGHT_SIZE, bn=False):
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    init = OrderedDict(weight=torch.randn(P - 10, generator=g), bias=torch.randn(10, generator=g))
    if bn:
        init["num_batches_tracked"] = torch.tensor(5, dtype=torch.int64)
        init["weight"] = init["weight"][:-1].clone()
    meta = {"client_num_in_total": n_total, "comm_round": len(rounds), "threshold": threshold, "rounds": []}
    states = []
    for t, (K, itr) in enumerate(rounds):
        K = min(K, n_total)
        idx = sorted(rng.choice(n_total, size=K, replace=False).tolist())
        if t == 2 and K >= 3:
            idx[-1] = idx[0]  # a duplicate: the later client's row wins (sequential :210 writes)
        rng.shuffle(idx)
        meta["rounds"].append({"client_indexes": idx, "local_itr": itr,
                               "sample_nums": rng.integers(1, 500, size=K).tolist()})
        # client states are drawn around the initial model; the replay's last_w is the running average
        round_states = []
        for _ in range(K):
            sd = OrderedDict()
            for k, v in init.items():
                sd[k] = (v + 1 if v.dtype == torch.int64
                         else v + 0.05 * torch.randn(v.shape, generator=g) * (1 + t))
            round_states.append(sd)
        states.append(round_states)
    return fpf_replay.FPFCase(meta, init, states, None)


def _replay_both(case, after, g2=FO.G2):
    tr = _TrackerImpl(case.meta, case.init, g2)
    orc = _OracleImpl(case.meta, case.init, g2)
    rows_t = fpf_replay.replay(case, tr, record_after_aggregate=after)
    rows_o = fpf_replay.replay(case, orc)
    return tr.t, orc.o, rows_t, rows_o


ROUNDS = [(20, 2), (35, 3), (12, 1), (40, 0), (1, 5), (64, 2)]


@pytest.mark.parametrize("after", [False, True], ids=["record_client", "record_round"])
def test_fpf_state_vs_oracle_reference_size(after):
    """1000 vehicles x MNIST-LR (P = 7850), the reference's own FPF2 configuration."""
    case = _random_case(1000, 7850, ROUNDS, seed=7)
    t, o, rows_t, rows_o = _replay_both(case, after)
    assert t.full and o.full
    assert torch.equal(t.local_w_diffs.cpu(), o.local_w_diffs)  # bit-identical
    assert torch.equal(t.G_mat.cpu(), o.G_mat)
    assert torch.equal(t.local_itr_lst.cpu(), o.local_itr_lst)
    a_t, a_o = t.A_mat.cpu().double().numpy(), o.A_mat.double().numpy()
    np.testing.assert_allclose(a_t, a_o, rtol=RTOL, atol=RTOL * np.abs(a_o).max())
    for r in range(len(ROUNDS)):
        assert_fpf_rows(rows_t[r], rows_o[r])


def test_fpf_state_vs_oracle_int_buffer_and_odd_p():
    case = _random_case(37, 1013, ROUNDS, seed=11, bn=True)
    t, o, rows_t, rows_o = _replay_both(case, True)
    assert torch.equal(t.local_w_diffs.cpu(), o.local_w_diffs)
    assert torch.equal(t.G_mat.cpu(), o.G_mat)
    for r in range(len(ROUNDS)):
        assert_fpf_rows(rows_t[r], rows_o[r])


def test_fpf_lru_mode_exact():
    case = _random_case(300, 2000, ROUNDS, seed=3, threshold=1000)
    t, o, rows_t, rows_o = _replay_both(case, False)
    assert not t.full and not o.full
    assert torch.equal(t.LRU_itr_lst.cpu(), o.LRU_itr_lst)
    assert torch.equal(t.G_mat.cpu(), o.G_mat)
    assert np.array_equal(rows_t, rows_o)


def test_fpf_near_threshold_many_blocks():
    """P just under THRESHOLD_WEIGHT_SIZE: multi-block mean partials, 1000 rows."""
    case = _random_case(1000, 99_990, [(50, 2), (100, 1), (30, 3)], seed=5)
    t, o, rows_t, rows_o = _replay_both(case, True)
    assert torch.equal(t.local_w_diffs.cpu(), o.local_w_diffs)
    a_t, a_o = t.A_mat.cpu().double().numpy(), o.A_mat.double().numpy()
    np.testing.assert_allclose(a_t, a_o, rtol=RTOL, atol=RTOL * np.abs(a_o).max())
    for r in range(3):
        assert_fpf_rows(rows_t[r], rows_o[r])


def test_fpf_errors_like_reference():
    init = OrderedDict(weight=torch.zeros(10, 5), bias=torch.zeros(10))
    t = mfl_amd.FPFTracker(8, init, 3, device=DEV)
    t.begin_round(init)
    with pytest.raises(IndexError):
        t.record_client(8, init)  # local_w_diffs[8] with 8 rows (:210)
    t.record_client(-1, init)  # negative indexes wrap like torch's
    with pytest.raises(IndexError):
        t.end_round(3, [0], 1, init)  # local_itr_lst[3] with comm_round = 3 (:322)
    with pytest.raises(IndexError):
        t.end_round(0, [9], 1, init)
    with pytest.raises(ValueError):
        t.record_round([0], [(1, copy.deepcopy(init))], init)  # no device rows of this round
    tb = mfl_amd.FPFTracker(8, OrderedDict(w=torch.zeros(3), m=torch.zeros(2, dtype=torch.bool)), 3, device=DEV)
    tb.begin_round(OrderedDict(w=torch.zeros(3), m=torch.zeros(2, dtype=torch.bool)))
    with pytest.raises(RuntimeError):
        tb.record_client(0, OrderedDict(w=torch.ones(3), m=torch.ones(2, dtype=torch.bool)))


# ---------------------------------------------------------------------------
# models with fp64 / fp16 / bf16 keys: torch.cat's promotion at :210 / :316
# ---------------------------------------------------------------------------
F16, BF16, F32, F64 = torch.float16, torch.bfloat16, torch.float32, torch.float64

# (weight dtype, bias dtype, integer buffer?) -> torch.cat's dtype T
MIXED = {
    "f32w_f64b": ((F32, F64, False), F64),
    "f64_only": ((F64, F64, False), F64),
    "f64w_int": ((F64, F32, True), F64),
    "f32w_f16b": ((F32, F16, False), F32),
    "bf16w_f32b_int": ((BF16, F32, True), F32),
    "f16w_bf16b": ((F16, BF16, False), F32),
    "f16_only_int": ((F16, F16, True), F16),
    "bf16_only": ((BF16, BF16, False), BF16),
}
# A_mat / index tolerance by T: one fp64 / fp32 mean each (ours summed in fp64
# in a fixed order); a 16-bit T rounds the mean and the :319 term to 16 bits,
# where a different mean rounding moves the term by one 16-bit ulp
MIXED_RTOL = {F64: 1e-12, F32: RTOL, F16: 2e-3, BF16: 1.6e-2}


def _mixed_case(n_total, P, rounds, seed, wdt, bdt, int_key):
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    nb = 10
    init = OrderedDict(weight=torch.randn(P - nb - int(int_key), generator=g).to(wdt),
                       bias=torch.randn(nb, generator=g).to(bdt))
    if int_key:
        init["num_batches_tracked"] = torch.tensor(5, dtype=torch.int64)
    meta = {"client_num_in_total": n_total, "comm_round": len(rounds), "threshold": FO.THRESHOLD_WEIGHT_SIZE,
            "rounds": []}
    states = []
    for t, (K, itr) in enumerate(rounds):
        K = min(K, n_total)
        idx = sorted(rng.choice(n_total, size=K, replace=False).tolist())
        if t == 2 and K >= 3:
            idx[-1] = idx[0]
        rng.shuffle(idx)
        meta["rounds"].append({"client_indexes": idx, "local_itr": itr,
                               "sample_nums": rng.integers(1, 500, size=K).tolist()})
        round_states = []
        for _ in range(K):
            sd = OrderedDict()
            for k, v in init.items():
                sd[k] = (v + 1 if v.dtype == torch.int64
                         else (v.float() + 0.05 * torch.randn(v.shape, generator=g) * (1 + t)).to(v.dtype))
            round_states.append(sd)
        states.append(round_states)
    return fpf_replay.FPFCase(meta, init, states, None)


@pytest.mark.parametrize("after", [False, True], ids=["record_client", "record_round"])
@pytest.mark.parametrize("name", list(MIXED))
def test_fpf_promoted_dtypes_vs_oracle(name, after):
    """fedavg_trainer.py:210/:316-319/:272 on models whose keys promote torch.cat
    to fp64 / fp32 / fp16 / bf16: local_w_diffs, G_mat and local_itr_lst
    bit-identical to the oracle (the reference's own torch expressions), A_mat
    of the reference's dtype (fp64 once an fp64 key is in the model) and the
    FPF2 index of its dtype, within MIXED_RTOL."""
    (wdt, bdt, int_key), T = MIXED[name]
    case = _mixed_case(60, 1500, ROUNDS, seed=17, wdt=wdt, bdt=bdt, int_key=int_key)
    t, o, rows_t, rows_o = _replay_both(case, after)
    assert t._mixed and t.T == T
    assert torch.equal(t.local_w_diffs.cpu(), o.local_w_diffs)  # bit-identical
    assert torch.equal(t.G_mat.cpu(), o.G_mat)
    assert torch.equal(t.local_itr_lst.cpu(), o.local_itr_lst)
    assert t.A_mat.dtype == o.A_mat.dtype  # fp64 after the first round when T is fp64
    rtol = MIXED_RTOL[T]
    a_t, a_o = t.A_mat.cpu().double().numpy(), o.A_mat.double().numpy()
    np.testing.assert_allclose(a_t, a_o, rtol=rtol, atol=rtol * np.abs(a_o).max())
    got, exp = t.fpf_index(), o.fpf_index()
    assert got.dtype == exp.dtype  # fp64 index once A_mat is fp64
    assert np.array_equal(got == 0, exp == 0)
    np.testing.assert_allclose(got, exp, rtol=rtol, atol=0)
    for r in range(len(ROUNDS)):
        assert np.array_equal(rows_t[r] == 0, rows_o[r] == 0)
        np.testing.assert_allclose(rows_t[r], rows_o[r], rtol=max(rtol, RTOL), atol=0)


@pytest.mark.parametrize("name", ["f32w_f64b", "f16_only_int"])
def test_fpf_promoted_device_clients(name):
    """The promoted path with every state_dict on the GPU: same bits as the
    host-client loop."""
    (wdt, bdt, int_key), T = MIXED[name]
    case = _mixed_case(40, 900, ROUNDS[:4], seed=23, wdt=wdt, bdt=bdt, int_key=int_key)
    for after in (False, True):
        got = fpf_replay.replay(case, _DeviceTrackerImpl(case.meta, case.init), record_after_aggregate=after)
        host = fpf_replay.replay(case, _TrackerImpl(case.meta, case.init), record_after_aggregate=after)
        assert np.array_equal(got.view(np.uint32), host.view(np.uint32))


@pytest.mark.parametrize("name", ["f32w_f64b", "f64_only", "f32w_f16b"])
def test_fpf_g2_not_a_power_of_two(name):
    """G2 = 3: (1 - 1/G2) is not an fp32 number.  The reference's first
    end_round multiplies its fp32 A_mat (:114) by it in fp32 and only then
    promotes (:319) -- A_mat after every round of the fp64 models within
    1e-12 of the oracle, the fp32 model within the fp32 tolerance."""
    (wdt, bdt, int_key), T = MIXED[name]
    case = _mixed_case(30, 700, ROUNDS[:4], seed=29, wdt=wdt, bdt=bdt, int_key=int_key)
    for r_end in range(1, 5):
        sub = fpf_replay.FPFCase(dict(case.meta, rounds=case.meta["rounds"][:r_end], comm_round=r_end), case.init,
                                 case.client_states[:r_end], None)
        t, o, _, _ = _replay_both(sub, False, g2=3)
        assert t.A_mat.dtype == o.A_mat.dtype
        rtol = MIXED_RTOL[T]
        a_t, a_o = t.A_mat.cpu().double().numpy(), o.A_mat.double().numpy()
        np.testing.assert_allclose(a_t, a_o, rtol=rtol, atol=rtol * np.abs(a_o).max(), err_msg=f"round {r_end}")


def test_fpf_promoted_first_round_index_is_fp32():
    """Before the first end_round A_mat is the fp32 ones of :114, so the
    index of a model with an fp64 key is still fp32 (norm of fp32 * fp32)."""
    init = OrderedDict(w=torch.randn(50), b=torch.randn(5, dtype=torch.float64))
    t = mfl_amd.FPFTracker(8, init, 3, device=DEV)
    o = FO.FPFOracle(8, 55, 3)
    t.begin_round(init)
    w = OrderedDict(w=init["w"] + 0.5, b=init["b"] - 0.25)
    t.record_client(3, w)
    o.record_client(3, w, init)
    got, exp = t.fpf_index(), o.fpf_index()
    assert got.dtype == exp.dtype == np.float32
    assert torch.equal(t.local_w_diffs.cpu(), o.local_w_diffs)
    np.testing.assert_array_equal(got, exp)  # G_mat = 0: inf/NaN scrubbed to 0 on both sides


@pytest.mark.parametrize("name", ["float64_key_k3", "float16_key_k3", "bfloat16_key_k3"])
def test_fpf_promoted_on_reference_dtype_goldens(name):
    """One FPF2 round over the reference-captured dtype goldens: last_w is the
    first client's model, the K clients are the round's, w_glob is the
    reference's own aggregate output (tests/golden)."""
    from golden_io import load_case

    meta, w_locals, expected = load_case(name)
    last_w = copy.deepcopy(w_locals[0][1])
    P = sum(v.numel() for v in last_w.values())
    n = len(w_locals) + 2
    t = mfl_amd.FPFTracker(n, last_w, 2, device=DEV)
    o = FO.FPFOracle(n, P, 2)
    t.begin_round(last_w)
    idx = list(range(1, len(w_locals) + 1))
    for c, (_, w) in zip(idx, w_locals):
        t.record_client(c, w)
        o.record_client(c, w, last_w)
    t.end_round(0, idx, 2, expected)
    o.end_round(0, idx, 2, expected, last_w)
    assert torch.equal(t.local_w_diffs.cpu(), o.local_w_diffs)
    assert t.A_mat.dtype == o.A_mat.dtype
    rtol = MIXED_RTOL[t.T]
    np.testing.assert_allclose(t.A_mat.cpu().double().numpy(), o.A_mat.double().numpy(), rtol=rtol)
    got, exp = t.fpf_index(), o.fpf_index()
    assert got.dtype == exp.dtype
    np.testing.assert_allclose(got, exp, rtol=rtol, atol=0)
