"""Pin the CPU oracle against the reference's own outputs (CPU only).

The golden vectors were produced by running the reference
``FedAvgTrainer.aggregate`` (fedavg_trainer.py:441-458) in the build
container (oracle/gen_golden.py).  Both oracle restatements -- the torch loop
(also the bench's CPU baseline) and the numpy one -- must reproduce them bit
for bit.
"""
import copy
import hashlib

import numpy as np
import pytest
import torch

import fedavg_oracle as O
from golden_io import bits_equal, case_names, load_case

CASES = case_names()


def test_golden_present():
    assert len(CASES) >= 20


@pytest.mark.parametrize("name", CASES)
def test_golden_sha256(name):
    meta, _, expected = load_case(name)
    for k in meta["out_keys"]:
        t = expected[k["name"]]
        if t.dtype == torch.bfloat16:
            raw = t.view(torch.int16).numpy()
        else:
            raw = t.numpy()
        assert hashlib.sha256(np.ascontiguousarray(raw).tobytes()).hexdigest() == k["sha256"]


@pytest.mark.parametrize("name", CASES)
def test_torch_restatement_matches_reference(name):
    meta, w_locals, expected = load_case(name)
    if meta["K"] == 0:
        pytest.skip("empty w_locals is covered by test_empty_case")
    first = w_locals[0][1]
    out = O.aggregate_torch(w_locals)
    assert out is first  # fedavg_trainer.py:449 aliasing
    assert list(out.keys()) == list(expected.keys())
    for k in expected:
        assert bits_equal(out[k], expected[k]), k


@pytest.mark.parametrize("name", CASES)
def test_numpy_restatement_matches_reference(name):
    meta, w_locals, expected = load_case(name)
    if meta["K"] == 0:
        pytest.skip("empty")
    bf16 = [k["name"] for k in meta["in_keys"] if k["dtype"] == "bfloat16"]
    np_locals = []
    for n, sd in w_locals:
        np_locals.append((n, {k: (v.view(torch.int16).numpy() if v.dtype == torch.bfloat16 else v.numpy())
                              for k, v in sd.items()}))
    out = O.aggregate_numpy(np_locals, bf16_keys=bf16)
    for k, exp in expected.items():
        got = out[k]
        if exp.dtype == torch.bfloat16:
            got_t = torch.from_numpy(np.asarray(got).astype(np.uint16).view(np.int16).copy()).view(torch.bfloat16)
        else:
            got_t = torch.from_numpy(np.array(got))
        assert bits_equal(got_t.reshape(exp.shape), exp), k


def test_empty_case():
    meta, w_locals, expected = load_case("empty_w_locals")
    assert meta["K"] == 0 and not meta["aliased"]
    torch.manual_seed(0)
    glob = torch.nn.Linear(5, 3)
    out = O.empty_result(glob)
    for k in expected:
        assert bits_equal(out[k], expected[k])


def test_zero_total_raises():
    with pytest.raises(ZeroDivisionError):
        O.sample_weights([0, 0])


def test_int64_example_value():
    # survey-verified: nbt 7, 8, 9 with n = 10, 20, 30 -> 8.3333 (fp32)
    _, _, expected = load_case("int64_nbt_example")
    assert expected["nbt"].dtype == torch.float32
    assert abs(float(expected["nbt"]) - 8.333333) < 1e-5


@pytest.mark.parametrize("name", ["mnist_lr_k10", "resnet_like_bn_k5", "adversarial_k10", "sixths_k3"])
def test_distance_oracles_agree(name):
    """fedavg_trainer.py:291: ATen's fp32 norm and the fp64-accurate restatement
    agree to ATen's rounding error; client 0 (aliased to w_glob) is 0."""
    _, w_locals, _ = load_case(name)
    w_glob = O.aggregate_torch(w_locals)
    t = O.client_distances_torch(w_locals, w_glob)
    e = O.client_distances_exact(w_locals, w_glob)
    assert t[0] == 0.0 and e[0] == 0.0
    assert np.allclose(t, e, rtol=1e-5, atol=0)
    d = O.delta_from_norms([n for n, _ in w_locals], t, 0.03)
    assert np.isfinite(d)


def test_distance_with_bool_buffer_raises_like_reference():
    _, w_locals, _ = load_case("int_dtypes_k3")  # has a bool key
    w_glob = O.aggregate_torch(w_locals)
    with pytest.raises(RuntimeError):
        O.client_distances_torch(w_locals, w_glob)


# ---------------------------------------------------------------------------
# FPF2 bookkeeping (fedavg_trainer.py:108-119, 210, 271-278, 314-327)
import fpf_oracle as FO  # noqa: E402
import fpf_replay  # noqa: E402

FPF_CASES = fpf_replay.case_names()


class _OracleImpl:
    def __init__(self, case):
        m = case.meta
        self.o = FO.FPFOracle(m["client_num_in_total"], m["weight_size"], m["comm_round"], m["threshold"])

    def begin_round(self, last_w):
        pass

    def record_client(self, c, w, last_w):
        self.o.record_client(c, w, last_w)

    def aggregate(self, w_locals, model_state):
        if not w_locals:
            return copy.deepcopy(model_state)  # fedavg_trainer.py:442-443
        return O.aggregate_torch(w_locals)

    def fpf_index(self):
        return self.o.fpf_index()

    def end_round(self, t, idx, itr, w_glob, last_w):
        self.o.end_round(t, idx, itr, w_glob, last_w)


def test_fpf_golden_present():
    assert {"lr_full", "bn_full", "lr_lru"} <= set(FPF_CASES)


@pytest.mark.parametrize("name", FPF_CASES)
def test_fpf_oracle_matches_reference_loop(name):
    """The restatement reproduces the reference train() loop's FPF CSV bit for bit."""
    case = fpf_replay.load_case(name)
    got = fpf_replay.replay(case, _OracleImpl(case))
    assert got.shape == case.fpf.shape
    assert np.array_equal(got.astype(np.float64), case.fpf)
    assert case.meta["full"] == (not name.endswith("_lru"))
    if case.meta["full"]:
        # empty round 6 -> A_mat NaN (0/0 at :319) -> every later index scrubbed to 0
        assert np.count_nonzero(case.fpf[6]) > 0 and not np.any(case.fpf[7])


@pytest.mark.parametrize("name", ["float64_key_k3", "float16_key_k3", "bfloat16_key_k3"])
def test_distance_oracles_agree_other_dtypes(name):
    """:291 on fp64 / fp16 / bf16 keys: torch.cat promotes the per-key
    differences (fp64 + fp32 -> fp64; fp16 alone -> fp16; bf16 alone -> bf16)
    and the norm is of that dtype.  The accurate restatement rounds to the same
    dtype and agrees with ATen's norm to within one unit of that dtype."""
    import torch

    _, w_locals, _ = load_case(name)
    w_glob = O.aggregate_torch(w_locals)
    t = O.client_distances_torch(w_locals, w_glob)
    e = O.client_distances_exact(w_locals, w_glob)
    d = torch.cat([w_locals[1][1][k].reshape(-1) - w_glob[k].reshape(-1) for k in w_glob]).dtype
    assert d == {"float64_key_k3": torch.float64, "float16_key_k3": torch.float16,
                 "bfloat16_key_k3": torch.bfloat16}[name]
    eps = torch.finfo(d).eps
    assert t[0] == 0.0 and e[0] == 0.0
    assert np.allclose(t, e, rtol=2 * eps, atol=0), (t, e)


# ---------------------------------------------------------------------------
# The loop's scheduler statistics (fedavg_trainer.py:289-305): delta from the
# :291 norms, rho and beta -- the reference's own values from its train()
STATS_CASES = [n for n in fpf_replay.case_names(stats_only=True) if "stats" in np.load(
    fpf_replay.FPF_DIR / f"{n}.npz").files]


def test_stats_golden_present():
    assert {"lr_full", "big_lru", "target_lru"} <= set(STATS_CASES)


@pytest.mark.parametrize("name", STATS_CASES)
def test_round_stats_oracle_matches_reference_loop(name):
    """The restatement (aggregate_torch, client_distances_torch, round_stats_update)
    reproduces the reference's delta / rho / beta after every round bit for bit:
    same torch CPU expressions on the same inputs.  ``big_lru`` (P = 1,001,000)
    and ``target_lru`` (P = 25,005,000, ~15 s) also check that their regenerated
    client states are the reference's inputs (sha256 per client, in
    FPFCase.client_state)."""
    case = fpf_replay.load_case(name)
    agg = lambda wl, ms: copy.deepcopy(ms) if not wl else O.aggregate_torch(wl)  # noqa: E731
    got, _ = fpf_replay.replay_stats(case, agg, O.client_distances_torch)
    assert got.shape == case.stats.shape
    assert np.array_equal(got, case.stats), (got - case.stats)


def test_big_lru_fpf_rows_match_reference():
    case = fpf_replay.load_case("big_lru")
    assert case.meta["weight_size"] == 1_001_000 and not case.meta["full"]
    got = fpf_replay.replay(case, _OracleImpl(case))
    assert np.array_equal(got.astype(np.float64), case.fpf)
