"""GPU parity of :291 -> delta against the REFERENCE's own delta.

``tests/golden/fpf`` holds, per scenario, ``(rho, beta, delta)`` after every
round of the reference's own ``train()`` loop (fedavg_trainer.py:289-305;
captured by oracle/gen_golden_fpf.py where the loop hands them to its
scheduler, :309-310).  These tests replay the same rounds with the GPU
aggregate (:217) and the GPU :291 norms (``mfl_amd.client_distances`` /
``estimate_delta``) and compare delta with the reference's.

Tolerance.  The GPU norms are the accurate value of :291 (squares summed in
fp64, the root rounded to torch.cat's dtype: within 1 ulp of
``oracle.client_distances_exact``).  The reference's own norm accumulates in
fp32 SIMD lanes (ATen's CPU ``norm``), so its error grows with P: measured
1.2e-7 at P = 1,010 and 1.3e-5 at P = 1,001,000 against the exact norm (the
reference's delta is itself that far from exact; its value depends on the
host's vector width).  DELTA_RTOL bounds |delta_gpu - delta_ref| /
|delta_ref| by 4x the measured error of the reference's norm at that P:
1e-6 for the fp32 scenarios with P <= 1,010, 1e-12 for fp64 (the reference
accumulates fp64 norms in fp64), 0 for fp16 (the root rounded to fp16 hides
the accumulation), 5e-5 at P = 1,001,000 and 6e-3 at the target's P =
25,005,000 (measured 1.42e-3: the reference's own fp32 norm error there).
Against delta from the exact norms the GPU's is within EXACT_RTOL (about
one unit of the norm's dtype) at every size.  ``rho`` and ``beta`` (host
arithmetic on the clients' scalars) must match exactly.  Measured errors are
written to $MFL_REPORT_DIR/delta_parity.json when that is set (DESIGN.md
section 4 quotes them).
"""
import copy
import json
import os
from collections import OrderedDict

import numpy as np
import pytest
import torch

import fedavg_oracle as O
import fpf_replay
import mfl_amd
from loop_replay import fresh_classes

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
CASES = [n for n in fpf_replay.case_names(stats_only=True)
         if "stats" in np.load(fpf_replay.FPF_DIR / f"{n}.npz").files]
DELTA_RTOL = {"big_lru": 5e-5, "target_lru": 6e-3, "lr64_full": 1e-12, "lr64_lru": 1e-12, "bnmix64_full": 1e-12,
              "lr16_full": 0.0}
# GPU delta against delta from the exact norms (oracle.client_distances_exact), by torch.cat's dtype:
# every norm within one unit of that dtype, so their weighted mean within about one unit too
EXACT_RTOL = {torch.float32: 2.5e-7, torch.float64: 1e-13, torch.float16: 2e-3}
DEFAULT_RTOL = 1e-6
_REPORT = {}


@pytest.fixture(scope="module", autouse=True)
def _gpu(gpu_available):
    mfl_amd._lib.load()
    torch.cuda.set_device(DEV)
    yield
    out = os.environ.get("MFL_REPORT_DIR")
    if out and _REPORT:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "delta_parity.json"), "w") as fh:
            json.dump(_REPORT, fh, indent=1, sort_keys=True)


def _check(name, got, case, how):
    ref = case.stats
    assert got.shape == ref.shape
    assert np.array_equal(got[:, :2], ref[:, :2]), "rho / beta differ"
    rel = np.abs(got[:, 2] - ref[:, 2]) / np.abs(ref[:, 2])
    _REPORT.setdefault(name, {})[how] = {"delta_max_rel_err": float(rel.max()),
                                         "P": case.meta["weight_size"], "rounds": len(rel)}
    tol = DELTA_RTOL.get(name, DEFAULT_RTOL)
    assert rel.max() <= tol, (how, rel, tol)


def _host_agg(w_locals, model_state):
    if not w_locals:
        return copy.deepcopy(model_state)  # fedavg_trainer.py:442-443
    return mfl_amd.aggregate(w_locals, device=DEV)


@pytest.mark.parametrize("name", CASES)
def test_delta_matches_reference_functional(name):
    """aggregate + client_distances on host state_dicts (the rows the aggregate
    left in HBM, or its fused :291 sums); the norms within 1 ulp of the exact
    restatement, delta within DELTA_RTOL of the reference's."""
    case = fpf_replay.load_case(name)
    exact = []

    def norms(w_locals, w_glob):
        d = mfl_amd.client_distances(w_locals, w_glob, device=DEV)
        e = O.client_distances_exact(w_locals, w_glob)
        exact.append((d, e))
        return d

    got, _ = fpf_replay.replay_stats(case, _host_agg, norms)
    _check(name, got, case, "functional")
    cat = None  # torch.cat's promoted dtype at :291: the norm's dtype
    for v in case.init.values():
        cat = v.dtype if cat is None else torch.promote_types(cat, v.dtype)
    # delta (:293) from the GPU norms against delta from the exact ones, every non-empty round
    worst = 0.0
    rounds = [rd for rd in case.meta["rounds"] if rd["sample_nums"]]
    for rd, (d, e) in zip(rounds, exact):
        dg = O.delta_from_norms(rd["sample_nums"], d, case.meta["lr"])
        de = O.delta_from_norms(rd["sample_nums"], e, case.meta["lr"])
        worst = max(worst, abs(dg - de) / abs(de))
    _REPORT.setdefault(name, {})["gpu_vs_exact_delta_max_rel_err"] = worst
    assert worst <= EXACT_RTOL[cat], (worst, cat)
    for d, e in exact:
        if cat == torch.float64:  # fp64 sums in another order: a few fp64 ulps
            np.testing.assert_allclose(d, e, rtol=1e-13, atol=0)
        else:  # within one unit of the norm's dtype
            ulp = torch.from_numpy(np.abs(e)).to(cat)
            ulp = np.array([float(torch.nextafter(u, torch.tensor(float("inf"), dtype=cat)) - u) for u in ulp])
            assert np.all(np.abs(d - e) <= ulp), (d, e)


@pytest.mark.parametrize("name", ["big_lru", "lr_full", "bn_full"])
def test_delta_matches_reference_device_clients(name):
    """The same rounds with every client state_dict on the GPU: the zero-copy
    round (fused :291 sums from the clients' own tensors) and the same delta."""
    case = fpf_replay.load_case(name)

    def agg(w_locals, model_state):
        if not w_locals:
            return copy.deepcopy(model_state)
        dl = [(n, OrderedDict((k, v.to(DEV)) for k, v in sd.items())) for n, sd in w_locals]
        out = mfl_amd.aggregate(dl)
        agg.last = dl
        host = OrderedDict((k, v.cpu()) for k, v in out.items())
        agg.dev_out = out
        return host

    def norms(w_locals, w_glob):
        return mfl_amd.client_distances(agg.last, agg.dev_out)

    got, _ = fpf_replay.replay_stats(case, agg, norms)
    _check(name, got, case, "device_clients")


@pytest.mark.parametrize("name", CASES)
def test_delta_through_installed_streaming_loop(name, monkeypatch):
    """The zero-edit path: ``mfl_amd.install`` on the loop harness with
    streaming on (each client uploaded as it returns, :217 only reduces),
    ``mfl_amd.estimate_delta`` at :291-293 after :219.  delta after every
    round within DELTA_RTOL of the reference's own."""
    monkeypatch.setattr("mfl_amd.autostream.ClientFeed.SMALL_ROUND_BYTES", 0)  # stream even the small rounds
    case = fpf_replay.load_case(name)
    T, C = fresh_classes()
    mfl_amd.install(T, device=DEV, client_cls=C, stream_clients=True)
    rounds = []
    for t, rd in enumerate(case.meta["rounds"]):
        specs = []
        for j, n in enumerate(rd["sample_nums"]):
            def attempt(net, t=t, j=j, rd=rd):
                w = case.client_state(t, j, net.state_dict())
                return w, rd["losses"][j], rd["betas"][j], rd["rhos"][j], 0.5, 1
            specs.append((n, [attempt]))
        rounds.append(specs)
    rho0, beta0, delta0 = case.meta["stats_init"]
    state = {"st": (delta0, rho0, beta0, True, True)}
    got = []

    def after(r, w_locals, w_glob, trained):
        st = state["st"]
        if w_locals and trained:  # :289
            rd = case.meta["rounds"][r]
            delta = mfl_amd.estimate_delta(w_locals, w_glob, case.meta["lr"], device=DEV)  # :290-293
            # rho / beta (:296-305) from the loop's own per-client values
            st = O.round_stats_update(st, rd["sample_nums"], np.zeros(len(w_locals)), [t[2] for t in trained],
                                      [t[1] for t in trained], case.meta["lr"])
            st = ((delta if np.isfinite(delta) else state["st"][0]),) + tuple(st[1:])  # :294-295
            state["st"] = st
        got.append((st[1], st[2], st[0]))

    tr = T(OrderedDict((k, v.clone()) for k, v in case.init.items()), rounds,
           n_clients=case.meta["client_num_in_total"], after_aggregate=after)
    tr.train()
    feed = tr.__dict__["_mfl_feed"]
    nonempty = sum(1 for rd in case.meta["rounds"] if rd["sample_nums"])
    assert feed.stats["rounds_streamed"] == nonempty, feed.stats
    _check(name, np.array(got, dtype=np.float64), case, "installed_streaming")
