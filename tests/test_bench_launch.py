"""bench.py's multi-rank machinery on CPU (no GPU here):

* ``python bench.py --gpus N`` outside torch.distributed.run starts the N
  ranks itself (a child torch.distributed.run; the parent never touches the
  GPU) and relays rank 0's single JSON line and a failing rank's status;
* the strong/weak workload arithmetic and the pipeline depth rule;
* the parity machinery bench.py runs after its timed region -- sampled
  windows of the gathered model against the oracle on host-regenerated
  inputs, and the checksum-of-checksums of the reassembly -- at world size 2
  with gloo, including that a corrupted reassembly is caught.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from mfl_amd import synthetic  # noqa: E402
from mfl_amd.distributed import ShardedReducer  # noqa: E402


def _run_bench(*args, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=str(ROOT))


@pytest.mark.parametrize("n", [2, 3, 8])
def test_self_launch_starts_n_ranks_and_relays_one_json_line(n):
    r = _run_bench("--gpus", str(n), "--launch-check")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["world"] == n and out["rank_sum"] == out["expected"]


def test_self_launch_relays_a_failing_rank():
    r = _run_bench("--gpus", "2", "--launch-check", "--fail-rank", "1")
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_single_gpu_does_not_self_launch():
    assert bench.self_launch(["--gpus", "1"]) is None


def test_no_self_launch_under_torchrun(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.self_launch(["--gpus", "2"]) is None  # already launched: run in-process


@pytest.mark.parametrize("K,P,world,expect", [
    (100, 25_000_000, 1, 1),          # N = 1: no exchange, one chunk
    (100, 25_000_000, 8, 2),          # target at 8 GPUs: 3.125M columns -> 2 x 1.56M (one group per CU)
    (100, 25_000_000, 4, 4),          # 6.25M -> 4 x 1.56M (5 x 1.25M would give 0.8 groups per CU)
    (100, 25_000_000, 2, 8),          # 12.5M -> 8 x 1.56M
    (500, 11_227_812, 8, 2),          # cfg4: 1.4M -> 2 x 702K (3-slice band, K >= 256)
    (1000, 100_000_000, 8, 8),        # cfg5: 12.5M -> 8 x 1.56M
    (10, 1_206_590, 8, 1),            # tiny shards are not split
    (20, 25_000_000, 8, 4),           # few clients: no band, the >= 700K rule (4 x 781K)
])
def test_auto_chunks(K, P, world, expect):
    shard = -(-P // world)
    c = bench.auto_chunks(K, shard, world, host_out=False)
    assert c == expect
    assert c == 1 or shard // c >= bench.MIN_CHUNK_COLS


def test_one_group_per_cu_bands():
    assert bench.one_group_per_cu(100, 1_562_560) and not bench.one_group_per_cu(100, 781_312)
    assert not bench.one_group_per_cu(63, 1_562_560)  # the 6-slice band starts at K = 64
    assert bench.one_group_per_cu(500, 760_000) and not bench.one_group_per_cu(100, 760_000)
    assert not bench.one_group_per_cu(100, 1_250_000)  # 0.8 groups per CU


def test_strong_and_weak_workloads():
    K, P, _ = bench.WORKLOADS["target"]
    assert (K, P) == (100, 25_000_000)
    assert bench.WORKLOADS["resnet18_gn"][:2] == (500, 11_227_812)
    assert bench.WORKLOADS["synthetic_1000x100m"][:2] == (1000, 100_000_000)
    # cfg5 at N = 1 exceeds one GPU's rows: P-chunked passes
    assert 4 * 1000 * 100_000_000 > bench.ROW_BUDGET_BYTES
    # ... but fits from 2 GPUs up
    assert 4 * 1000 * 50_000_000 <= bench.ROW_BUDGET_BYTES


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torch_loop_reduce(clients, weights, P, out):
    # test-local stand-in for the HIP kernel (client 0 first, mul then add)
    acc = clients[0, :P] * weights[0]
    for i in range(1, clients.shape[0]):
        acc = acc + clients[i, :P] * weights[i]
    out[:P].copy_(acc)


def _parity_worker(rank, ws, port, K, P, chunks, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        red = ShardedReducer(K, P, chunks=chunks, device="cpu", local_reduce=_torch_loop_reduce)
        synthetic.fill_rows(red.clients, red.plan.local_segments())
        import mfl_amd
        w = mfl_amd.sample_weights(synthetic.sample_counts(K))
        red.step(torch.tensor(np.array(w, np.float64).astype(np.float32)))
        par = bench.sampled_parity(red, w, n_windows=3, width=257)
        ok_sums = bench.reassembly_checksums(red, dist, torch.device("cpu"))
        # corrupt one column of another rank's part of the reassembled model
        other = (rank + 1) % ws
        from mfl_amd.distributed import plan_shards
        _, g, n = plan_shards(P, ws, other, chunks).local_segments()[-1]
        red.full[g + n - 1] += 1.0
        bad_sums = bench.reassembly_checksums(red, dist, torch.device("cpu"))
        q.put((rank, par["ok"], par.get("gathered_checked", False), ok_sums, bad_sums))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws,K,P,chunks", [(2, 5, 10_007, 3), (2, 12, 4_099, 1), (8, 4, 60_013, 3)])
def test_bench_parity_and_reassembly_checks_gloo(ws, K, P, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parity_worker, args=(r, ws, port, K, P, chunks, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, par_ok, gathered, ok_sums, bad_sums in res:
        assert par_ok and gathered, rank
        assert ok_sums, rank
        assert not bad_sums, rank  # the corrupted reassembly is caught on every rank


def test_sampled_parity_single_rank_and_passes():
    """World size 1 (no gather) and the P-chunked pass layout: every pass's
    output slice is checked against pass 0's columns."""
    import mfl_amd
    K, P = 7, 3_001
    red = ShardedReducer(K, P, chunks=1, device="cpu", local_reduce=_torch_loop_reduce)
    synthetic.fill_rows(red.clients, red.plan.local_segments())
    w = mfl_amd.sample_weights(synthetic.sample_counts(K))
    wt = torch.tensor(np.array(w, np.float64).astype(np.float32))
    red.pass_out = torch.empty(3 * red.plan.local_cols)
    for p in range(3):
        red.local_out = red.pass_out[p * red.plan.local_cols:(p + 1) * red.plan.local_cols]
        red.step(wt)
    par = bench.sampled_parity(red, w, passes=3, pass_cols=red.plan.local_cols, n_windows=2, width=100)
    assert par["ok"], par
    red.pass_out[red.plan.local_cols + 5] += 1.0  # pass 1, inside the first-column window
    par = bench.sampled_parity(red, w, passes=3, pass_cols=red.plan.local_cols, n_windows=2, width=100)
    assert not par["ok"]


def test_as_rank_plans_one_shard_of_a_larger_world():
    """bench.py --shard-of N: ShardedReducer(as_rank=(N, r)) owns exactly rank
    r's block-cyclic segments of the N-rank plan and never gathers."""
    from mfl_amd.distributed import plan_shards
    for P, N, chunks in [(25_000_000, 8, 4), (11_227_812, 8, 2), (7_001, 3, 2)]:
        for r in (0, N - 1):
            red = ShardedReducer(4, P, chunks=chunks, device="cpu", local_reduce=_torch_loop_reduce, as_rank=(N, r))
            assert not red.gather and red.full is None
            assert red.plan.local_segments() == plan_shards(P, N, r, chunks).local_segments()
    with pytest.raises(ValueError):
        ShardedReducer(4, 100, device="cpu", local_reduce=_torch_loop_reduce, as_rank=(2, 0), gather=True)


@pytest.mark.parametrize("n", [2, 8])
def test_cpu_rehearsal_line_has_chunk_sweep(n):
    """``bench.py --gpus N --cpu-rehearsal``: the whole N > 1 bench path on CPU
    with gloo (a torch stand-in for the kernel).  Rank 0's one JSON line
    carries the warm-up chunk sweep (the chosen depth is the fastest step of
    the candidates) and the parity checks of the gathered model -- the same
    line the driver's N-GPU run prints.  The CPU baseline is timed at N = 1
    only (the bench contract); the N-GPU line says so."""
    r = _run_bench("--gpus", str(n), "--cpu-rehearsal", "--steps", "2", "--warmup", "1", timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["value"] is None and "NOT a measurement" in out["rehearsal"]
    sweep = out["diagnostics"]["chunk_sweep"]
    ms = {int(c): v for c, v in sweep["step_ms"].items()}
    assert sweep["chosen"] == min(ms, key=ms.get) == out["config"]["chunks"]
    assert sweep["rule_choice"] in ms and len(ms) >= 2
    assert out["config"]["chunks_from"].startswith("warm-up step sweep")
    assert out["parity"]["ok"] and out["parity"]["ranks"] == n and out["parity"]["reassembly_checksums_ok"]
    cb = out["cpu_baseline"]
    assert cb["value"] is None and cb["n_gpus_in_run"] == n and "N = 1 only" in cb["note"]
    ns = out["north_star"]  # the bar, the quantity it is met on, and the step fraction beside it
    assert ns["bar"] == 0.70 and ns["met_on"] == "per_rank_kernel_frac"
    assert ns["per_rank_kernel_frac"] is None  # the rehearsal has no kernel timing
    assert ns["step_frac_of_node_hbm"] == out["step_frac_of_node_hbm"] and "exchange" in ns["why_step_differs"]


def test_north_star_block_carries_the_written_prediction():
    """At the target's N = 8 the block holds DESIGN.md section 7's prediction
    (profiles/r06/scale_prediction.json): the per-rank kernel above the bar,
    the step exchange-bound, its node-HBM fraction as a range below 0.70."""
    roof = {"frac": 0.851}
    ns = bench.north_star_block("target", 8, roof, 0.40, "strong", measured_world=8)
    assert ns["per_rank_kernel_meets_bar"] is True and ns["step_meets_bar"] is False
    pred = ns["prediction"]
    assert pred["bound"] == "exchange" and pred["per_rank_kernel_frac"] > 0.70
    lo, hi = pred["step_frac_of_node_hbm"]
    assert 0 < lo <= hi < 0.70
    assert pred["value_GBps"][0] <= pred["value_GBps"][1]
    assert "prediction" in bench.north_star_block("resnet18_gn", 4, roof, 0.8, "strong", 4)
    assert "prediction" not in bench.north_star_block("target", 8, roof, 0.4, "weak", 8)
    assert "note" in bench.north_star_block("target", 8, roof, 0.8, "strong", measured_world=1)


def test_cpu_rehearsal_one_rank_times_the_cpu_baseline():
    """At N = 1 rank 0 times the reference's CPU loop after the timed region:
    both layouts, the affinity-thread value and the value at the job's share."""
    r = _run_bench("--gpus", "1", "--cpu-rehearsal", "--steps", "2", "--warmup", "1", timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    cb = json.loads(lines[0])["cpu_baseline"]
    assert cb["value"] > 0 and cb["n_gpus_in_run"] == 1 and cb["value_at_share"] > 0
    assert {lay["layout"] for lay in cb["layouts"]} >= {"flat", "model-shaped (mnist_lr)"}


def test_chunk_candidates():
    # the target at N = 8: 1/2/4/8 chunks of rank 0's 3.125M columns, incl. the rule's 2
    assert bench.chunk_candidates(25_000_000, 8, 2) == [1, 2, 4, 8]
    # a tiny shard: only depths whose chunks keep >= SWEEP_MIN_BLOCK columns (and the rule's pick)
    assert bench.chunk_candidates(10_000, 8, 1) == [1]


def test_attach_traffic_exact_shape_then_ratio(tmp_path):
    """The PMC traffic of the launch shape when a summary holds it (N-GPU
    shard files may list several chunk geometries), else the kernel's PMC
    ratio applied and labelled as another geometry."""
    import types
    f = tmp_path / "t.json"
    f.write_text(json.dumps({"algorithmic_bytes_per_launch": 1000, "hbm_bytes_per_launch": 1010,
                             "traffic_over_algorithmic": 1.01,
                             "launches": [{"algorithmic_bytes_per_launch": 500, "hbm_bytes_per_launch": 501,
                                           "traffic_over_algorithmic": 1.002}]}))
    args = types.SimpleNamespace(traffic_json=str(f), shard_of=0, workload="none")
    for b, exp in ((1000, 1010), (500, 501)):
        rf = {"bytes_per_launch": b}
        bench.attach_traffic(rf, args, world=8)
        assert rf["traffic"] == exp and "this launch shape" in rf["traffic_source"]
    rf = {"bytes_per_launch": 2000}
    bench.attach_traffic(rf, args, world=8)
    assert rf["traffic"] == 2020 and "not this geometry" in rf["traffic_source"]
