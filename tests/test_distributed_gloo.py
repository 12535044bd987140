"""World-size-2 (and 3) tests of the P-sharded path on CPU with ``gloo``.

The HIP kernel cannot run here, so each rank's local reduction is a plain
torch loop defined in this file (the product path injects the HIP kernel);
what is under test is the shard plan, the block-cyclic chunk layout, the
strided host->shard load and the all-gather reassembly.  The reassembled
vector must equal the oracle's single-process result bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import fedavg_oracle as O
from mfl_amd.distributed import ShardedReducer, plan_shards


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torch_loop_reduce(clients, weights, P, out):
    # test-local stand-in for the HIP kernel (same order: client 0 first)
    acc = clients[0, :P] * weights[0]
    for i in range(1, clients.shape[0]):
        acc = acc + clients[i, :P] * weights[i]
    out[:P].copy_(acc)


def _worker(rank, ws, port, K, P, chunks, seed, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        rng = np.random.default_rng(seed)
        host = torch.from_numpy(rng.normal(0, 0.05, size=(K, P)).astype(np.float32))
        n = rng.integers(1, 1000, size=K)
        w = torch.tensor(np.array(O.sample_weights([int(v) for v in n]), np.float64).astype(np.float32))
        red = ShardedReducer(K, P, chunks=chunks, device="cpu", local_reduce=_torch_loop_reduce)
        red.load_from_host(host)
        full = red.step(w)
        expect = O.reduce_f32(host.numpy(), O.sample_weights([int(v) for v in n]))
        ok = full.numpy().tobytes() == expect.tobytes()
        red.full.zero_()
        red.gather_only()  # the exchange step alone reassembles the same model
        ok = ok and red.full[:P].numpy().tobytes() == expect.tobytes()
        q.put((rank, ok, red.plan.valid_local_cols()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws,K,P,chunks", [(2, 5, 1001, 1), (2, 7, 4096, 3), (3, 4, 777, 2), (2, 1, 65, 1),
                                            # the driver's 8-GPU shape: 8 ranks, uneven last block, 3 and 5 chunks
                                            (8, 5, 100_003, 3), (8, 3, 40_961, 5), (8, 2, 130, 1)])
def test_sharded_reduce_allgather_matches_oracle(ws, K, P, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, K, P, chunks, 11 + P, q)) for r in range(ws)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in results), results
    assert sum(n for _, _, n in results) == P  # every column owned exactly once


@pytest.mark.parametrize("P,ws,chunks", [(1, 2, 1), (100, 8, 1), (25_000_000, 8, 4), (11_227_812, 8, 2), (7850, 3, 5),
                                          (200_000_000, 8, 8), (50_000_000, 2, 8), (100_000_000, 4, 8)])
def test_shard_plan_partitions_columns(P, ws, chunks):
    owned = np.zeros(P, dtype=np.int32)
    for r in range(ws):
        plan = plan_shards(P, ws, r, chunks)
        assert plan.block % 64 == 0
        for lstart, gstart, n in plan.local_segments():
            assert lstart % 64 == 0 and lstart + n <= plan.local_cols
            owned[gstart:gstart + n] += 1
    assert (owned == 1).all()


def _worker_host_out(rank, ws, port, K, P, chunks, seed, q):
    """SURVEY §8e host-consumer alternative: every rank D2Hs its shard into a
    host output at global positions; no collective.  Ranks send their host
    buffers back and the test merges them (in production one shared mapping)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        rng = np.random.default_rng(seed)
        host = torch.from_numpy(rng.normal(0, 0.05, size=(K, P)).astype(np.float32))
        n = rng.integers(1, 1000, size=K)
        w = torch.tensor(np.array(O.sample_weights([int(v) for v in n]), np.float64).astype(np.float32))
        host_out = torch.full((P,), float("nan"))
        red = ShardedReducer(K, P, chunks=chunks, device="cpu", local_reduce=_torch_loop_reduce, host_out=host_out)
        assert not red.gather
        red.load_from_host(host)
        got = red.step(w)
        assert got.data_ptr() == host_out.data_ptr()
        q.put((rank, host_out.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws,K,P,chunks", [(2, 5, 1001, 1), (3, 4, 4099, 3), (8, 3, 50_001, 3)])
def test_sharded_reduce_host_out_matches_oracle(ws, K, P, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    seed = 23 + P
    procs = [ctx.Process(target=_worker_host_out, args=(r, ws, port, K, P, chunks, seed, q)) for r in range(ws)]
    for p in procs:
        p.start()
    parts = dict(q.get(timeout=240) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = np.full(P, np.nan, dtype=np.float32)
    for r in range(ws):
        for _, g, n in plan_shards(P, ws, r, chunks).local_segments():
            assert not np.isnan(parts[r][g:g + n]).any()
            merged[g:g + n] = parts[r][g:g + n]
    rng = np.random.default_rng(seed)
    host = rng.normal(0, 0.05, size=(K, P)).astype(np.float32)
    n = rng.integers(1, 1000, size=K)
    expect = O.reduce_f32(host, O.sample_weights([int(v) for v in n]))
    assert merged.tobytes() == expect.tobytes()
