"""multi.ShardedAggregator's host logic on CPU: the column split and the
device-list routing (the GPU runs are tests/test_gpu_multi.py)."""
import pytest
import torch

import mfl_amd
from mfl_amd.multi import devices_from_env, shard_bounds


@pytest.mark.parametrize("P,n", [(25_000_000, 8), (600_372, 8), (7_850, 2), (1, 8), (64, 3), (1_000_003, 7)])
def test_shard_bounds_partition_aligned(P, n):
    b = shard_bounds(P, n)
    assert len(b) == n + 1 and b[0] == 0 and b[-1] == P
    assert all(b[i] <= b[i + 1] for i in range(n))  # contiguous, ordered, covering
    assert all(x % 64 == 0 for x in b[1:-1] if x < P)  # interior starts 256-B aligned
    widths = [b[i + 1] - b[i] for i in range(n)]
    if P >= 64 * n:
        assert max(widths) - min(widths) <= 128  # balanced to two alignment units


def test_shard_bounds_target():
    assert shard_bounds(25_000_000, 8)[1] == 3_125_056


def test_devices_from_env(monkeypatch):
    monkeypatch.delenv("FEDAVG_DEVICES", raising=False)
    assert devices_from_env() is None
    monkeypatch.setenv("FEDAVG_DEVICES", "0, 1,2,3")
    assert devices_from_env() == [torch.device("cuda", i) for i in range(4)]


def test_sharded_aggregator_refuses_cpu_devices():
    with pytest.raises(ValueError):
        mfl_amd.ShardedAggregator([torch.device("cpu")])


def test_single_entry_device_list_names_that_device(monkeypatch):
    """install(devices=[3]) / FEDAVG_DEVICES=3 run on cuda:3, not on the current device."""
    from mfl_amd.aggregate import _devices_arg, _single_device
    from loop_replay import fresh_classes

    monkeypatch.delenv("FEDAVG_DEVICES", raising=False)
    assert _devices_arg(None, [3]) is None and _single_device(None, [3]) == torch.device("cuda", 3)
    assert _single_device(torch.device("cuda", 1), [3]) == torch.device("cuda", 1)
    assert _single_device(None, None) is None
    monkeypatch.setenv("FEDAVG_DEVICES", "5")
    assert _single_device(None, None) == torch.device("cuda", 5)
    monkeypatch.delenv("FEDAVG_DEVICES")
    # install() warms the listed devices up eagerly when a GPU is visible; this
    # checks the routing only (a one-GPU box has no cuda:1 or cuda:3)
    monkeypatch.setattr(mfl_amd.DeviceAggregator, "WARMUP", False)
    T, C = fresh_classes()
    mfl_amd.install(T, client_cls=C, devices=[3])
    assert T._mfl_stream_device == torch.device("cuda", 3) and T._mfl_stream_devices is None
    T2, C2 = fresh_classes()
    mfl_amd.install(T2, client_cls=C2, devices=[0, 1])
    assert T2._mfl_stream_devices == [0, 1]


def test_normalize_device_forms():
    from mfl_amd.multi import normalize_device

    assert normalize_device(2) == torch.device("cuda", 2)
    assert normalize_device("cuda:4") == torch.device("cuda", 4)
    assert normalize_device(torch.device("cuda", 1)) == torch.device("cuda", 1)
    with pytest.raises(ValueError):
        normalize_device("cpu")
