"""Zero-edit streaming (mfl_amd.install wraps Client.train and the round loop)
on CPU: the feed/fallback decisions, with a stand-in aggregator that records
what the patched loop hands it.  The GPU runs of the same harness are in
test_gpu_autostream.py."""
import sys
from collections import OrderedDict

import pytest
import torch

import mfl_amd
from loop_replay import fresh_classes

AGG_MOD = sys.modules["mfl_amd.aggregate"]


class _FakeStaging:
    def __init__(self, K, ld, dtype):
        self.host = torch.zeros((K, ld), dtype=dtype)  # the pinned rows' stand-in


class _FakeSession:
    """A RoundSession stand-in: the real key table and host packer
    (fedavg_pack_rows runs on the CPU), no GPU -- so the feed's native
    verification (verify_rows) compares w_locals against real packed rows."""

    def __init__(self, template, max_clients):
        from mfl_amd.layout import KeyTable

        self.keys = list(template.keys())
        self.max_clients = max_clients
        self.counts, self.dicts = [], []
        self._finished = False
        self.verified = None
        self.keep_dicts = True
        self.table = KeyTable(template)
        self._staging = {g.dtype: _FakeStaging(max_clients, g.ld, g.dtype) for g in self.table.groups.values()}

    def add(self, n, sd):
        assert list(sd.keys()) == self.keys
        ptrs, _ = self.table.collect([sd])
        lib = mfl_amd._lib.load()
        for g in self.table.groups.values():
            st = self._staging[g.dtype]
            items = self.table.pack_items(g, ptrs, len(self.counts), g.ld)
            mfl_amd._lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], st.host.data_ptr(),
                                                    st.host.element_size(), 1), "fedavg_pack_rows")
        self.counts.append(n)
        self.dicts.append(sd)

    def finish(self, w_locals, verify=None):
        self._finished = True
        assert [n for n, _ in w_locals] == self.counts
        self.verified = verify()
        if not self.verified:
            return None
        out = w_locals[0][1]
        out["__streamed__"] = torch.tensor(len(self.counts))
        return out

    def abandon(self):
        self._finished = True


class _FakeAgg:
    def __init__(self):
        self.sessions = []

    def begin_round(self, template, max_clients):
        s = _FakeSession(template, max_clients)
        self.sessions.append(s)
        return s


def _rounds(n_rounds=2, K=4, P=10, fail_first=()):
    g = torch.Generator().manual_seed(0)
    rounds = []
    for r in range(n_rounds):
        specs = []
        for i in range(K):
            sd = OrderedDict(w=torch.randn(P, generator=g), b=torch.randn(3, generator=g),
                             nbt=torch.tensor(7 + i, dtype=torch.int64))
            attempts = [None, sd] if i in fail_first else [sd]
            specs.append((10 * (i + 1) + r, attempts))
        rounds.append(specs)
    return rounds


@pytest.fixture
def plain_calls(monkeypatch):
    calls = []

    def fake_plain(w_locals, model_global=None, device=None, devices=None):
        calls.append([n for n, _ in w_locals])
        out = w_locals[0][1]
        out["__plain__"] = torch.tensor(1)
        return out

    monkeypatch.setattr(AGG_MOD, "aggregate", fake_plain)
    return calls


def _run(rounds, after_append=None, stream=None, small_round_bytes=0):
    T, C = fresh_classes()
    mfl_amd.install(T, stream_clients=stream)
    tr = T({"w": torch.zeros(10)}, rounds, after_append=after_append)
    agg = _FakeAgg()
    from mfl_amd.autostream import ClientFeed

    feed = ClientFeed(lambda: agg, len(tr.client_list))
    feed.SMALL_ROUND_BYTES = small_round_bytes  # the toy dicts here are tiny: stream them anyway
    tr.__dict__["_mfl_feed"] = feed
    tr.train()
    return tr, agg


def test_every_round_streams(plain_calls):
    rounds = _rounds(3, fail_first=(1,))  # client 1 diverges once and is retried (:181-195)
    tr, agg = _run(rounds)
    assert plain_calls == []
    assert len(agg.sessions) == 3
    for r, s in enumerate(agg.sessions):
        assert s.counts == [n for n, _ in rounds[r]] and s.verified
        assert s.max_clients == 4
    assert all("__streamed__" in res for res in tr.results)
    feed = tr.__dict__["_mfl_feed"]
    assert feed.stats["rounds_streamed"] == 3 and feed._worker is None  # the loop's end stopped the worker


def test_small_round_left_to_plain_path(plain_calls):
    # K x row bytes <= SMALL_ROUND_BYTES: the plain drop-in's one native call wins
    rounds = _rounds(2, K=4, P=10)
    row = 4 * (10 + 3 + 1)
    tr, agg = _run(rounds, small_round_bytes=4 * row)
    assert agg.sessions == [] and len(plain_calls) == 2
    assert all("__plain__" in res for res in tr.results)
    feed = tr.__dict__["_mfl_feed"]
    assert feed.stats["rounds_small"] == 2 and feed.stats["rounds_fallback"] == 0
    assert feed._worker is None  # never started
    tr, agg = _run(_rounds(1, K=4, P=10), small_round_bytes=4 * row - 1)
    assert len(agg.sessions) == 1 and "__streamed__" in tr.results[0]


@pytest.mark.parametrize("key,pos", [("w", 0), ("w", 7), ("b", 2), ("nbt", None)])
def test_sampled_value_change_falls_back(plain_calls, key, pos):
    # a small round (<= VERIFY_FULL_ELEMS) is compared element by element:
    # any edit of any key, int64 buffers included, is seen
    def mutate(r, w_locals):
        if r == 1:
            t = w_locals[2][1][key]
            if pos is None:
                t += 1
            else:
                t[pos] += 1.0

    tr, agg = _run(_rounds(2), after_append=mutate)
    assert "__streamed__" in tr.results[0] and "__plain__" in tr.results[1]
    assert agg.sessions[1].verified is False
    assert len(plain_calls) == 1


def test_extra_client_falls_back(plain_calls):
    def extra(r, w_locals):
        if r == 0:
            w_locals.append(w_locals[-1])

    tr, agg = _run(_rounds(2), after_append=extra)
    assert "__plain__" in tr.results[0] and "__streamed__" in tr.results[1]
    assert agg.sessions[0]._finished  # abandoned: the staging is free for the plain path


def test_sample_number_change_falls_back(plain_calls):
    def renumber(r, w_locals):
        w_locals[0] = (w_locals[0][0] + 1, w_locals[0][1])

    tr, _ = _run(_rounds(1), after_append=renumber)
    assert "__plain__" in tr.results[0]


def test_key_set_change_falls_back(plain_calls):
    def drop(r, w_locals):
        del w_locals[1][1]["b"]

    tr, _ = _run(_rounds(1), after_append=drop)
    assert "__plain__" in tr.results[0]


def test_streaming_off(plain_calls, monkeypatch):
    monkeypatch.setenv("FEDAVG_STREAM_CLIENTS", "0")
    T, C = fresh_classes()
    mfl_amd.install(T)
    assert not getattr(T.train, "__mfl_stream__", False)
    tr = T({"w": torch.zeros(10)}, _rounds(1))
    tr.train()
    assert "__plain__" in tr.results[0]


def test_valid_train_result_mirrors_reference_check():
    from mfl_amd.autostream import valid_train_result

    assert valid_train_result(({}, 0.1, 0.2, 0.3, 0.4, 1.0))
    assert valid_train_result(({}, 0.0, 0.0, 0.0, 0.0, None))  # cycles are not part of :190
    for i in range(1, 5):
        r = [{}, 0.1, 0.2, 0.3, 0.4, 1.0]
        r[i] = None
        assert not valid_train_result(tuple(r))
    assert not valid_train_result(None)


def test_client_subclass_overriding_train_is_not_streamed(plain_calls):
    """A Client subclass whose train() edits what the wrapped reference
    method returned (clipping, noise, ...): the feed saw the pre-edit dict,
    so the round must not be streamed."""
    T, C = fresh_classes()

    class Clipping(C):
        def train(self, *a, **k):
            res = super().train(*a, **k)
            if res[1] is not None:
                for v in res[0].values():
                    if v.is_floating_point():
                        v.clamp_(-0.5, 0.5)
            return res

    T.client_cls = Clipping
    mfl_amd.install(T, client_cls=C)
    tr = T({"w": torch.zeros(10)}, _rounds(2))
    agg = _FakeAgg()
    from mfl_amd.autostream import ClientFeed

    feed = ClientFeed(lambda: agg, len(tr.client_list))
    feed.SMALL_ROUND_BYTES = 0
    tr.__dict__["_mfl_feed"] = feed
    tr.train()
    assert agg.sessions == [] and len(plain_calls) == 2
    assert feed.stats["rounds_fallback"] == 2 and "overridden" in feed.stats["last_fallback"]


def test_reinstall_with_streaming_off_stops_the_feed(plain_calls):
    T, C = fresh_classes()
    mfl_amd.install(T, stream_clients=True)
    mfl_amd.install(T, stream_clients=False)  # the wrappers stay, but read the class's setting
    tr = T({"w": torch.zeros(10)}, _rounds(2))
    tr.train()
    assert "_mfl_feed" not in tr.__dict__ and len(plain_calls) == 2
    mfl_amd.install(T, stream_clients=True)  # and on again
    agg = _FakeAgg()
    from mfl_amd.autostream import ClientFeed

    feed = ClientFeed(lambda: agg, len(tr.client_list))
    feed.SMALL_ROUND_BYTES = 0
    tr.__dict__["_mfl_feed"] = feed
    tr.results.clear()
    tr.train()
    assert feed.stats["rounds_streamed"] == 2


def test_tensor_changed_while_packed_breaks_the_round(plain_calls):
    """The feed records each fed tensor's version counter on the loop's
    thread; an in-place update before the worker packed it (a Client.train
    whose tensors the next client's training updates) fails the round."""
    import threading

    from mfl_amd.autostream import ClientFeed

    gate = threading.Event()
    agg = _FakeAgg()

    def slow_agg():
        gate.wait(10)
        return agg

    feed = ClientFeed(slow_agg, 4)
    feed.SMALL_ROUND_BYTES = 0
    sd = OrderedDict(w=torch.arange(10.0), b=torch.zeros(3))
    feed.feed(5, sd)
    sd["w"].add_(1.0)  # in place, after train() returned, before the worker packed it
    gate.set()
    w_locals = [(5, OrderedDict((k, v.clone()) for k, v in sd.items()))]
    assert feed.take(w_locals) is None
    assert "changed while they were packed" in feed.stats["last_fallback"]
    feed.close()


@pytest.mark.parametrize("seed", range(20))
def test_single_in_place_edit_falls_back_every_time(plain_calls, seed):
    """A round large enough for sampled value checks (64 clients x 130 keys >
    4,096 probes): one element of one client edited in place between :199
    and :217, at a seed-chosen position, falls back deterministically -- the
    edited tensor's version counter is no longer a fresh deep copy's."""
    g = torch.Generator().manual_seed(seed)
    K, n_keys = 64, 130
    specs = []
    for i in range(K):
        sd = OrderedDict((f"k{j}", torch.randn(300, generator=g)) for j in range(n_keys))
        specs.append((i + 1, [sd]))
    rounds = [specs, specs]
    where = torch.randint(0, K, (1,), generator=g).item(), torch.randint(0, n_keys, (1,), generator=g).item()
    pos = torch.randint(0, 300, (1,), generator=g).item()

    def edit(r, w_locals):
        if r == 1:
            w_locals[where[0]][1][f"k{where[1]}"][pos] += 1e-6

    T, C = fresh_classes()
    mfl_amd.install(T, stream_clients=True)
    tr = T({"k0": torch.zeros(300)}, rounds, after_append=edit)
    agg = _FakeAgg()
    from mfl_amd.autostream import ClientFeed

    feed = ClientFeed(lambda: agg, K)
    feed.SMALL_ROUND_BYTES = 0
    feed.VERIFY_FULL_ELEMS = 0  # sampled values: the version counter alone must catch it
    tr.__dict__["_mfl_feed"] = feed
    tr.train()
    assert "__streamed__" in tr.results[0] and "__plain__" in tr.results[1]
    assert feed.stats["last_verify"]["status"] == 8
    assert (feed.stats["last_verify"]["client"], feed.stats["last_verify"]["key"]) == where


@pytest.mark.parametrize("which", ["middle", "last"])
def test_fed_dict_edited_before_its_deep_copy_falls_back(plain_calls, which):
    """A Client.train result edited in place AFTER the worker packed it and
    BEFORE the loop's :199 deep copy: w_locals then holds the edited values
    under fresh deep-copy counters, so only the fed dict itself shows the
    edit.  The worker re-reads the last packed dict's counters when the next
    client arrives (a middle client: the feed breaks) and :217 re-reads the
    round's last one (verify status 9)."""
    K = 6
    g = torch.Generator().manual_seed(3)
    specs = [(i + 1, [OrderedDict((f"k{j}", torch.randn(200, generator=g)) for j in range(4))]) for i in range(K)]
    rounds = [specs, specs]
    target = 2 if which == "middle" else K - 1
    feeds = []

    def edit(r, idx, w):
        if r == 1 and idx == target:
            feeds[0]._drain()  # the worker has packed this client: the edit comes after
            w["k1"][7] += 1e-3

    T, C = fresh_classes()
    mfl_amd.install(T, stream_clients=True)
    tr = T({"k0": torch.zeros(200)}, rounds, before_append=edit)
    agg = _FakeAgg()
    from mfl_amd.autostream import ClientFeed

    feed = ClientFeed(lambda: agg, K)
    feed.SMALL_ROUND_BYTES = 0
    feeds.append(feed)
    tr.__dict__["_mfl_feed"] = feed
    tr.train()
    assert "__streamed__" in tr.results[0] and "__plain__" in tr.results[1]
    if which == "last":
        assert feed.stats["last_verify"]["status"] == 9
    else:
        assert "changed after they were packed" in feed.stats["last_fallback"]


@pytest.mark.parametrize("hooked", [True, False], ids=["ordered_dict", "plain_dict"])
@pytest.mark.parametrize("seed", range(6))
def test_tensor_replaced_by_a_deep_copy_falls_back(plain_calls, seed, hooked):
    """A w_locals tensor REPLACED between :199 and :217 by another deep copy
    (``w_locals[i] = (n, copy.deepcopy(edited))``, one element changed at an
    unsampled-in-general position): its version counter is a deep copy's and
    its keys are the same objects, so counters cannot see it.  For the
    reference's OrderedDict state_dicts the feed recorded the loop's own :199
    deep copies (autostream._hook_deepcopy) and verify_rows requires identity
    with them: a deterministic fallback (status 10) every time.  A plain
    ``dict`` result carries no hook; there only the ~4,096 value probes can
    see it, so the streamed result is returned unless a probe lands on the
    element (this round has 64 x 130 x 300 elements: it rarely does)."""
    import copy

    g = torch.Generator().manual_seed(100 + seed)
    K, n_keys = 64, 130
    specs = []
    for i in range(K):
        sd = OrderedDict((f"k{j}", torch.randn(300, generator=g)) for j in range(n_keys))
        if hooked:
            specs.append((i + 1, [sd]))
        else:  # Client.train returning a plain dict of fresh tensors
            specs.append((i + 1, [lambda net, sd=sd: (dict((k, v.clone()) for k, v in sd.items()),
                                                      0.25, 0.5, 0.75, 0.9, 100.0)]))
    rounds = [specs, specs]
    where = torch.randint(0, K, (1,), generator=g).item(), torch.randint(0, n_keys, (1,), generator=g).item()
    pos = torch.randint(0, 300, (1,), generator=g).item()

    def replace(r, w_locals):
        if r == 1:
            n, sd = w_locals[where[0]]
            edited = copy.deepcopy(sd)
            edited[f"k{where[1]}"][pos] += 1e-3
            w_locals[where[0]] = (n, copy.deepcopy(edited))  # fresh deep copies: version 1, same key objects

    T, C = fresh_classes()
    mfl_amd.install(T, stream_clients=True)
    tr = T({"k0": torch.zeros(300)}, rounds, after_append=replace)
    agg = _FakeAgg()
    from mfl_amd.autostream import ClientFeed

    feed = ClientFeed(lambda: agg, K)
    feed.SMALL_ROUND_BYTES = 0
    feed.VERIFY_FULL_ELEMS = 0
    tr.__dict__["_mfl_feed"] = feed
    tr.train()
    assert "__streamed__" in tr.results[0]
    if hooked:
        assert "__plain__" in tr.results[1]
        assert feed.stats["last_verify"]["status"] == 10
        assert feed.stats["last_verify"]["client"] == where[0] and feed.stats["last_verify"]["key"] == 0
    else:  # the documented limit: caught only when a value probe hits the edited element
        st = feed.stats["last_verify"]["status"]
        assert st in (0, 7)
        assert ("__plain__" in tr.results[1]) == (st == 7)


def test_deepcopy_hook_leaves_the_copy_unchanged():
    """The one-shot hook's deep copy is the plain one: same type, same
    ``_metadata`` attribute, no hook carried over; the hook is gone from the
    fed dict after it fired and a second deep copy is plain."""
    import copy

    from mfl_amd.autostream import ClientFeed

    sd = torch.nn.Linear(3, 2).state_dict()  # an OrderedDict with _metadata, as client.py:96 returns
    feed = ClientFeed(lambda: None, 4)
    feed.fed.append(1)
    feed._copies.append(None)
    feed._hook_deepcopy(sd, 0)
    assert "__deepcopy__" in sd.__dict__
    y = copy.deepcopy(sd)
    assert "__deepcopy__" not in sd.__dict__ and "__deepcopy__" not in y.__dict__
    assert type(y) is type(sd) and y._metadata == sd._metadata and list(y) == list(sd)
    assert all(torch.equal(a, b) and a is not b for a, b in zip(y.values(), sd.values()))
    assert feed._copies[0] is not None and all(a is b for a, b in zip(feed._copies[0], y.values()))
    y2 = copy.deepcopy(sd)
    assert all(a is not b for a, b in zip(y2.values(), y.values()))
    feed._reset()
    sd2 = torch.nn.Linear(3, 2).state_dict()
    feed.fed.append(1)
    feed._copies.append(None)
    feed._hook_deepcopy(sd2, 0)
    gen = feed._gen
    feed._reset()  # the round ended before the loop's deep copy: the hook records nothing
    assert feed._gen == gen + 1
    copy.deepcopy(sd2)
    assert feed._copies == []


def test_install_devices_streams_into_the_sharded_aggregator(plain_calls, monkeypatch):
    """install(devices=[...]): the feed's rounds open on the devices'
    ShardedAggregator (multi.ShardedRoundSession), not on the first device."""
    agg = _FakeAgg()
    asked = []

    def fake_sharded(devs):
        asked.append(list(devs))
        return agg

    monkeypatch.setattr("mfl_amd.multi.sharded_aggregator", fake_sharded)
    monkeypatch.setattr("mfl_amd.autostream.ClientFeed.SMALL_ROUND_BYTES", 0)
    monkeypatch.setenv("FEDAVG_STREAM_DISTINCT_DEVICES", "1")  # distinct devices stream only when opted in
    T, C = fresh_classes()
    mfl_amd.install(T, stream_clients=True, devices=[0, 1, 2])
    tr = T({"w": torch.zeros(10)}, _rounds(2))
    tr.train()
    assert asked and all(a == [0, 1, 2] for a in asked)
    assert len(agg.sessions) == 2 and all("__streamed__" in r for r in tr.results)
    assert plain_calls == []


def test_install_distinct_devices_do_not_stream_by_default(monkeypatch):
    """Streaming over distinct GPUs is opt-in (FEDAVG_STREAM_DISTINCT_DEVICES=1):
    without it install(devices=[0, 1]) keeps the wrappers off and :217 runs
    the plain sharded path; N shards on one device (the rehearsed form) stream."""
    from mfl_amd.aggregate import stream_distinct_ok

    monkeypatch.delenv("FEDAVG_STREAM_DISTINCT_DEVICES", raising=False)
    monkeypatch.setattr(mfl_amd.DeviceAggregator, "WARMUP", False)
    assert not stream_distinct_ok([0, 1]) and stream_distinct_ok([0, 0, 0]) and stream_distinct_ok(["cuda:2"])
    T, C = fresh_classes()
    mfl_amd.install(T, stream_clients=True, devices=[0, 1])
    assert T._mfl_stream_on is False and T._mfl_stream_devices == [0, 1]
    T2, C2 = fresh_classes()
    mfl_amd.install(T2, stream_clients=True, devices=[0, 0])
    assert T2._mfl_stream_on is True
    monkeypatch.setenv("FEDAVG_STREAM_DISTINCT_DEVICES", "1")
    assert stream_distinct_ok([0, 1])
