"""fedavg_collect_ext.verify_rows on CPU: the check a streamed round runs at
:217 (autostream.py) before it trusts the rows it packed while the loop went
on.  The staging rows here are packed by the product's host packer
(fedavg_pack_rows, csrc/fedavg_host.cpp), exactly as RoundSession.add packs
them; no GPU is involved."""
import copy
from collections import OrderedDict

import numpy as np
import pytest
import torch

import mfl_amd
from mfl_amd.layout import _PACK_KIND, KeyTable, _collect_ext

ext = _collect_ext()
pytestmark = pytest.mark.skipif(ext is None or not hasattr(ext, "verify_rows"), reason="collect ext not built")


def _clients(K, n_keys, numel, seed=0, int_key=True):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(K):
        sd = OrderedDict()
        for j in range(n_keys):
            sd[f"layer{j}.weight"] = torch.randn(numel if j % 3 else max(1, numel // 7), generator=g)
        if int_key:
            sd["bn.num_batches_tracked"] = torch.tensor(1000 + i, dtype=torch.int64)
        sd["h"] = torch.randn(5, generator=g, dtype=torch.float64)
        out.append(sd)
    return out


class Round:
    """A packed round: staging rows + the arrays verify_rows takes."""

    def __init__(self, dicts, counts):
        self.table = t = KeyTable(dicts[0])
        self.stage = {g.dtype: torch.zeros((len(dicts), g.ld), dtype=g.dtype) for g in t.groups.values()}
        ptrs, _ = t.collect(dicts)
        lib = mfl_amd._lib.load()
        for g in t.groups.values():
            items = t.pack_items(g, ptrs, 0, g.ld)
            st = self.stage[g.dtype]
            mfl_amd._lib.check(lib.fedavg_pack_rows(items.ctypes.data, items.shape[0], st.data_ptr(), st.element_size(),
                                                    2), "fedavg_pack_rows")
        gidx = {dt: k for k, dt in enumerate(t.groups)}
        st = [self.stage[dt] for dt in t.groups]
        self.args = ([e.name for e in t.entries],
                     [torch.empty(e.shape, dtype=e.src_dtype, device="meta") for e in t.entries],
                     [gidx[e.dtype] for e in t.entries], [int(e.offset) for e in t.entries],
                     [0 if e.src_dtype == e.dtype else _PACK_KIND[e.src_dtype] for e in t.entries],
                     [x.data_ptr() for x in st], [int(x.stride(0)) for x in st], [x.element_size() for x in st])
        self.counts = list(counts)

    def verify(self, w_locals, seed=1, probes=4096, full_elems=0, expect_version=-1, fed_keys=None, copies=None):
        return ext.verify_rows(w_locals, self.counts, *self.args, probes, seed, full_elems, expect_version, fed_keys,
                               copies)


def _round(K=8, n_keys=40, numel=40_000, **kw):
    dicts = _clients(K, n_keys, numel, **kw)
    counts = [10 * (i + 1) for i in range(K)]
    r = Round(dicts, counts)
    return r, [(n, copy.deepcopy(d)) for n, d in zip(counts, dicts)]  # :199's deep copies


def test_fed_round_passes():
    r, wl = _round()
    st = r.verify(wl)
    assert st[0] == 0 and st[3] > 0
    assert r.verify(wl, full_elems=1 << 30)[0] == 0  # full comparison: every element


@pytest.mark.parametrize("edit,status", [
    ("count", 1), ("sample_number", 2), ("not_a_pair", 3), ("alias", 4), ("key_order", 5), ("extra_key", 5),
    ("missing_key", 5), ("dtype", 6), ("shape", 6), ("noncontig", 6)])
def test_structural_mismatches(edit, status):
    r, wl = _round(K=4, n_keys=6, numel=1000)
    if edit == "count":
        wl.append(wl[-1])
    elif edit == "sample_number":
        wl[2] = (wl[2][0] + 1, wl[2][1])
    elif edit == "not_a_pair":
        wl[1] = list(wl[1])
    elif edit == "alias":
        wl[3] = (wl[3][0], wl[1][1])
    elif edit == "key_order":  # another insertion order (the packed row followed the table's)
        d = wl[2][1]
        wl[2] = (wl[2][0], OrderedDict(reversed(list(d.items()))))
    elif edit == "extra_key":
        wl[0][1]["extra"] = torch.zeros(1)
    elif edit == "missing_key":
        del wl[1][1]["h"]
    elif edit == "dtype":
        wl[1][1]["layer2.weight"] = wl[1][1]["layer2.weight"].double()
    elif edit == "shape":
        wl[1][1]["layer2.weight"] = wl[1][1]["layer2.weight"][:-1].clone()
    elif edit == "noncontig":
        t = wl[1][1]["layer2.weight"]
        wl[1][1]["layer2.weight"] = torch.stack([t, t], 1)[:, 0]
    assert r.verify(wl)[0] == status


def test_same_key_set_reordered_in_place_passes():
    """OrderedDict.move_to_end keeps the dict's own entry order: the key set and
    every value are unchanged, so the reduction is too (the result is written
    into client 0's dict key by key, its order untouched)."""
    r, wl = _round(K=4, n_keys=6, numel=1000)
    wl[0][1].move_to_end("layer0.weight")
    wl[2][1].move_to_end("h", last=False)
    assert r.verify(wl)[0] == 0


def test_key_edited_in_every_client_is_always_caught():
    """A systematic edit (clipping / noise / quantisation of a key in every
    client) meets the probes of that key in every round: each key is probed
    at least at one client per round."""
    r, wl = _round(K=64, n_keys=120, numel=20_000)  # 7,680 pairs > 4,096 probes: sampled mode
    for _, sd in wl:
        sd["layer77.weight"].mul_(0.9)
    for seed in range(20):
        st = r.verify(wl, seed=seed)
        assert st[0] == 7 and st[2] == list(wl[0][1]).index("layer77.weight"), st


def test_every_pair_probed_while_pairs_fit_the_budget():
    """K x keys <= probes: every (client, key) pair is probed every round, so a
    whole-key edit of ONE client is always caught."""
    r, wl = _round(K=8, n_keys=40, numel=40_000)
    wl[5][1]["layer13.weight"].add_(1e-3)
    assert all(r.verify(wl, seed=s)[0] == 7 for s in range(20))


def test_single_element_edit_is_found_at_the_sampling_rate():
    """One changed element is found with probability ~ (probes at that pair) /
    numel per round, from fresh positions every round -- small keys are
    covered densely, a fixed pattern never blinds a position."""
    r, wl = _round(K=8, n_keys=40, numel=40_000)
    key = "layer3.weight"  # j % 3 == 0: 40_000 // 7 = 5,714 elements
    wl[2][1][key][17] += 1.0
    hits = sum(r.verify(wl, seed=s)[0] == 7 for s in range(3000))
    # every pair probed (320 pairs <= 4,096), 2 positions each: p = 2 / 5,714
    assert 0 < hits < 15, hits
    r2, wl2 = _round(K=4, n_keys=6, numel=21)  # keys of 21 and 3 elements
    wl2[1][1]["layer1.weight"][4] += 1.0
    hits = sum(r2.verify(wl2, seed=s)[0] == 7 for s in range(300))
    assert 10 < hits < 60, hits  # p = 1 - (20/21)^2 ~ 0.093
    assert r2.verify(wl2, full_elems=1 << 20)[0] == 7  # small rounds are compared in full


def test_int_keys_compare_as_the_packer_converts():
    """int64 buffers are staged as fp32 (static_cast, fedavg_host.cpp): values
    that round to the same fp32 reduce to the same bits and pass; a change
    that alters the fp32 value is caught."""
    r, wl = _round(K=4, n_keys=3, numel=100)
    name = "bn.num_batches_tracked"
    base = int(wl[2][1][name])
    assert r.verify(wl, full_elems=1 << 20)[0] == 0
    wl[2][1][name].fill_(base + 1)
    st = r.verify(wl, full_elems=1 << 20)
    assert st[0] == 7 and st[1] == 2
    # 2^24 + 1 and 2^24 are one fp32 value: the packed row cannot tell them apart, nor can the reduction
    dicts = _clients(2, 2, 10)
    dicts[1][name].fill_(1 << 24)
    r3 = Round(dicts, [1, 2])
    wl3 = [(1, copy.deepcopy(dicts[0])), (2, copy.deepcopy(dicts[1]))]
    wl3[1][1][name].fill_((1 << 24) + 1)
    assert r3.verify(wl3, full_elems=1 << 20)[0] == 0


def test_verify_cost_scales_with_the_walk_not_the_model():
    """The resnet56 x 100 layout (350 keys, 35,000 tensors): one call walks
    every tensor's metadata and probes ~9,000 values (the streaming :217 budget)."""
    import sys
    import time
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "scripts"))
    from model_shapes import CONFIGS

    K, shapes = CONFIGS["resnet56"]
    g = torch.Generator().manual_seed(0)
    dicts = [OrderedDict((k, torch.tensor(i, dtype=torch.int64) if k.endswith("num_batches_tracked")
                          else torch.randn(s, generator=g)) for k, s in shapes) for i in range(K)]
    r = Round(dicts, list(range(1, K + 1)))
    wl = [(n, copy.deepcopy(d)) for n, d in zip(r.counts, dicts)]
    ts = []
    for s in range(5):
        t0 = time.perf_counter()
        st = r.verify(wl, seed=s)
        ts.append(time.perf_counter() - t0)
        assert st[0] == 0
    assert st[3] >= 2 * 4096 * 0.9
    assert float(np.median(ts)) < 0.05  # generous on a shared CPU; ~1 ms on 8 cores


def _dc_version():
    return int(copy.deepcopy(torch.zeros(1))._version)


@pytest.mark.parametrize("op", ["add_", "clamp_", "mul_", "copy_", "setitem", "replace", "zero_size_key"])
def test_in_place_edit_is_caught_every_round_by_the_version_counter(op):
    """One element of one client edited in place at a position the probes do
    not sample (sampled mode: 64 x 121 pairs > 4,096 probes), or the tensor
    object replaced: the version counter differs from a fresh deep copy's
    (:199), so the check fails for every seed -- deterministic, unlike the
    value probes (test_single_element_edit_is_found_at_the_sampling_rate)."""
    r, wl = _round(K=64, n_keys=120, numel=20_000)
    v = _dc_version()
    assert all(r.verify(wl, seed=s, expect_version=v)[0] == 0 for s in range(5))
    sd = wl[37][1]
    key = "layer50.weight"
    t = sd[key]
    if op == "add_":
        t[12_345:12_346].add_(1e-7)
    elif op == "clamp_":
        t.clamp_(-1e9, 1e9)  # changes no value at all: still an in-place op on the deep copy
    elif op == "mul_":
        t.mul_(1.0)
    elif op == "copy_":
        t.copy_(t.clone())
    elif op == "setitem":
        t[9_999] = t[9_999] + 1
    elif op == "replace":
        sd[key] = t.clone()  # a fresh tensor object: version 0, not a deep copy's
    elif op == "zero_size_key":
        sd["h"].add_(0.0)
        key = "h"
    j = list(sd).index(key)
    for seed in range(20):
        st = r.verify(wl, seed=seed, expect_version=v)
        assert st[0] == 8 and st[1] == 37 and st[2] == j, (seed, st)
    # without the version expectation only the sampled values could see it
    assert r.verify(wl, seed=0)[0] in (0, 7)


def test_metadata_checked_at_every_pair_not_only_probed_ones():
    """A dtype or shape change at ONE (client, key) pair is found every round
    (advisor finding: metadata used to be read at the probed pairs only)."""
    r, wl = _round(K=64, n_keys=120, numel=2_000)
    wl[11][1]["layer80.weight"] = wl[11][1]["layer80.weight"].double()
    assert all(r.verify(wl, seed=s)[0] == 6 for s in range(20))
    r, wl = _round(K=64, n_keys=120, numel=2_000)
    wl[50][1]["layer81.weight"] = wl[50][1]["layer81.weight"][:-1].clone()
    assert all(r.verify(wl, seed=s)[0] == 6 for s in range(20))


class _HashTwin(str):
    """A str subclass whose hash collides with a table name's but whose text differs."""

    def __hash__(self):
        return hash(self.target)


def test_key_with_a_colliding_hash_is_not_taken_for_the_name():
    """The fast walk matches keys by the hash in the dict's entry table and then
    compares the strings (advisor finding: a same-hash key used to pass)."""
    r, wl = _round(K=4, n_keys=6, numel=100)
    sd = wl[2][1]
    items = list(sd.items())
    twin = _HashTwin("layer9.weight")
    twin.target = items[3][0]
    items[3] = (twin, items[3][1])
    wl[2] = (wl[2][0], OrderedDict(items))
    assert r.verify(wl)[0] == 5


def test_version_walk_cost_resnet56():
    """Every tensor's version counter read (35,000 of them) stays within the
    walk's budget: the :217 check overlaps the GPU work of the finish."""
    import sys
    import time
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "scripts"))
    from model_shapes import CONFIGS

    K, shapes = CONFIGS["resnet56"]
    g = torch.Generator().manual_seed(0)
    dicts = [OrderedDict((k, torch.tensor(i, dtype=torch.int64) if k.endswith("num_batches_tracked")
                          else torch.randn(s, generator=g)) for k, s in shapes) for i in range(K)]
    r = Round(dicts, list(range(1, K + 1)))
    wl = [(n, copy.deepcopy(d)) for n, d in zip(r.counts, dicts)]
    v = _dc_version()
    ts = []
    for s in range(5):
        t0 = time.perf_counter()
        st = r.verify(wl, seed=s, expect_version=v)
        ts.append(time.perf_counter() - t0)
        assert st[0] == 0, st
    assert float(np.median(ts)) < 0.05


def test_fed_key_objects_match_by_identity():
    """fed_keys (autostream: the key objects of each fed dict, which the :199
    deep copy shares) short-cut the string compare; an equal key that is not
    the fed object is still compared, and a hash twin still fails."""
    r, wl = _round(K=4, n_keys=6, numel=100)
    fed = [tuple(sd) for _, sd in wl]
    assert r.verify(wl, fed_keys=fed)[0] == 0
    fresh = [tuple("".join(list(k)) for k in sd) for _, sd in wl]  # equal strings, other objects
    assert r.verify(wl, fed_keys=fresh)[0] == 0
    sd = wl[2][1]
    items = list(sd.items())
    twin = _HashTwin("layer9.weight")
    twin.target = items[3][0]
    items[3] = (twin, items[3][1])
    wl[2] = (wl[2][0], OrderedDict(items))
    assert r.verify(wl, fed_keys=fed)[0] == 5
    with pytest.raises(ValueError):
        r.verify(wl, fed_keys=fed[:2])


def test_copies_identity_catches_a_replacement_by_a_deep_copy():
    """``copies[i]``: the values of the loop's :199 deep copy of client i.  A
    value that is not that object -- here one key replaced by a deep copy
    with equal values and a deep copy's version counter -- is status 10 at
    (client, key); None entries skip the check; a tuple of the wrong length
    is status 10 with key -1."""
    r, wl = _round(K=5, n_keys=6, numel=1000)
    copies = [tuple(d.values()) for _, d in wl]
    assert r.verify(wl, copies=copies)[0] == 0
    n, d = wl[3]
    d2 = OrderedDict(d)
    k = list(d2)[4]
    d2[k] = copy.deepcopy(d2[k])  # same values, version counter of a deep copy
    wl[3] = (n, d2)
    assert r.verify(wl, expect_version=1)[0] == 0  # counters and values cannot see it
    st = r.verify(wl, expect_version=1, copies=copies)
    assert (st[0], st[1], st[2]) == (10, 3, 4)
    copies[3] = None
    assert r.verify(wl, expect_version=1, copies=copies)[0] == 0
    copies[3] = copies[2][:2]
    assert r.verify(wl, copies=copies)[:3] == (10, 3, -1)
