"""GPU parity: libvmqgpu's HIP match path vs the CPU oracle, through the C ABI.

Bar: bit-exact — for every publish the sorted multiset of FoldFun entries
equals vmq_reg_trie:fold/4's (restated by the oracle).  Sizes the oracle
finishes in seconds are compared publish-for-publish; the full config C is
checked by size-independent properties plus an oracle sample."""
import numpy as np
import pytest

from oracle import feed
from oracle import oracle as O
from tests import harness as H
from tests import scenarios as S

pytestmark = pytest.mark.gpu

SCEN_FILES = ["pattern_matching.json", "upgrade.json", "overlapping_subscriptions.json",
              "dollar_topics.json", "shared_subscriptions.json", "quirks.json"]


# Both output modes of libvmqgpu: 16-B FoldFun records (vmqg_match_batch)
# and key ranges expanded on the host (vmqg_match_ranges + vmqg_records).
MODES = ["records", "ranges"]


def _driver(node, mode="records", **kw):
    return H.ProductDriver(node, device=0, mode=mode, **kw)


def _scen():
    for f in SCEN_FILES:
        for sc in S.load(f)["scenarios"]:
            yield pytest.param(sc, id="%s:%s" % (f, sc["name"]))


def test_native_library_is_the_in_tree_build():
    from vernemq_amd import _lib
    L = _lib.lib()
    assert L._name == _lib.LIB_PATH
    v = H.ProductDriver("n@h", device=0).view
    assert v.stats_raw()["device_bytes"] > 0


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("scen", list(_scen()))
def test_golden_scenarios_on_gpu(scen, mode):
    S.run_scenario(scen, lambda node: _driver(node, mode))


def _compare_batches(prod, orc, pubs, ctx=""):
    got = prod.fold_batch(pubs)   # (vmqg_match_batch checks status -> deferred counters in stats)
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in pubs])
    for i, (g, w) in enumerate(zip(got, want)):
        assert sorted(g) == sorted(w), "%s publish %r: got %r want %r" % (ctx, pubs[i], sorted(g)[:8], sorted(w)[:8])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", range(4))
def test_random_churn_fold_parity(seed, mode):
    wl = H.ChurnWorkload(seed, n_clients=60)
    prod = _driver(wl.self_node, mode)
    orc = O.TrieOracle(wl.self_node)
    for step in range(20):
        evs = [wl.event() for _ in range(25)]
        prod.apply(evs)
        orc.apply(evs)
        _compare_batches(prod, orc, wl.publishes(200), "seed %d batch %d" % (seed, step))


def _load_both(w, with_oracle=True):
    from vernemq_amd.reg_view import RegGpuView
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v)
    orc = None
    if with_oracle:
        orc = feed.load(w)
    return v, orc


def _match(v, pubs, words, mode="records", **kw):
    if mode == "ranges":
        rng, offs = v.match_ranges(pubs, words)
        return v.expand_ranges(rng, offs)
    return v.match_arrays(pubs, words, **kw)


def _gpu_canon(v, w, lo, hi, mode="records"):
    pubs, words = w.publish_arrays(v, lo, hi)
    recs, offs = _match(v, pubs, words, mode)
    return [sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
            for i in range(hi - lo)]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("cfg", ["A", "B"])
def test_config_full_parity(cfg, mode):
    from vernemq_amd import workloads as W
    w = W.CONFIGS[cfg]()
    v, orc = _load_both(w)
    n = w.n_pubs
    got = _gpu_canon(v, w, 0, n, mode)
    want = orc.fold_batch([(w.mps[w.pub_mp[i]], b"pub", w.pub_topic(i)) for i in range(n)])
    bad = [i for i in range(n) if got[i] != sorted(want[i])]
    assert not bad, "config %s: %d/%d publishes differ, first %r: got %r want %r" % (
        cfg, len(bad), n, w.pub_topic(bad[0]), got[bad[0]][:6], sorted(want[bad[0]])[:6])
    assert sum(len(x) for x in got) > n // 10   # the workload does match


@pytest.mark.parametrize("exfilter", [0, 1])
def test_exact_filter_modes_give_the_same_answers(exfilter):
    """The exbits filter only decides whether the exact table is probed:
    forced off and forced on, config A equals the oracle publish for publish
    (the default, auto, is what every other test runs)."""
    from vernemq_amd import workloads as W
    w = W.CONFIGS["A"]()
    v, orc = _load_both(w)
    v.set_option("exfilter", exfilter)
    n = w.n_pubs
    got = _gpu_canon(v, w, 0, n)
    want = orc.fold_batch([(w.mps[w.pub_mp[i]], b"pub", w.pub_topic(i)) for i in range(n)])
    bad = [i for i in range(n) if got[i] != sorted(want[i])]
    assert not bad, (len(bad), w.pub_topic(bad[0]))


@pytest.mark.parametrize("heavy_min", [2, 40])
def test_heavy_publishes_copied_by_xcd_write_the_same_bytes(heavy_min):
    """Heavy publishes (vmqg_set_option "heavy_min": >= that many records
    from <= 2 keys) are copied by the EMIT tail on the XCD their first key
    hashes to instead of by the fast EMIT: the output is byte-identical to
    heavy_min 0 and equal to the oracle (config A, records mode), with dedupe
    off and on (duplicates take their representative's bucket)."""
    from vernemq_amd import workloads as W
    w = W.CONFIGS["A"]()
    v, orc = _load_both(w)
    pubs, words = w.publish_arrays(v)
    outs = {}
    for hm, dd in ((0, 0), (heavy_min, 0), (0, 1), (heavy_min, 1)):
        v.set_option("heavy_min", hm)
        v.set_option("dedupe", dd)
        recs, offs = v.match_arrays(pubs, words)
        outs[hm, dd] = (np.asarray(offs).copy(), np.asarray(recs).view(np.uint8).copy())
    v.set_option("heavy_min", heavy_min)   # the oracle check below: heavy routing with dedupe on
    v.set_option("dedupe", 1)
    # byte-identical at the same dedupe setting (a deduped representative
    # walks four lanes wide, so its keys may come in another order than the
    # one-lane walk's: the same multiset, checked against the oracle below)
    for dd in (0, 1):
        a, b = outs[0, dd], outs[heavy_min, dd]
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), dd
    n = w.n_pubs
    got = _gpu_canon(v, w, 0, n)
    want = orc.fold_batch([(w.mps[w.pub_mp[i]], b"pub", w.pub_topic(i)) for i in range(n)])
    assert all(got[i] == sorted(want[i]) for i in range(n))
    assert int((np.diff(outs[0, 0][0].astype(np.int64)) >= heavy_min).sum()) > 100   # the path is exercised


def test_store_policies_write_the_same_records():
    """Both EMIT store policies (vmqg_set_option "nt_stores": non-temporal,
    the default, and plain) write the same bytes; the default is checked
    against the oracle by every other test."""
    from vernemq_amd import workloads as W
    w = W.CONFIGS["B"]()
    v, orc = _load_both(w)
    pubs, words = w.publish_arrays(v, 0, w.n_pubs)
    outs = []
    for sp in (1, 0):
        v.set_option("nt_stores", sp)
        recs, offs = v.match_arrays(pubs, words)
        outs.append((np.asarray(offs).copy(), np.asarray(recs).view(np.uint8).copy()))
    v.set_option("nt_stores", 1)
    assert np.array_equal(outs[1][0], outs[0][0]), "offsets differ under plain stores"
    assert np.array_equal(outs[1][1], outs[0][1]), "records differ under plain stores"
    assert int(outs[0][0][-1]) > w.n_pubs // 10


def test_config_c_full_size():
    """Config C at full size (1,000,064 subs, 2^20 publishes): every publish
    devices/{d}/telemetry/{m} emits the 64 wildcard subscribers plus c{d}
    when d < 10^6 — checked for all publishes; plus an oracle sample."""
    from vernemq_amd import workloads as W
    w = W.config_c()
    v, _ = _load_both(w, with_oracle=False)
    pubs, words = w.publish_arrays(v)
    recs, offs = v.match_arrays(pubs, words, out_cap=70 * w.n_pubs)
    d = w.pw[1::4] - 18
    hit = d < w.notes["n_dev"]
    counts = np.diff(offs.astype(np.int64))
    assert np.array_equal(counts, np.where(hit, 65, 64))
    kinds = recs["kind_node"] >> 24
    assert np.all(kinds == 1)
    # per publish: the multiset of subscriber ids
    sid_of = {c: i for i, c in enumerate(v.subscribers.terms)}
    wild = np.sort(np.array([sid_of[("", b"w%d" % i)] for i in range(64)], dtype=np.uint32))
    dev_sid = np.array([sid_of[("", b"c%d" % k)] for k in range(w.notes["n_dev"])], dtype=np.uint32)
    seg = np.repeat(np.arange(len(counts)), counts)
    order = np.lexsort((recs["subscriber"], seg))
    s_sorted = recs["subscriber"][order]
    starts = offs.astype(np.int64)
    for idx in np.linspace(0, len(counts) - 1, 2000).astype(np.int64):
        a = s_sorted[starts[idx]:starts[idx + 1]]
        want = wild if not hit[idx] else np.sort(np.append(wild, dev_sid[d[idx]]))
        assert np.array_equal(a, want), idx
    # every hit publish contains its own device subscriber exactly once
    own = np.zeros(len(counts), dtype=np.int64)
    subs_arr = recs["subscriber"].astype(np.int64)
    sid_to_dev = np.full(len(v.subscribers.terms), -1, dtype=np.int64)
    sid_to_dev[dev_sid] = np.arange(len(dev_sid))
    dev_of_rec = sid_to_dev[subs_arr]
    np.add.at(own, seg, (dev_of_rec == d[seg]).astype(np.int64))
    assert np.array_equal(own, hit.astype(np.int64))
    # oracle sample (4,096 publishes) on a 100k-device slice of the same shape
    ws = W.config_c(n_dev=100_000, n_pubs=4096)
    vs, orc = _load_both(ws)
    got = _gpu_canon(vs, ws, 0, ws.n_pubs)
    want = orc.fold_batch([("", b"pub", ws.pub_topic(i)) for i in range(ws.n_pubs)])
    assert all(g == sorted(x) for g, x in zip(got, want))
    # range mode on the full batch: 2 entries per hit publish (the wildcard
    # list + the device's own key), 1 per miss; expands to the same records
    rng, roffs = v.match_ranges(pubs, words, out_cap=2 * w.n_pubs)
    assert np.array_equal(np.diff(roffs.astype(np.int64)), np.where(hit, 2, 1))
    assert np.all(rng["count"] > 0)
    erec, eoffs = v.expand_ranges(rng, roffs)
    assert np.array_equal(eoffs, offs)
    for idx in np.linspace(0, len(counts) - 1, 500).astype(np.int64):
        a = np.sort(erec["subscriber"][offs[idx]:offs[idx + 1]])
        b = np.sort(recs["subscriber"][offs[idx]:offs[idx + 1]])
        assert np.array_equal(a, b), idx


def test_r1_r2_bench_shapes():
    """vmq_reg_trie_bench_SUITE.erl:137-146, :189-192, :209-211 at n = 100,000."""
    from vernemq_amd import workloads as W
    w = W.config_r1(100_000)
    v, _ = _load_both(w, with_oracle=False)
    pubs, words = w.publish_arrays(v)
    recs, offs = v.match_arrays(pubs, words)
    assert np.array_equal(np.diff(offs.astype(np.int64)), np.ones(w.n_pubs, dtype=np.int64))
    for i in (0, 1, 4242, w.n_pubs - 1):
        assert v.decode(recs[i]) == (("a", b"%d" % (i + 1)), 0)
    w2 = W.config_r2(100_000)
    v2, _ = _load_both(w2, with_oracle=False)
    em = v2.fold_batch([("a", (b"some", b"topic"))])[0]
    assert sorted(em) == sorted((("a", b"%d" % i), 0) for i in range(1, 100_001))
    v2.handle_events([("deleted", ("a", b"%d" % i), [(w2.self_node, True, [((b"some", b"topic"), 0)])])
                      for i in range(1, 100_001)])
    assert v2.fold_batch([("a", (b"some", b"topic"))])[0] == []
    st = v2.stats_raw()
    assert st["subs_objects"] == 0 and st["fanout_objects"] == 0


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("levels,tier", [(7, 1), (10, 2)])
def test_wide_frontier_deferred_tiers(levels, tier, mode):
    """2^levels filters over {x, +} at every level: the frontier / candidate
    lists overflow the fast tier's LDS lists, so a whole wave walks the
    publish, streaming candidates and keys through bounded LDS buffers;
    levels 7: its frontier stack fits LDS (tier 1); levels 10: the stack
    moves to global memory (tier 2)."""
    import itertools
    node = "n@h"
    prod = _driver(node, mode)
    prod.view.set_option("dedupe", 0)   # this test pins the deferral tiers' counters
    orc = O.TrieOracle(node)
    subs = []
    for i, combo in enumerate(itertools.product([b"x", b"+"], repeat=levels)):
        t = combo if i % 3 else combo[:levels - 1] + (b"#",)
        subs.append(("updated", ("", b"s%d" % i), None, [(node, True, [(t, i % 3)])]))
    prod.apply(subs)
    orc.apply(subs)
    pubs = [("", (b"x",) * levels), ("", (b"x", b"y") * (levels // 2) + (b"x",) * (levels % 2)),
            ("", (b"x",) * (levels - 1)), ("", (b"x",) * (levels + 1)), ("", (b"$x",) * levels)] + \
           [("", (b"q%d" % i,)) for i in range(40)]
    _compare_batches(prod, orc, pubs, "wide%d" % levels)
    st = prod.view.stats_raw()
    assert st["deferred_tier1"] >= 1
    assert (st["deferred_tier2"] >= 1) == (tier == 2)
    assert len(prod.fold(*pubs[0])) > 64


def test_frontier_2_16_is_answered():
    """A 2^16-wide frontier (16 levels of {x, +}: 65,536 filters all matching
    x^16) — vmq_reg_trie's trie_match/4 (:358-383) always answers; so must
    the product (the wave tier streams its candidates, the stack is sized
    from the trie depth)."""
    import itertools
    node = "n@h"
    prod = _driver(node)
    prod.view.set_option("dedupe", 0)   # this test pins the deferral tiers' counters
    orc = O.TrieOracle(node)
    subs = [("updated", ("", b"s%d" % i), None, [(node, True, [(combo, i % 3)])])
            for i, combo in enumerate(itertools.product([b"x", b"+"], repeat=16))]
    for lo in range(0, len(subs), 8192):
        prod.apply(subs[lo:lo + 8192])
        orc.apply(subs[lo:lo + 8192])
    pubs = [("", (b"x",) * 16), ("", (b"x", b"y") * 8), ("", (b"y",) * 16), ("", (b"x",) * 15)]
    _compare_batches(prod, orc, pubs, "2^16")
    assert len(prod.fold(*pubs[0])) == 1 << 16
    assert prod.view.stats_raw()["deferred_tier2"] >= 1


@pytest.mark.parametrize("mode", MODES)
def test_cluster_of_100_nodes(mode):
    """Remote subscriptions from 100 nodes (ids beyond the 64-bit inline
    masks): get_remote_subscribers/2 and the wildcard node lists
    (vmq_reg_trie.erl:503-520, :78-84) — each remote node once per publish,
    in any mix of exact and wildcard matches."""
    import random
    r = random.Random(100)
    nodes = ["n%d@h" % i for i in range(100)]
    node = nodes[0]
    prod = _driver(node, mode, nodes=nodes)
    orc = O.TrieOracle(node)
    filters = [(b"a", b"b"), (b"a", b"+"), (b"a", b"#"), (b"+", b"b"), (b"#",), (b"a", b"b", b"c"),
               (b"x", b"y"), (b"$share", b"g", b"a", b"+")]
    evs = []
    for i in range(400):
        n = r.choice(nodes)
        evs.append(("updated", ("", b"c%d" % i), None, [(n, True, [(r.choice(filters), r.randint(0, 2))])]))
    prod.apply(evs)
    orc.apply(evs)
    pubs = [("", t) for t in [(b"a", b"b"), (b"a", b"q"), (b"z", b"b"), (b"a", b"b", b"c"), (b"x", b"y"),
                              (b"q",), (b"$SYS", b"b")]]
    _compare_batches(prod, orc, pubs, "100 nodes")
    got = prod.fold("", (b"a", b"b"))
    remotes = [e for e in got if e[0] == "C"]
    assert len(remotes) == len(set(remotes)) > 64
    # deletes shrink the node lists again
    dels = [("deleted", ev[1], ev[3]) for ev in evs[::2]]
    prod.apply(dels)
    orc.apply(dels)
    _compare_batches(prod, orc, pubs, "100 nodes after deletes")


def test_match_status_errors_are_sticky():
    """An overflow in one of several pipelined vmqg_match_device calls is
    still reported by the vmqg_match_status after the last one."""
    import torch
    prod = _driver("n@h")
    v = prod.view
    v.handle_events([("updated", ("", b"c%d" % i), None, [("n@h", True, [((b"t",), 0)])]) for i in range(100)])
    pubs, words = v.prepare([("", (b"t",))] * 4)
    dev = torch.device("cuda:0")
    d_pubs = torch.from_numpy(pubs.view(np.uint32).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    d_out = torch.zeros(400 * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(5, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    v.match_device(d_pubs.data_ptr(), 4, d_words.data_ptr(), d_out.data_ptr(), 10, d_offs.data_ptr(), sp)   # overflows
    v.match_device(d_pubs.data_ptr(), 4, d_words.data_ptr(), d_out.data_ptr(), 400, d_offs.data_ptr(), sp)  # clean
    from vernemq_amd import _lib
    assert v.match_status(sp) == _lib.E_OVERFLOW
    v.match_device(d_pubs.data_ptr(), 4, d_words.data_ptr(), d_out.data_ptr(), 400, d_offs.data_ptr(), sp)
    assert v.match_status(sp) == 0
    assert int(d_offs[-1].item()) == 400


@pytest.mark.parametrize("mode", MODES)
def test_long_topics(mode):
    node = "n@h"
    prod = _driver(node, mode)
    orc = O.TrieOracle(node)
    long_t = tuple(b"w%d" % (i % 7) for i in range(150))
    evs = [("updated", ("", b"a"), None, [(node, True, [(long_t, 1), (long_t[:80] + (b"#",), 0),
                                                       ((b"+",) * 149 + (b"w2",), 2), ((b"#",), 0)])])]
    prod.apply(evs)
    orc.apply(evs)
    pubs = [("", long_t), ("", long_t[:80]), ("", long_t[:100]), ("", long_t[:149] + (b"w2",)),
            ("", long_t[:149] + (b"zz",))]
    _compare_batches(prod, orc, pubs, "long")


def test_mountpoints_are_disjoint_roots():
    node = "n@h"
    prod = H.ProductDriver(node, device=0)
    orc = O.TrieOracle(node)
    evs = [("updated", (mp, b"c"), None, [(node, True, [((b"a", b"+"), 1), ((b"a", b"b"), 0)])])
           for mp in ("", "tenant1", "tenant2")]
    evs.append(("updated", ("tenant1", b"d"), None, [(node, True, [((b"#",), 2)])]))
    prod.apply(evs)
    orc.apply(evs)
    pubs = [(mp, (b"a", b"b")) for mp in ("", "tenant1", "tenant2", "unknown")] + [("tenant1", (b"q",))]
    _compare_batches(prod, orc, pubs, "mp")


@pytest.mark.parametrize("mode", MODES)
def test_5000_mountpoints_grow_the_roots(mode):
    """5,000 mountpoints (vmq_reg_trie has no limit: vmq_reg_trie.erl:60,
    279-281, 320) on a context created with 16 roots: the root range grows by
    re-layouts while subscriptions arrive, and every publish — each
    mountpoint's own topics, other tenants' topics, an unknown mountpoint —
    folds to the oracle's entries, before and after deletes."""
    from tests.test_host_engine import _mp_events
    node = "n@h"
    prod = _driver(node, mode, max_mountpoints=16)
    orc = O.TrieOracle(node)
    adds, dels = _mp_events(5000, node)
    for lo in range(0, len(adds), 4000):
        prod.apply(adds[lo:lo + 4000])
        orc.apply(adds[lo:lo + 4000])
    import random
    r = random.Random(7)
    pubs = []
    for _ in range(6000):
        mp = "t%d" % r.randrange(5200)    # ~4 % unknown mountpoints
        pubs.append((mp, (b"w%d" % r.randrange(4), b"x%d" % r.randrange(3)) + ((b"z",) if r.random() < 0.3 else ())))
    pubs.append(("", (b"w0", b"x0")))
    _compare_batches(prod, orc, pubs, "5000 mountpoints")
    assert sum(len(x) for x in prod.fold_batch(pubs[:500])) > 100   # the tenants do match
    prod.apply(dels)
    orc.apply(dels)
    _compare_batches(prod, orc, pubs, "5000 mountpoints after deletes")


def test_empty_batch_and_output_growth():
    prod = _driver("n@h")
    v = prod.view
    v.handle_events([("updated", ("", b"c%d" % i), None, [("n@h", True, [((b"t",), 0)])]) for i in range(5000)])
    recs, offs = v.match_arrays(*v.prepare([]))
    assert len(recs) == 0 and list(offs) == [0]
    recs, offs = v.match_arrays(*v.prepare([("", (b"t",))] * 3), out_cap=10)   # grows internally
    assert list(offs) == [0, 5000, 10000, 15000]


def test_device_entry_point_with_torch_buffers():
    """vmqg_match_device on torch-allocated device memory and torch's stream."""
    import torch
    from vernemq_amd import workloads as W
    w = W.config_b(n_subs=20_000, n_pubs=4096)
    v, _ = _load_both(w, with_oracle=False)
    pubs, words = w.publish_arrays(v)
    ref_recs, ref_offs = v.match_arrays(pubs, words)
    dev = torch.device("cuda:0")
    d_pubs = torch.from_numpy(pubs.view(np.uint32).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = int(ref_offs[-1]) + 16
    d_out = torch.zeros(cap * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(len(pubs) + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    v.match_device(d_pubs.data_ptr(), len(pubs), d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(),
                   s.cuda_stream)
    assert v.match_status(s.cuda_stream) == 0
    offs = d_offs.cpu().numpy().astype(np.uint64)
    assert np.array_equal(offs, ref_offs)
    out = d_out.cpu().numpy().view(np.uint32).reshape(-1, 4)[: int(offs[-1])]
    ref = ref_recs.view(np.uint32).reshape(-1, 4)
    # identical per-publish multisets (the order inside a publish is deterministic too)
    assert np.array_equal(out, ref)


def test_null_stream_is_ordered_with_torch_default_stream():
    """stream = NULL (torch's default stream handle) runs on the legacy
    default stream: the match waits for inputs still being copied in behind a
    long default-stream queue, and a default-stream read-back waits for the
    match — no torch.cuda.synchronize() in between (vmqg_nullorder.h)."""
    import torch
    from vernemq_amd import workloads as W
    w = W.config_b(n_subs=20_000, n_pubs=4096)
    v, _ = _load_both(w, with_oracle=False)
    pubs, words = w.publish_arrays(v)
    ref_recs, ref_offs = v.match_arrays(pubs, words)
    dev = torch.device("cuda:0")
    assert torch.cuda.current_stream().cuda_stream == 0
    h_pubs = torch.from_numpy(pubs.view(np.uint32).view(np.int32).copy()).pin_memory()
    h_words = torch.from_numpy(words.astype(np.int32)).pin_memory()
    d_pubs = torch.zeros(h_pubs.numel(), dtype=torch.int32, device=dev)   # all publishes on an empty mountpoint...
    d_words = torch.zeros(h_words.numel(), dtype=torch.int32, device=dev)
    cap = int(ref_offs[-1]) + 16
    d_out = torch.zeros(cap * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(len(pubs) + 1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for rep in range(3):
        d_pubs.zero_()
        d_offs.zero_()
        x = torch.randn(4096, 4096, device=dev)
        for _ in range(8):                      # tens of ms of default-stream work ahead of the copies
            x = torch.tanh(x @ x)
        d_pubs.copy_(h_pubs, non_blocking=True)   # ...until these land
        d_words.copy_(h_words, non_blocking=True)
        v.match_device(d_pubs.data_ptr(), len(pubs), d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(), 0)
        offs = d_offs.cpu().numpy().astype(np.uint64)     # default stream, no synchronize
        assert np.array_equal(offs, ref_offs), rep
        assert v.match_status(0) == 0
    out = d_out.cpu().numpy().view(np.uint32).reshape(-1, 4)[: int(offs[-1])]
    assert np.array_equal(out, ref_recs.view(np.uint32).reshape(-1, 4))


def test_replica_follows_primary_by_image_and_patches():
    """A replica context fed the primary's arena image and then its patch
    stream answers identically (the RCCL broadcast payloads, minus RCCL)."""
    import torch
    from vernemq_amd import dist as vd
    wl = H.ChurnWorkload(7, n_clients=50)
    prim = H.ProductDriver(wl.self_node, device=0)
    from vernemq_amd.reg_view import RegGpuView
    rep = RegGpuView(node=wl.self_node, device=0, replica=True)
    prim.apply([wl.event() for _ in range(100)])
    ptr, nbytes, lay = prim.view.arena()
    # D2D copy of the primary arena into a torch buffer (the RCCL broadcast
    # buffer in bench.py), then into the replica
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    vd.hip_memcpy_d2d(img.data_ptr(), ptr, nbytes)
    rep.replica_load(lay, img.data_ptr())
    torch.cuda.synchronize()
    for step in range(10):
        prim.apply([wl.event() for _ in range(20)])
        data, full = prim.view.last_patches()
        if full:
            ptr, nbytes, lay = prim.view.arena()
            img = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
            vd.hip_memcpy_d2d(img.data_ptr(), ptr, nbytes)
            rep.replica_load(lay, img.data_ptr())
        elif data:
            buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda:0")
            rep.replica_sync_layout(prim.view.arena()[2])
            rep.apply_patches_device(buf.data_ptr(), len(data))
        torch.cuda.synchronize()
        pubs = wl.publishes(100)
        arr, words = prim.view.prepare(pubs)
        r1, o1 = prim.view.match_arrays(arr, words)
        r2, o2 = rep.match_arrays(arr, words)
        assert np.array_equal(o1, o2) and np.array_equal(r1, r2), step


def _config_d_expected_counts(w, live, pubs_lo, pubs_hi):
    """Known answer per publish of config D from the live mask: state
    publishes emit every live exact subscriber of (s, d); alarm publishes
    every live site/s/+/alarm/# subscriber; jobs/q/x publishes every live
    member of every group on q once per distinct node hosting a live member
    of that group (Q2, vmq_reg_trie.erl:68-72, 301-303)."""
    from collections import Counter, defaultdict
    idx = np.flatnonzero(live)
    topics = {}
    exact, alarm = Counter(), Counter()
    groups = defaultdict(list)
    for i in idx:
        t = w.sub_topic(i)
        if t[0] == b"site" and t[2] == b"dev":
            exact[(t[1], t[3])] += 1
        elif t[0] == b"site":
            alarm[t[1]] += 1
        else:
            groups[(t[1], t[3])].append(w.sub_node[i])
    jobs = Counter()
    for (g, q), nodes in groups.items():
        jobs[q] += len(nodes) * len(set(nodes))
    out = []
    for i in range(pubs_lo, pubs_hi):
        t = w.pub_topic(i)
        if t[0] == b"jobs":
            out.append(jobs[t[1]])
        elif t[2] == b"dev":
            out.append(exact[(t[1], t[3])])
        else:
            out.append(alarm[t[1]])
    return np.array(out, dtype=np.int64)


@pytest.mark.parametrize("mode", MODES)
def test_config_d_churn_parity(mode):
    """Config D at 1/20 scale (500k subs incl. $share groups over 4 nodes):
    after every churn batch, all publishes match the known answer and a
    sample matches the oracle publish for publish."""
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    w = W.config_d(scale=0.05, n_pubs=20_000)
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    ids = w.load_into(v, n=w.notes["n_live"])
    orc = feed.load_prefix(w, w.notes["n_live"])
    ch = W.Churn(w)
    pubs, words = w.publish_arrays(v)
    for step in range(4):
        if step:
            dels, adds = ch.batch(5000)
            ops, wds = ch.ops(ids, dels, adds)
            v.apply_op_arrays(ops, wds)
            orc.apply(ch.events(dels, adds))
        recs, offs = _match(v, pubs, words, mode)
        counts = np.diff(offs.astype(np.int64))
        assert np.array_equal(counts, _config_d_expected_counts(w, ch.live, 0, w.n_pubs)), step
        sample = list(range(0, w.n_pubs, 40))
        got = [sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1]))) for i in sample]
        want = orc.fold_batch([("", b"pub", w.pub_topic(i)) for i in sample])
        assert all(g == sorted(x) for g, x in zip(got, want)), step


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fast_g", [1, 2, 4])
def test_output_offsets_of_a_large_deferral_heavy_batch(mode, fast_g):
    """Output offsets over 300,000 publishes (9,375 chunks of 32 publishes,
    18,750 of 16) where every 23rd is h/x/y/z, which 31 filters match (more
    keys than the fast lists hold: deferred to the wave tier all over the
    batch, its count added to its chunk's total after COUNT), the others
    n/{j} matched by a few filters: every publish's count must equal the
    oracle's, and a sample its records."""
    import itertools
    node = "n@h"
    prod = _driver(node, mode)
    prod.view.set_option("dedupe", 0)   # this test pins the deferral tiers' counters
    prod.view.set_option("fast_g", fast_g)
    orc = O.TrieOracle(node)
    evs = []
    hot = (b"h", b"x", b"y", b"z")
    filters = set()
    for combo in itertools.product([0, 1], repeat=4):
        t = tuple(b"+" if c else hot[i] for i, c in enumerate(combo))
        filters.add(t)
        for k in range(4):
            filters.add(t[:k] + (b"#",))
    for i, t in enumerate(sorted(filters)):
        evs.append(("updated", ("", b"f%d" % i), None, [(node, True, [(t, i % 3)])]))
    for j in range(0, 1000, 2):
        evs.append(("updated", ("", b"n%d" % j), None, [(node, True, [((b"n", b"%d" % j), 1)])]))
    prod.apply(evs)
    orc.apply(evs)
    topics = [("", (b"n", b"%d" % j)) for j in range(1000)] + [("", hot)]
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in topics])
    assert len(want[-1]) == len(filters) > 16
    v = prod.view
    arr, words = v.prepare(topics)
    n = 300_000
    idx = np.arange(n) % 1000
    idx[::23] = 1000
    recs, offs = prod.match_arrays(arr[idx], words)
    assert v.stats_raw()["deferred_tier1"] == len(idx[::23])
    counts = np.diff(offs.astype(np.int64))
    assert int(offs[0]) == 0
    assert np.array_equal(counts, np.array([len(x) for x in want], dtype=np.int64)[idx])
    for i in list(range(0, n, 1999)) + list(range(n - 40, n)):
        got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
        assert got == sorted(want[idx[i]]), i


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fast_g", [1, 2])
def test_config_e_multitenant_parity(mode, fast_g):
    """Config E shape at 1/500 scale (100k subs over 1,000 Zipf-sized
    mountpoints, 12-level topics, hot-topic skew): every publish vs the
    oracle, under both fast-tier mappings."""
    from vernemq_amd import workloads as W
    w = W.config_e(scale=0.002, n_pubs=8192)
    v, orc = _load_both(w)
    v.set_option("fast_g", fast_g)
    got = _gpu_canon(v, w, 0, w.n_pubs, mode)
    want = orc.fold_batch([(w.mps[w.pub_mp[i]], b"pub", w.pub_topic(i)) for i in range(w.n_pubs)])
    bad = [i for i in range(w.n_pubs) if got[i] != sorted(want[i])]
    assert not bad, (len(bad), w.pub_topic(bad[0]))
    assert sum(len(x) for x in got) > w.n_pubs // 4


def _many_key_events(node):
    """$share groups hosted on 8 nodes: one filter node carries one key per
    {Node, Group} entry (vmq_reg_trie.erl:68-72, 290-303), so a publish meets
    far more keys than the fast tier's lists hold while its frontier stays
    small — the many-key mode (no deferral)."""
    nodes = [node] + ["n%d@h" % k for k in range(1, 8)]
    evs = []
    sub = lambda cid, nd, t, q: ("updated", ("", cid), None, [(nd, True, [(t, q)])])
    for g in range(12):   # jobs/+ : 12 groups x 16 members over the 8 nodes = 96 keys, 1,536 records
        for m in range(16):
            evs.append(sub(b"g%dm%d" % (g, m), nodes[m % 8], (b"$share", b"g%d" % g, b"jobs", b"+"), m % 3))
    for m in range(8):    # '#' alias candidate with many keys, and a group of one member per node
        evs.append(sub(b"h%d" % m, nodes[m], (b"$share", b"gh", b"jobs", b"#"), 1))
    evs.append(sub(b"plain", node, (b"jobs", b"#"), 0))              # one local key
    evs.append(sub(b"remote3", nodes[3], (b"jobs", b"+"), 0))        # a remote node in the mask
    evs.append(sub(b"exact5", node, (b"jobs", b"x5"), 2))            # the exact key, in many-key mode
    for m in range(8):    # k/+ : 8 keys, + the exact key k/x = 9 (overflows G=2's 8 at the exact probe)
        evs.append(sub(b"k%d" % m, nodes[m], (b"$share", b"gk", b"k", b"+"), 0))
    evs.append(sub(b"kx", node, (b"k", b"x"), 1))
    for m in range(8):    # $SYS/+ (valid for $-topics) and +/x5 (skipped for them, MQTT-4.7.2-1)
        evs.append(sub(b"s%d" % m, nodes[m], (b"$share", b"gs", b"$SYS", b"+"), 0))
        evs.append(sub(b"d%d" % m, nodes[m], (b"$share", b"gd", b"+", b"x5"), 0))
    for j in range(64):   # ordinary publishes: one exact subscriber each
        evs.append(sub(b"o%d" % j, node, (b"o", b"%d" % j), 0))
    return evs


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fast_g", [1, 2, 4])
def test_many_key_publishes_stay_in_the_fast_tier(mode, fast_g):
    """Publishes matching $share groups on many nodes (up to 105 keys, 1,600
    records each) are counted by the fast tier and written wave-wide by the
    EMIT wave-tier launch — none deferred — and equal the oracle's, mixed
    with ordinary publishes in one batch."""
    node = "n0@h"
    prod = _driver(node, mode, nodes=[node] + ["n%d@h" % k for k in range(1, 8)])
    prod.view.set_option("dedupe", 0)   # this test pins the deferral tiers' counters
    prod.view.set_option("fast_g", fast_g)
    orc = O.TrieOracle(node)
    evs = _many_key_events(node)
    prod.apply(evs)
    orc.apply(evs)
    kinds = [("", (b"jobs", b"x%d" % j)) for j in range(8)] + [("", (b"k", b"x")), ("", (b"k", b"y")),
             ("", (b"$SYS", b"x5")), ("", (b"$SYS", b"q")), ("", (b"jobs",))]
    kinds += [("", (b"o", b"%d" % j)) for j in range(64)]
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in kinds])
    assert max(len(x) for x in want) > 1500
    v = prod.view
    arr, words = v.prepare(kinds)
    rs = np.random.RandomState(7)
    idx = rs.randint(0, len(kinds), size=6000)
    idx[:len(kinds)] = np.arange(len(kinds))
    recs, offs = prod.match_arrays(arr[idx], words)
    st = v.stats_raw()
    assert st["deferred_tier1"] == 0, st
    assert st["many_key"] > 0, st
    counts = np.diff(offs.astype(np.int64))
    assert np.array_equal(counts, np.array([len(x) for x in want], dtype=np.int64)[idx])
    for i in list(range(len(kinds))) + list(range(len(kinds), len(idx), 97)):
        got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
        assert got == sorted(want[idx[i]]), (i, kinds[idx[i]])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fast_g", [1, 2, 4])
def test_two_key_publishes_with_one_record_keys(mode, fast_g):
    """Every two-key publish whose second (or first, or both) key holds
    exactly one record: the EMIT resolve preloads one-record keys, per lane
    of the group (the one-lane case included)."""
    node = "n@h"
    prod = _driver(node, mode)
    prod.view.set_option("fast_g", fast_g)
    orc = O.TrieOracle(node)
    sub = lambda cid, t, q: ("updated", ("", cid), None, [(node, True, [(t, q)])])
    evs = [sub(b"a%d" % i, (b"a", b"+"), i % 3) for i in range(40)]           # key 0: 40 records
    evs += [sub(b"b0", (b"b", b"+"), 1)]                                      # key 0: 1 record
    evs += [sub(b"c%d" % i, (b"c", b"+"), 0) for i in range(3)]               # key 0: 3 records
    for j in range(50):
        evs.append(sub(b"ax%d" % j, (b"a", b"%d" % j), 2))                    # key 1: 1 record
        evs.append(sub(b"bx%d" % j, (b"b", b"%d" % j), 0))                    # key 1: 1 record
        evs += [sub(b"cx%d_%d" % (j, i), (b"c", b"%d" % j), 1) for i in range(2)]   # key 1: 2 records
    prod.apply(evs)
    orc.apply(evs)
    kinds = [("", (p, b"%d" % j)) for p in (b"a", b"b", b"c") for j in range(60)]
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in kinds])
    v = prod.view
    arr, words = v.prepare(kinds)
    idx = np.random.RandomState(3).randint(0, len(kinds), size=20_000)
    recs, offs = prod.match_arrays(arr[idx], words)
    counts = np.diff(offs.astype(np.int64))
    assert np.array_equal(counts, np.array([len(x) for x in want], dtype=np.int64)[idx])
    for i in range(0, len(idx), 7):
        got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
        assert got == sorted(want[idx[i]]), (i, kinds[idx[i]])


def test_range_results_are_epoch_safe():
    """A range match queued before an apply that rewrites record slots cannot
    be expanded against the post-apply table (vmqg_records_at refuses its
    epoch); matched again, the ranges expand to the oracle's answer at the
    new epoch, and a range result with no apply after it expands to the
    oracle's answer at its own epoch (lookup_subs/1 never returns a stale
    list, vmq_reg_trie.erl:87-94)."""
    import torch
    from vernemq_amd import _lib
    node = "n@h"
    prod = _driver(node)
    v = prod.view
    orc = O.TrieOracle(node)
    sub = lambda cid, t, q: ("updated", ("", cid), None, [(node, True, [(t, q)])])
    evs = [sub(b"w%d" % i, (b"a", b"+"), i % 3) for i in range(50)]
    evs += [sub(b"x%d" % i, (b"a", b"%d" % (i % 5)), 1) for i in range(20)]
    prod.apply(evs)
    orc.apply(evs)
    topics = [("", (b"a", b"%d" % j)) for j in range(8)]
    arr, words = v.prepare(topics)
    dev = torch.device("cuda:0")
    d_pubs = torch.from_numpy(arr.view(np.uint32).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = 1024
    d_rng = torch.zeros(cap * 2, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(len(arr) + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def queue():
        e = v.epoch()
        v.match_ranges_device(d_pubs.data_ptr(), len(arr), d_words.data_ptr(), d_rng.data_ptr(), cap,
                              d_offs.data_ptr(), s)
        return e

    def expand(e):
        assert v.match_status(s) == 0
        offs = d_offs.cpu().numpy().astype(np.uint64)
        rng = d_rng.cpu().numpy().view(np.uint32).reshape(-1, 2)[: int(offs[-1])]
        r = np.zeros(len(rng), dtype=[("off", "<u4"), ("count", "<u4")])
        r["off"], r["count"] = rng[:, 0], rng[:, 1]
        recs, eo = v.expand_ranges(r, offs, recs=v.records(epoch=e))
        return [sorted(H.canon(v.decode(recs[j])) for j in range(int(eo[i]), int(eo[i + 1]))) for i in range(len(arr))]

    def want():
        return [sorted(x) for x in orc.fold_batch([(mp, b"pub", t) for mp, t in topics])]

    e0 = queue()
    assert expand(e0) == want()                     # no apply in between
    e1 = queue()
    dels = [("deleted", ("", b"w%d" % i), [(node, True, [((b"a", b"+"), i % 3)])]) for i in range(0, 50, 3)]
    prod.apply(dels)                                # deletes move records into the freed slots
    orc.apply(dels)
    torch.cuda.synchronize()
    with pytest.raises(_lib.VmqgError):
        v.records(epoch=e1)
    e2 = queue()
    assert e2 > e1
    assert expand(e2) == want()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fast_g", [1, 2, 4])
def test_retry_tier_serves_one_lane_overflows(mode, fast_g):
    """16 filters over {x, +} at 4 levels all match x/x/x/x: more candidates
    than the one- and two-lane fast passes hold, so the COUNT wave-tier
    launch retries the publish four lanes per publish (16 candidates, 17 keys
    with the exact one: many-key mode) — no whole-wave walk — interleaved
    with publishes the fast pass serves."""
    import itertools
    node = "n@h"
    prod = _driver(node, mode)
    prod.view.set_option("dedupe", 0)   # this test pins the deferral tiers' counters
    prod.view.set_option("fast_g", fast_g)
    orc = O.TrieOracle(node)
    evs = []
    for i, combo in enumerate(itertools.product([b"x", b"+"], repeat=4)):
        evs.append(("updated", ("", b"f%d" % i), None, [(node, True, [(combo, i % 3)])]))
    evs.append(("updated", ("", b"ex"), None, [(node, True, [((b"x", b"x", b"x", b"x"), 1)])]))
    evs += [("updated", ("", b"o%d" % j), None, [(node, True, [((b"o", b"%d" % j), 0)])]) for j in range(32)]
    prod.apply(evs)
    orc.apply(evs)
    kinds = [("", (b"x",) * 4), ("", (b"x", b"y", b"x", b"y"))] + [("", (b"o", b"%d" % j)) for j in range(32)]
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in kinds])
    assert len(want[0]) == 17
    v = prod.view
    arr, words = v.prepare(kinds)
    idx = np.random.RandomState(5).randint(0, len(kinds), size=5000)
    idx[:2] = [0, 1]
    recs, offs = prod.match_arrays(arr[idx], words)
    st = v.stats_raw()
    assert st["deferred_tier1"] == 0, st
    assert (st["retried"] > 0) == (fast_g != 4), st
    counts = np.diff(offs.astype(np.int64))
    assert np.array_equal(counts, np.array([len(x) for x in want], dtype=np.int64)[idx])
    for i in range(0, len(idx), 3):
        got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
        assert got == sorted(want[idx[i]]), (i, kinds[idx[i]])


def test_released_stream_can_be_destroyed():
    """A caller stream released with vmqg_release_stream (the context's last
    work was on it) may be destroyed: the next call on another stream waits
    for the event recorded at release, not on the dead stream."""
    import gc
    import torch
    from vernemq_amd import workloads as W
    w = W.config_b(n_subs=20_000, n_pubs=4096)
    v, _ = _load_both(w, with_oracle=False)
    pubs, words = w.publish_arrays(v)
    ref_recs, ref_offs = v.match_arrays(pubs, words)
    dev = torch.device("cuda:0")
    d_pubs = torch.from_numpy(pubs.view(np.uint32).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = int(ref_offs[-1]) + 16
    d_out = torch.zeros(cap * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(len(pubs) + 1, dtype=torch.int64, device=dev)
    for rep in range(3):
        s = torch.cuda.Stream()
        v.match_device(d_pubs.data_ptr(), len(pubs), d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(),
                       s.cuda_stream)
        v.release_stream(s.cuda_stream)
        s.synchronize()
        del s
        gc.collect()
        d_offs.zero_()
        v.match_device(d_pubs.data_ptr(), len(pubs), d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(), 0)
        assert v.match_status(0) == 0
        assert np.array_equal(d_offs.cpu().numpy().astype(np.uint64), ref_offs), rep


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fast_g", [1, 2])
def test_wide_publishes_by_record_count(mode, fast_g):
    """Publishes of one or two keys but hundreds of records (a/+ with 300
    subscribers, plus an exact one), in batches that mix them with
    one-record publishes and with publishes of several hundred records under
    other keys: the fast EMIT copies them (wide publishes are those with more
    keys than the spill slots hold, not with many records: VMQG_WIDE_RECORDS,
    A/B in DESIGN.md), and every publish's records equal the oracle's."""
    node = "n@h"
    prod = _driver(node, mode)
    prod.view.set_option("dedupe", 0)   # this test pins the deferral tiers' counters
    prod.view.set_option("fast_g", fast_g)
    orc = O.TrieOracle(node)
    sub = lambda cid, t, q: ("updated", ("", cid), None, [(node, True, [(t, q)])])
    evs = [sub(b"a%d" % i, (b"a", b"+"), i % 3) for i in range(300)]
    evs += [sub(b"b%d" % i, (b"b", b"#"), 1) for i in range(255)]              # just below the threshold
    evs += [sub(b"c%d" % i, (b"c", b"+", b"x"), 2) for i in range(700)]
    evs += [sub(b"ax%d" % j, (b"a", b"%d" % j), 0) for j in range(0, 40, 2)]
    evs += [sub(b"o%d" % j, (b"o", b"%d" % j), 0) for j in range(40)]
    prod.apply(evs)
    orc.apply(evs)
    kinds = [("", (p, b"%d" % j)) for p in (b"a", b"b", b"o") for j in range(40)] + \
            [("", (b"c", b"%d" % j, b"x")) for j in range(8)]
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in kinds])
    v = prod.view
    arr, words = v.prepare(kinds)
    idx = np.random.RandomState(9).randint(0, len(kinds), size=12_000)
    recs, offs = prod.match_arrays(arr[idx], words)
    st = v.stats_raw()
    assert st["many_key"] == 0 and st["deferred_tier1"] == 0, st
    counts = np.diff(offs.astype(np.int64))
    assert np.array_equal(counts, np.array([len(x) for x in want], dtype=np.int64)[idx])
    for i in range(0, len(idx), 5):
        got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
        assert got == sorted(want[idx[i]]), (i, kinds[idx[i]])


def _device_match_records(v, pubs, words, total_hint):
    """Device-buffer records match (vmqg_match_device, the bench's path):
    returns the device output tensor (int32 view of the 16-B records) and the
    offsets on the host; the output is sized from the known answer."""
    import torch
    dev = torch.device("cuda", 0)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    n = len(pubs)
    cap = int(total_hint) + 1024
    d_out = torch.full((cap * 4,), -1, dtype=torch.int32, device=dev)   # a position never written stays all-ones
    d_offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    v.match_device(d_pubs.data_ptr(), n, d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(), sp)
    torch.cuda.synchronize()
    assert v.match_status(sp) == 0
    offs = d_offs.cpu().numpy()
    holes = torch.nonzero((d_out.view(-1, 4)[:int(offs[-1])] == -1).all(dim=1)).flatten().cpu().numpy()
    if len(holes):
        pub = np.searchsorted(offs.astype(np.int64), holes, side="right") - 1
        raise AssertionError("%d record positions never written, in %d publishes (first %d: count %d)" % (
            len(holes), len(np.unique(pub)), int(pub[0]), int(offs[pub[0] + 1] - offs[pub[0]])))
    return d_out, offs


def _sample_records(v, d_out, offs, sample, sub_term=None):
    """The records of the sampled publishes, gathered on the device, decoded
    (sub_term: SubscriberId terms of a lean workload, RegGpuView.decode)."""
    import torch
    from vernemq_amd.reg_view import EMIT_DTYPE
    lo = offs[sample].astype(np.int64)
    hi = offs[np.asarray(sample) + 1].astype(np.int64)
    lens = hi - lo
    pos = np.repeat(lo - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(int(lens.sum()))
    idx = torch.from_numpy(pos).to(d_out.device)
    recs = d_out.view(-1, 4).index_select(0, idx).cpu().numpy().view(EMIT_DTYPE).reshape(-1)
    out, k = [], 0
    for n in lens:
        out.append(sorted(H.canon(v.decode(recs[j], sub_term)) for j in range(k, k + int(n))))
        k += int(n)
    return out


def test_config_d_full_size_under_churn():
    """Verdict r3 item 5: config D at FULL size (10M live subscriptions, 8M
    exact + 1M site/s/+/alarm/# + 1M $share members on 4 nodes; 2^20
    publishes of which 30 % write hundreds to thousands of records) in the
    driver's GPU run: every publish's count against the known answer
    (workloads.config_d_counts), after the bulk load and after each of two
    10,000-op churn batches; plus a 2,048-publish oracle sample each time.
    The sample's publishes name 8 sites and 8 job queues, and the oracle
    holds exactly the subscriptions those can match (a site's exact and
    alarm filters, every group on a queue: a publish only meets filters with
    its own literal words), so the sample check is exact at full size.
    vmq_reg_trie.erl:305-316 (bulk load), :68-72 and :301-303 (Q2 on the
    $share groups, each member emitted once per hosting node)."""
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    w = W.config_d()
    n_live = w.notes["n_live"]
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes,
                   hints={"edges": 4 * n_live // 5, "paths": 4 * n_live // 5, "keys": n_live,
                          "records": n_live * 11 // 10, "exact": n_live})   # bench.py's config-D sizing
    ids = w.load_into(v, n=n_live)
    ch = W.Churn(w)
    pubs, words = w.publish_arrays(v)
    # the sample: publishes on 8 sites / 8 queues; the oracle holds what they can match
    T = w.tw.reshape(-1, 5)
    a = w.pw_off[:-1]
    first, second = w.pw[a], w.pw[a + 1] - 5
    is_jobs = first == 4
    sites = np.unique(second[~is_jobs])[::125][:8]
    queues = np.unique(second[is_jobs])[::125][:8]
    cand = np.flatnonzero((~is_jobs & np.isin(second, sites)) | (is_jobs & np.isin(second, queues)))
    sample = cand[np.linspace(0, len(cand) - 1, 2048).astype(np.int64)]
    relevant = ((T[:, 0] == 0) & np.isin(T[:, 1] - 8, sites)) | ((T[:, 0] == 6) & np.isin(T[:, 3] - 8, queues))
    orc = O.TrieOracle(w.self_node)
    orc.apply_raw(feed.init_bytes(w, idx=np.flatnonzero(relevant[:n_live])))
    for step in range(3):
        if step:
            dels, adds = ch.batch(10_000)
            ops, wds = ch.ops(ids, dels, adds)
            v.apply_op_arrays(ops, wds)
            orc.apply(ch.events(dels[relevant[dels]], adds[relevant[adds]]))
        want_counts = W.config_d_counts(w, ch.live)
        d_out, offs = _device_match_records(v, pubs, words, want_counts.sum())
        counts = np.diff(offs.astype(np.int64))
        assert np.array_equal(counts, want_counts), (step, int(np.count_nonzero(counts != want_counts)))
        got = _sample_records(v, d_out, offs, sample)
        want = orc.fold_batch([("", b"pub", w.pub_topic(int(i))) for i in sample])
        bad = [k for k in range(len(sample)) if got[k] != sorted(want[k])]
        assert not bad, (step, len(bad), w.pub_topic(int(sample[bad[0]])), got[bad[0]][:4], sorted(want[bad[0]])[:4])
        assert sum(len(x) for x in got) > len(sample)
        del d_out


def test_config_e_full_size_oracle_sample():
    """Config E at full size in the driver's GPU run (verdict r5 item 7; 0.2
    scale before): 50M subscriptions over 1,000 Zipf-sized mountpoints, 12
    levels, 2^20 Zipf(1.1) hot-topic publishes, library defaults.  A
    2,048-publish sample in the mountpoints of <= 1M subscriptions against an
    oracle holding exactly those mountpoints' subscriptions (a publish only
    walks its own mountpoint's trie, so the check is exact), plus every
    publish's count against the range-mode expansion of a second match.
    VMQG_E_TEST_SCALE scales it down for a quick run."""
    import os
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    w = W.config_e(scale=float(os.environ.get("VMQG_E_TEST_SCALE", "1.0")))
    n = w.n_subs
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes, max_mountpoints=max(1024, len(w.mps) + 1),
                   hints={"edges": 2 * n, "paths": 2 * n, "keys": n * 5 // 4, "records": n * 5 // 4,
                          "exact": n * 5 // 4})
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    # records: counts, then a sample
    rng, roffs = v.match_ranges(pubs, words)
    per = np.where(rng["count"] > 0, rng["count"], 1).astype(np.float64)
    cnt_r = np.bincount(np.repeat(np.arange(len(pubs)), np.diff(roffs.astype(np.int64))), weights=per,
                        minlength=len(pubs)).astype(np.int64)
    d_out, offs = _device_match_records(v, pubs, words, cnt_r.sum())
    assert np.array_equal(np.diff(offs.astype(np.int64)), cnt_r)
    # the oracle holds <= 1M subscriptions (its bulk load runs ~40k/s): the
    # mountpoints most published to that fit, in that order
    per_mp = np.bincount(w.client_mp[w.sub_client], minlength=len(w.mps))
    hot = np.argsort(-np.bincount(w.pub_mp, minlength=len(w.mps)), kind="stable")
    fit, tot = [], 0
    for m in hot:                     # greedy: skip the ones that do not fit
        if tot + per_mp[m] <= 1_000_000 and per_mp[m] > 0:
            fit.append(m)
            tot += per_mp[m]
    cand = np.flatnonzero(np.isin(w.pub_mp, fit))
    assert len(fit) >= 8 and len(cand) >= 2048, (len(fit), len(cand))
    sample = cand[np.linspace(0, len(cand) - 1, 2048).astype(np.int64)]
    mps = np.unique(w.pub_mp[sample])
    subs_idx = np.flatnonzero(np.isin(w.client_mp[w.sub_client], mps))
    orc = O.TrieOracle(w.self_node)
    for lo in range(0, len(subs_idx), 1 << 18):
        orc.apply_raw(feed.init_bytes(w, idx=subs_idx[lo:lo + (1 << 18)]))
    got = _sample_records(v, d_out, offs, sample, w.client_term)   # lean workload: subscriber id = client index
    want = orc.fold_batch([(w.mps[w.pub_mp[i]], b"pub", w.pub_topic(int(i))) for i in sample])
    bad = [k for k in range(len(sample)) if got[k] != sorted(want[k])]
    assert not bad, (len(bad), w.pub_topic(int(sample[bad[0]])))
    assert sum(len(x) for x in got) > len(sample) // 4


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("fast_g", [1, 2, 4])
@pytest.mark.parametrize("dd_g", [1, 4])
def test_batch_dedupe_repeated_topics(mode, fast_g, dd_g):
    """Batch-wide dedupe (verdict r3 item 4): 200,000 publishes drawn from 1,001
    topics — repeats across chunk and wave boundaries, many of them of
    h/x/y/z, which 31 filters match (deferred by the fast tier, so its
    duplicates cannot take a fast-pass answer and are walked by the fixup).
    With dedupe forced on every publish's count equals the oracle's and a
    sample its records; the stats show duplicates served from a
    representative and duplicates of a deferred representative walked."""
    import itertools
    node = "n@h"
    prod = _driver(node, mode)
    v = prod.view
    v.set_option("fast_g", fast_g)
    v.set_option("dedupe", 1)
    v.set_option("dd_g", dd_g)
    orc = O.TrieOracle(node)
    evs = []
    hot = (b"h", b"x", b"y", b"z")
    filters = set()
    for combo in itertools.product([0, 1], repeat=4):
        t = tuple(b"+" if c else hot[i] for i, c in enumerate(combo))
        filters.add(t)
        for k in range(4):
            filters.add(t[:k] + (b"#",))
    for i, t in enumerate(sorted(filters)):
        evs.append(("updated", ("", b"f%d" % i), None, [(node, True, [(t, i % 3)])]))
    for j in range(0, 1000, 2):
        evs.append(("updated", ("", b"n%d" % j), None, [(node, True, [((b"n", b"%d" % j), 1)])]))
    evs.append(("updated", ("", b"w"), None, [(node, True, [((b"n", b"+"), 2)])]))
    prod.apply(evs)
    orc.apply(evs)
    topics = [("", (b"n", b"%d" % j)) for j in range(1000)] + [("", hot)]
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in topics])
    arr, words = v.prepare(topics)
    r = np.random.default_rng(7)
    n = 200_000
    idx = r.integers(0, 1000, n)
    idx[r.random(n) < 0.03] = 1000
    recs, offs = prod.match_arrays(arr[idx], words)
    st = v.stats_raw()
    counts = np.diff(offs.astype(np.int64))
    assert np.array_equal(counts, np.array([len(x) for x in want], dtype=np.int64)[idx])
    for i in list(range(0, n, 997)) + list(range(n - 70, n)) + [int(k) for k in np.flatnonzero(idx == 1000)[:50]]:
        got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
        assert got == sorted(want[idx[i]]), i
    assert st["dedup"] > n // 2, st
    if fast_g != 4 and dd_g == 1:
        assert st["dedup_walked"] > 0, st   # duplicates of the deferred h/x/y/z representatives


def test_batch_dedupe_auto_mode_follows_the_repetition():
    """dedupe 2 (auto): one call in 64 runs deduped to measure the batch's
    repetition; the calls after it dedupe while more than half its publishes
    repeat, and stop when a probe sees distinct topics — with the same
    answers either way."""
    node = "n@h"
    prod = _driver(node)
    v = prod.view
    v.set_option("dedupe", 2)
    orc = O.TrieOracle(node)
    evs = [("updated", ("", b"c%d" % j), None, [(node, True, [((b"d", b"%d" % j, b"#"), 1)])]) for j in range(3000)]
    evs += [("updated", ("", b"all%d" % k), None, [(node, True, [((b"d", b"+", b"t%d" % k), 0)])]) for k in range(20)]
    prod.apply(evs)
    orc.apply(evs)
    # 60,000 distinct topics of known words only (publishes whose unknown
    # words sit at the same places are one topic to the matcher: deduped)
    distinct = [("", (b"d", b"%d" % (j % 3000), b"t%d" % (j // 3000))) for j in range(60_000)]
    arr, words = v.prepare(distinct)
    _, o1 = prod.match_arrays(arr, words)            # the first call is a probe: nothing repeats
    assert v.stats_raw()["dedup"] == 0
    _, o1b = prod.match_arrays(arr, words)
    c1 = np.diff(o1.astype(np.int64))
    assert np.array_equal(c1, np.diff(o1b.astype(np.int64)))
    rep = np.random.default_rng(3).integers(0, 100, 60_000)
    for _ in range(64):                              # one of these is a probe that sees the repetition
        _, o2 = prod.match_arrays(arr[rep], words)
        assert np.array_equal(np.diff(o2.astype(np.int64)), c1[rep])
    _, o3 = prod.match_arrays(arr[rep], words)       # ... so this call dedupes
    assert v.stats_raw()["dedup"] > 50_000
    assert np.array_equal(np.diff(o3.astype(np.int64)), c1[rep])
    for _ in range(64):                              # distinct topics again: a probe turns it off
        prod.match_arrays(arr, words)
    _, o4 = prod.match_arrays(arr, words)
    assert v.stats_raw()["dedup"] == 0
    assert np.array_equal(np.diff(o4.astype(np.int64)), c1)
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in distinct[:3000]])
    assert np.array_equal(c1[:3000], [len(x) for x in want])


def test_output_groups_and_dedupe_write_the_same_bytes():
    """The EMIT tail's output groups (big publishes written group by group)
    and COUNT's batch dedupe change where and when records are written, not
    what: on config D at 1/20 scale (alarm publishes of 1,000 records, $share
    jobs of 400) the offsets and every record byte are equal with each of
    them off and on; the default build's records are checked against the
    oracle by test_config_d_churn_parity."""
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    w = W.config_d(scale=0.05, n_pubs=60_000)
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v, n=w.notes["n_live"])
    pubs, words = w.publish_arrays(v)
    outs = []
    for groups, dedupe in ((0, 0), (1, 0), (1, 1), (0, 1)):
        v.set_option("groups", groups)
        v.set_option("dedupe", dedupe)
        recs, offs = v.match_arrays(pubs, words)
        st = v.stats_raw()
        outs.append((np.asarray(offs).copy(), np.asarray(recs).view(np.uint8).copy()))
        if dedupe:
            assert st["dedup"] > 0
    v.set_option("groups", 1)
    v.set_option("dedupe", 2)
    for o, r in outs[1:]:
        assert np.array_equal(o, outs[0][0])
        assert np.array_equal(r, outs[0][1])
    assert int(outs[0][0][-1]) > 1000 * len(pubs) // 10


def test_group_slots_of_older_calls_do_not_survive_a_tag_restart():
    """Output-group slots are claimed per call by the dedupe tag; the tag
    restarts when the dedupe table grows.  Call 1: 1,000 publishes of g/x
    (200 records, one key: output groups); call 2: 3,000 publishes of s/y
    (3 keys, spilled) — a bigger batch, so the dedupe table grows while the
    group table does not.  Call 2's publishes 0..999 must not be taken for
    call 1's group members (the tail would write them as one-key publishes)."""
    node = "n@h"
    prod = _driver(node)
    v = prod.view
    v.set_option("dedupe", 0)
    v.set_option("groups", 1)
    orc = O.TrieOracle(node)
    evs = [("updated", ("", b"g%d" % i), None, [(node, True, [((b"g", b"x"), i % 3)])]) for i in range(200)]
    for i, f in enumerate([(b"s", b"y"), (b"s", b"+"), (b"+", b"y")]):
        evs.append(("updated", ("", b"s%d" % i), None, [(node, True, [(f, 1)])]))
    prod.apply(evs)
    orc.apply(evs)
    want_g, want_s = orc.fold_batch([("", b"pub", (b"g", b"x")), ("", b"pub", (b"s", b"y"))])
    arr, words = v.prepare([("", (b"g", b"x")), ("", (b"s", b"y"))])
    recs, offs = prod.match_arrays(arr[np.zeros(1000, dtype=np.int64)], words)
    assert np.array_equal(np.diff(offs.astype(np.int64)), np.full(1000, len(want_g)))
    for n in (3000, 3000):
        recs, offs = prod.match_arrays(arr[np.ones(n, dtype=np.int64)], words)
        assert np.array_equal(np.diff(offs.astype(np.int64)), np.full(n, len(want_s)))
        for i in list(range(0, 1000, 37)) + [n - 1]:
            got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
            assert got == sorted(want_s), i


def test_more_global_stack_walks_than_stacks():
    """the EMIT tail borrows tier-2 global stacks from a bitmap
    (o_waves of them) while its grid has far more waves.  4,096 publishes
    of x^16 (each a 2^16-wide frontier walked by a whole wave with a global
    stack, dedupe off so every one is walked) make more concurrent borrowers
    than stacks: every count must be 65,536, sampled publishes must equal
    the oracle, the call's status must be clean, and a second call must
    succeed (the bitmap was released)."""
    import itertools
    node = "n@h"
    prod = _driver(node)
    v = prod.view
    v.set_option("dedupe", 0)
    orc = O.TrieOracle(node)
    subs = [("updated", ("", b"s%d" % i), None, [(node, True, [(combo, i % 3)])])
            for i, combo in enumerate(itertools.product([b"x", b"+"], repeat=16))]
    for lo in range(0, len(subs), 8192):
        prod.apply(subs[lo:lo + 8192])
        orc.apply(subs[lo:lo + 8192])
    want = sorted(orc.fold_batch([("", b"pub", (b"x",) * 16)])[0])
    arr, words = v.prepare([("", (b"x",) * 16)])
    n = 4096
    for call in range(2):
        recs, offs = prod.match_arrays(arr[np.zeros(n, dtype=np.int64)], words)
        assert np.array_equal(np.diff(offs.astype(np.int64)), np.full(n, 1 << 16)), call
        for i in (0, 1, n // 2, n - 1):
            got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
            assert got == want, (call, i)
        st = v.stats_raw()
        assert st["deferred_tier2"] >= n, st
        del recs


@pytest.mark.parametrize("mode", MODES)
def test_dedupe_keeps_dollar_topics_apart(mode):
    """z/b and $SYS/b carry the same word ids when neither first word is a
    filter word (one unknown id), but '$SYS/b' must not match '+/b' or '#'
    (MQTT-4.7.2-1, vmq_reg_trie.erl:457-462): dedupe must not make one the
    other's duplicate, whichever order they come in."""
    node = "n@h"
    prod = _driver(node, mode)
    v = prod.view
    v.set_option("dedupe", 1)
    orc = O.TrieOracle(node)
    evs = [("updated", ("", b"w%d" % i), None, [(node, True, [(f, i % 3)])])
           for i, f in enumerate([(b"+", b"b"), (b"#",), (b"q", b"b")])]
    prod.apply(evs)
    orc.apply(evs)
    topics = [("", (b"z", b"b")), ("", (b"$SYS", b"b")), ("", (b"y", b"b")), ("", (b"$X", b"b"))]
    want = [sorted(x) for x in orc.fold_batch([(mp, b"pub", t) for mp, t in topics])]
    assert want[0] != want[1]
    arr, words = v.prepare(topics)
    for order in (np.arange(4000) % 4, (np.arange(4000) % 4)[::-1].copy()):
        recs, offs = prod.match_arrays(arr[order], words)
        for i in list(range(0, 4000, 7)) + list(range(3990, 4000)):
            got = sorted(H.canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
            assert got == want[order[i]], (i, topics[order[i]])


@pytest.mark.parametrize("mode", MODES)
def test_trieless_tables_take_the_exact_only_count(mode):
    """Tables without any wildcard or $share filter (every subscription exact:
    bench_single_lookups' shape, vmq_reg_trie_bench_SUITE.erl:114-150): COUNT
    is one exact probe per publish, four per lane in flight (option
    "trieless").  Against the oracle and byte-identical to the general walk
    (trieless 0), with local and remote subscribers, remote nodes >= 64 (the
    slot's high list: the wave tier takes the publish), two mountpoints, topics
    longer than the slot's 7 inline words, publishes that hold '+' or unknown
    words, empty lists and an unknown mountpoint; heavy routing on and off."""
    import random
    nodes = ["n%d@h" % i for i in range(80)]
    prod = _driver(nodes[0], mode, nodes=nodes)
    orc = O.TrieOracle(nodes[0])
    r = random.Random(5)
    vocab = [b"a", b"b", b"c", b"dev", b"x%d" % 7]
    topics = []
    for k in range(3000):
        L = r.choice([1, 2, 3, 4, 8, 9])
        topics.append(tuple([r.choice(vocab) for _ in range(L - 1)] + [b"t%d" % k]))
    evs = []
    for k, t in enumerate(topics):
        mp = "" if k % 5 else "m2"
        for j in range(r.choice([1, 1, 2, 3, 40])):
            x = r.random()
            node = nodes[0] if x < 0.7 else (r.choice(nodes[1:60]) if x < 0.95 else r.choice(nodes[64:]))
            evs.append(("updated", (mp, b"c%d_%d" % (k, j)), None, [(node, True, [(t, j % 3)])]))
    prod.apply(evs)
    orc.apply(evs)
    pubs = []
    for i in range(20000):
        x = r.random()
        if x < 0.7:
            k = r.randrange(len(topics))
            pubs.append(("" if k % 5 else "m2", topics[k]))
        elif x < 0.8:
            pubs.append(("", tuple(r.choice(vocab) for _ in range(3))))
        elif x < 0.85:
            pubs.append(("", (b"a", b"+")))
        elif x < 0.9:
            pubs.append(("", ()))
        elif x < 0.95:
            pubs.append(("nomp", (b"a", b"t1")))
        else:
            pubs.append(("", (b"zz", b"t%d" % r.randrange(3000))))
    want = [sorted(x) for x in orc.fold_batch([(mp, b"p", t) for mp, t in pubs])]
    v = prod.view
    outs = {}
    # fast_g 1 / 2 / 4: chunks of 64 / 32 / 16 publishes, which the trie-less
    # EMIT (k_emit_exact, 64-publish blocks) must position alike
    # fused 1 (the default): the trie-less COUNT, scan and EMIT in one launch
    for fg in (1, 2, 4):
        v.set_option("fast_g", fg)
        for tl, hm, fu in ((1, 0, 1), (1, 0, 0), (0, 0, 1), (1, 8, 1), (0, 8, 1)):
            v.set_option("trieless", tl)
            v.set_option("heavy_min", hm)
            v.set_option("fused", fu)
            arr, words = v.prepare([(mp, tuple(t)) for mp, t in pubs])
            recs, offs = prod.match_arrays(arr, words)
            outs[tl, hm, fg, fu] = (np.asarray(offs).copy(), np.asarray(recs).view(np.uint8).copy())
            got = prod.fold_batch(pubs)
            bad = [i for i in range(len(pubs)) if sorted(got[i]) != want[i]]
            assert not bad, (fg, tl, hm, fu, len(bad), pubs[bad[0]], sorted(got[bad[0]])[:4], want[bad[0]][:4])
        for a, b in (((1, 0, fg, 1), (1, 0, fg, 0)), ((1, 0, fg, 0), (0, 0, fg, 1)), ((1, 8, fg, 1), (0, 8, fg, 1))):
            assert np.array_equal(outs[a][0], outs[b][0]), (a, b, "offsets")
            assert np.array_equal(outs[a][1], outs[b][1]), (a, b, "entries")
    v.set_option("fast_g", 0)
    v.set_option("trieless", 1)
    v.set_option("heavy_min", 0)
    v.set_option("fused", 1)


@pytest.mark.parametrize("mode", MODES)
def test_one_record_slots_follow_their_key_under_churn(mode):
    """Short exact topics (<= 3 words) with one local record keep it in the
    exact slot (option "exact_one"): every change of that record — a new
    SubInfo, the subscriber replaced, a second subscriber added and removed,
    remote nodes, the topic emptied and reused — must rewrite the slot.  Each
    round is folded against the oracle and byte-compared with a context that
    keeps no record in its slots (exact_one 0), fused and unfused."""
    import random
    nodes = ["n%d@h" % i for i in range(4)]
    prods = {}
    for one in (1, 0):
        p = _driver(nodes[0], mode, nodes=nodes)
        p.view.set_option("exact_one", one)
        prods[one] = p
    orc = O.TrieOracle(nodes[0])
    r = random.Random(11)
    topics = [tuple(b"w%d" % r.randrange(50) for _ in range(r.choice([1, 2, 3, 3, 4]) - 1)) + (b"t%d" % k,)
              for k in range(600)]
    subs = {}   # topic index -> {client: subscriber value}

    def val(k, node, qos):
        return [(node, True, [(topics[k], qos)])]

    for rnd in range(6):
        evs = []
        for k in range(len(topics)):
            x = r.random()
            cur = subs.setdefault(k, {})
            if not cur or x < 0.3:   # (re)subscribe a client: QoS and node may change
                sid = ("" if k % 3 else "m", b"c%d_%d" % (k, r.randrange(3)))
                node = nodes[0] if r.random() < 0.8 else r.choice(nodes[1:])
                new = val(k, node, r.randrange(3))
                evs.append(("updated", sid, cur.get(sid), new))
                cur[sid] = new
            elif x < 0.5:            # drop one
                sid = r.choice(sorted(cur))
                evs.append(("deleted", sid, cur.pop(sid)))
        for p in prods.values():
            p.apply(evs)
        orc.apply(evs)
        pubs = [("" if k % 3 else "m", topics[k]) for k in range(len(topics))] * 3
        want = [sorted(x) for x in orc.fold_batch([(mp, b"p", t) for mp, t in pubs])]
        outs = {}
        for one, p in prods.items():
            for fu in (1, 0):
                p.view.set_option("fused", fu)
                arr, words = p.view.prepare(pubs)
                recs, offs = p.match_arrays(arr, words)
                outs[one, fu] = (np.asarray(offs).copy(), np.asarray(recs).view(np.uint8).copy())
                got = p.fold_batch(pubs)
                bad = [i for i in range(len(pubs)) if sorted(got[i]) != want[i]]
                assert not bad, (rnd, one, fu, len(bad), pubs[bad[0]], sorted(got[bad[0]]), want[bad[0]])
            p.view.set_option("fused", 1)
        for key in ((1, 0), (0, 1), (0, 0)):
            assert np.array_equal(outs[1, 1][0], outs[key][0]), (rnd, key, "offsets")
            assert np.array_equal(outs[1, 1][1], outs[key][1]), (rnd, key, "entries")


@pytest.mark.parametrize("mode", MODES)
def test_reclaimed_ids_keep_parity(mode):
    """Subscribe -> unsubscribe cycles with unique client ids and words
    (paths, keys, topics dropped at each unsubscribe, words released after
    every cycle and their ids reused by the next): every cycle's publishes —
    on its own live topics and on the previous cycle's dead ones — fold to
    the oracle's entries, and the device arena does not grow."""
    from tests.test_host_engine import _cycle_events
    node = "n@h"
    prod = _driver(node, mode)
    orc = O.TrieOracle(node)
    arena = []
    for c in range(16):
        adds, dels = _cycle_events(c, n=200, node=node)
        prod.apply(adds)
        orc.apply(adds)
        pubs = []
        for cc in (c, c - 1):
            for i in range(0, 200, 3):
                u = b"u%d_%d" % (cc, i)
                pubs += [("", (b"dev", u, b"state")), ("", (b"dev", u, b"x")), ("", (b"all", u, b"y", b"z")),
                         ("", (b"jobs", u))]
        _compare_batches(prod, orc, pubs, "cycle %d" % c)
        prod.apply(dels)
        orc.apply(dels)
        prod.view.reclaim_words()
        _compare_batches(prod, orc, pubs[:100], "cycle %d after deletes" % c)
        arena.append(prod.view.stats_raw()["device_bytes"])
    assert prod.view.stats_raw()["words_released"] > 0
    assert arena[-1] <= arena[3], arena


def test_reclamation_keeps_parity_over_100k_cycles():
    """Verdict r5 item 2 on the GPU: 100,000 subscribe -> unsubscribe cycles
    (100 rounds of 1,000 subscribers with unique client ids and topic words:
    an exact topic, a '+' and a '#' filter, a $share group, every 7th on a
    remote node), words released after every round and their ids reused.
    Every round, a sample of publishes on the live topics and on the last
    round's dead ones folds to the oracle's entries; the live word, path,
    key and topic counts and the host and device bytes stay within 2x of
    the fourth round's (the tables' working size)."""
    from tests.test_host_engine import _cycle_events
    node = "n@h"
    prod = _driver(node, "records")
    orc = O.TrieOracle(node)
    first = None
    for c in range(100):
        adds, dels = _cycle_events(c, n=1000, node=node)
        prod.apply(adds)
        orc.apply(adds)
        pubs = []
        for cc in (c, c - 1):
            for i in range(0, 1000, 17):
                u = b"u%d_%d" % (cc, i)
                pubs += [("", (b"dev", u, b"state")), ("", (b"all", u, b"y")), ("", (b"jobs", u))]
        _compare_batches(prod, orc, pubs, "round %d" % c)
        st = prod.view.stats_raw()
        if c == 3:   # the tables have taken their working size (the first rounds may re-lay them out)
            first = st
        for k in ("words", "paths", "keys", "topics", "host_bytes", "device_bytes"):
            assert first is None or st[k] <= 2 * first[k] + 64, (c, k, first[k], st[k])
        prod.apply(dels)
        orc.apply(dels)
        prod.view.reclaim_words()
    st = prod.view.stats_raw()
    assert st["subs"] == 0 and st["words_released"] >= 99 * 1000, st
