"""CPU parity of the delta handling: the product's host engine (libvmqgpu,
host-only context) and the oracle must hold the same six logical tables —
object for object — after every event, on the golden scenarios and under
random churn that exercises Q1-Q3.  No GPU needed (no match calls)."""
import pytest

from oracle import oracle as O
from tests import harness as H
from tests import scenarios as S

SCEN_FILES = ["pattern_matching.json", "upgrade.json", "overlapping_subscriptions.json",
              "dollar_topics.json", "shared_subscriptions.json", "quirks.json"]


def _scen():
    for f in SCEN_FILES:
        for sc in S.load(f)["scenarios"]:
            yield pytest.param(sc, id="%s:%s" % (f, sc["name"]))


def _compare(prod, orc, ctx):
    a = H.normalize_product_dump(prod.view)
    b = H.normalize_oracle_dump(orc)
    if a != b:
        sa, sb = set(a), set(b)
        raise AssertionError("%s\nonly product: %s\nonly oracle: %s" % (ctx, sorted(sa - sb)[:20],
                                                                       sorted(sb - sa)[:20]))
    ps = prod.view.stats_raw()
    osz = orc.sizes()
    assert ps["subs"] == osz["stats_subs"], ctx
    assert ps["trie_edges"] == osz["trie"] and ps["trie_nodes"] == osz["trie_node"], ctx
    assert ps["trie_topics"] == osz["trie_topic"] and ps["fanout_objects"] == osz["trie_subs_fanout"], ctx


@pytest.mark.parametrize("scen", list(_scen()))
def test_golden_event_streams_same_tables(scen):
    prod = H.ProductDriver(scen["node"], device=-1)
    orc = O.TrieOracle(scen["node"])
    for i, step in enumerate(scen["steps"]):
        if "event" in step:
            ev = S.event(step["event"])
            prod.apply([ev])
            orc.apply([ev])
            _compare(prod, orc, "%s step %d" % (scen["name"], i))


@pytest.mark.parametrize("seed", range(6))
def test_random_churn_same_tables(seed):
    wl = H.ChurnWorkload(seed)
    prod = H.ProductDriver(wl.self_node, device=-1)
    orc = O.TrieOracle(wl.self_node)
    for step in range(300):
        ev = wl.event()
        prod.apply([ev])
        orc.apply([ev])
        if step % 10 == 9:
            _compare(prod, orc, "seed %d step %d" % (seed, step))
    _compare(prod, orc, "seed %d end" % seed)


def test_batched_events_equal_sequential():
    """One apply batch of many events == the same events one by one."""
    wl = H.ChurnWorkload(99)
    evs = [wl.event() for _ in range(400)]
    a = H.ProductDriver(wl.self_node, device=-1)
    a.apply(evs)
    orc = O.TrieOracle(wl.self_node)
    orc.apply(evs)
    _compare(a, orc, "batched")


def test_invalid_share_op_rejects_batch():
    from vernemq_amd import _lib
    prod = H.ProductDriver("n@h", device=-1)
    with pytest.raises(_lib.VmqgError) as ei:
        prod.view.apply_ops([("add", ("", b"x"), (b"a",), 0, "n@h"),
                             ("add", ("", b"x"), (b"$share", b"g"), 0, "n@h")])
    assert ei.value.rc == _lib.E_INVAL
    assert prod.view.stats_raw()["subs"] == 0


def test_bulk_growth_rebuilds():
    """Tables grow past their initial capacity (full re-layout) and stay equal."""
    prod = H.ProductDriver("n@h", device=-1)
    orc = O.TrieOracle("n@h")
    evs = [("updated", ("", b"c%d" % i), None,
            [("n@h", True, [((b"dev", b"%d" % i, b"+", b"#"), i % 3), ((b"x%d" % (i % 97),), 1)])])
           for i in range(6000)]
    prod.apply(evs)
    orc.apply(evs)
    assert prod.view.stats_raw()["rebuilds"] >= 2
    _compare(prod, orc, "bulk")


def test_record_epochs_refuse_stale_ranges():
    """vmqg_epoch / vmqg_records_at on the host engine: an apply that rewrites
    record slots makes the older epochs' record tables unavailable (range
    results of those epochs must be matched again); an epoch with no
    record-writing apply after it stays valid."""
    from vernemq_amd import _lib
    node = "n@h"
    prod = H.ProductDriver(node, device=-1)
    v = prod.view
    sub = lambda cid, t, q: ("updated", ("", cid), None, [(node, True, [(t, q)])])
    prod.apply([sub(b"w%d" % i, (b"a", b"+"), 1) for i in range(10)])
    e1 = v.epoch()
    assert len(v.records(epoch=e1)) > 0
    with pytest.raises(_lib.VmqgError):
        v.records(epoch=e1 + 1)                       # not yet applied
    prod.apply([("deleted", ("", b"w3"), [(node, True, [((b"a", b"+"), 1)])])])
    e2 = v.epoch()
    assert e2 == e1 + 1
    with pytest.raises(_lib.VmqgError):
        v.records(epoch=e1)                           # a slot was rewritten
    recs = v.records(epoch=e2)
    assert len(recs) > 0


def _mp_events(n_mps, node="n@h", seed=5):
    """Per mountpoint t<k>: a wildcard, a '#', a $share and an exact filter
    (different subscribers), remote subscribers on every 7th; every 3rd
    mountpoint later loses two of them (deletes walk the trie paths back)."""
    import random
    r = random.Random(seed)
    adds, dels = [], []
    for k in range(n_mps):
        mp = "t%d" % k
        w = (b"w%d" % r.randrange(4), b"x%d" % r.randrange(3))
        subs = [(b"a", (w[0], b"+"), r.randint(0, 2)), (b"b", (w[0], b"#"), 1),
                (b"c", (b"$share", b"g%d" % (k % 3), w[0], w[1]), 0), (b"d", w, 2)]
        for cid, t, q in subs:
            nd = "n%d@h" % (1 + k % 3) if (k % 7 == 0 and cid == b"d") else node
            adds.append(("updated", (mp, cid), None, [(nd, True, [(t, q)])]))
        if k % 3 == 0:
            for cid, t, q in subs[:2]:
                dels.append(("deleted", (mp, cid), [(node, True, [(t, q)])]))
    return adds, dels


def test_mountpoints_grow_past_the_initial_roots():
    """vmq_reg_trie has no mountpoint limit (a mountpoint is part of every
    key, vmq_reg_trie.erl:60, 279-281, 320): 5,000 mountpoints on a context
    created with 16 roots grow the root range (re-layouts renumbering every
    path) and the tables stay equal to the oracle's, through the deletes too."""
    node = "n@h"
    prod = H.ProductDriver(node, device=-1, max_mountpoints=16)
    orc = O.TrieOracle(node)
    adds, dels = _mp_events(5000, node)
    for lo in range(0, len(adds), 4000):   # several applies, each growing the roots
        prod.apply(adds[lo:lo + 4000])
        orc.apply(adds[lo:lo + 4000])
    _compare(prod, orc, "5000 mountpoints")
    prod.apply(dels)
    orc.apply(dels)
    _compare(prod, orc, "5000 mountpoints after deletes")
    assert prod.view.stats_raw()["paths"] >= 5000


@pytest.mark.parametrize("seed", range(3))
def test_random_churn_over_growing_mountpoints(seed):
    """Churn whose clients live on 40 mountpoints, on a context created with
    2 roots: growth happens between and inside event batches."""
    wl = H.ChurnWorkload(seed, mps=[""] + ["m%d" % i for i in range(39)])
    prod = H.ProductDriver(wl.self_node, device=-1, max_mountpoints=2)
    orc = O.TrieOracle(wl.self_node)
    for step in range(40):
        evs = [wl.event() for _ in range(8)]
        prod.apply(evs)
        orc.apply(evs)
        _compare(prod, orc, "seed %d step %d" % (seed, step))


def _cycle_events(c, n=300, node="n@h"):
    """Cycle c: n subscribers with unique client ids subscribe to filters
    holding words of their own (an exact topic, a '+' filter, a '#' filter,
    a $share group named after the cycle, a remote subscription), then the
    deletes of all of them."""
    subs = []
    for i in range(n):
        u = b"u%d_%d" % (c, i)
        t = [((b"dev", u, b"state"), 1), ((b"dev", u, b"+"), 0), ((b"all", u, b"#"), 2)]
        if i % 10 == 0:
            t.append(((b"$share", b"g%d" % c, b"jobs", u), 1))
        nd = "n2@h" if i % 7 == 0 else node
        subs.append((("", b"client_%d_%d" % (c, i)), [(nd, True, sorted(t))]))
    adds = [("updated", sid, None, v) for sid, v in subs]
    dels = [("deleted", sid, v) for sid, v in subs]
    return adds, dels


def test_reclamation_follows_the_live_set():
    """Subscribe -> unsubscribe cycles with unique client ids and unique
    topic words: vmq_reg_trie deletes its rows with their last value
    (vmq_reg_trie.erl:417-441, 472-539), so its tables track the live set;
    here paths, keys, topics and (after vmqg_dict_release) words are dropped
    too and their ids reused — the counts stay within 2x of one cycle's, the
    tables equal the oracle's throughout, and the host bytes stop growing."""
    node = "n@h"
    prod = H.ProductDriver(node, device=-1)
    orc = O.TrieOracle(node)
    peak, hb = None, []
    for c in range(60):
        adds, dels = _cycle_events(c, node=node)
        prod.apply(adds)
        orc.apply(adds)
        st = prod.view.stats_raw()
        if peak is None:
            peak = {k: st[k] for k in ("paths", "keys", "topics", "words")}
        for k, v in peak.items():
            assert st[k] <= 2 * v + 16, (c, k, st[k], v)
        if c % 15 == 7:
            _compare(prod, orc, "cycle %d live" % c)
        prod.apply(dels)
        orc.apply(dels)
        prod.view.reclaim_words()
        st = prod.view.stats_raw()
        assert st["keys"] == 0 and st["topics"] == 0, (c, st["keys"], st["topics"])
        assert st["paths"] <= 1024 + 4 and st["words"] <= 3 + 4, (c, st["paths"], st["words"])
        hb.append(st["host_bytes"])
        if c % 15 == 14:
            _compare(prod, orc, "cycle %d empty" % c)
    assert st["words_released"] >= 59 * 300
    assert hb[-1] <= hb[10] * 1.25 + (1 << 20), (hb[10], hb[-1])
