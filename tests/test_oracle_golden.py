"""Pins the CPU oracle (oracle/vmq_trie_oracle.cpp) to the golden vectors
transcribed from the reference's own tests (tests/golden/make_golden.py).
CPU only."""
import pytest

from oracle import oracle as O
from tests import scenarios as S

SCENARIO_FILES = ["pattern_matching.json", "upgrade.json", "overlapping_subscriptions.json",
                  "dollar_topics.json", "shared_subscriptions.json", "quirks.json"]


def _scenarios():
    for f in SCENARIO_FILES:
        for sc in S.load(f)["scenarios"]:
            yield pytest.param(sc, id="%s:%s" % (f, sc["name"]))


@pytest.mark.parametrize("scen", list(_scenarios()))
def test_oracle_scenarios(scen):
    S.run_scenario(scen, lambda node: O.TrieOracle(node))


def test_topic_validation_kats():
    g = S.load("topic_validation.json")
    for c in g["cases"]:
        got = O.validate_topic(c["type"], c["topic"].encode())
        if "ok" in c:
            assert got == ("ok", tuple(w.encode() for w in c["ok"])), c
        else:
            assert got == ("error", c["error"]), c
    for words, want in g["contains_wildcard"]:
        assert O.contains_wildcard([w.encode() for w in words]) == want


def _ch(v):
    return [(n, [((t.encode(),), O.subinfo_repr(si)) for t, si in ents]) for n, ents in v]


def _subs(v):
    return [(n, c, [((t.encode(),), si) for t, si in ents]) for n, c, ents in v]


def test_subscriber_get_changes_kats():
    g = S.load("subscriber_changes.json")
    o = O.TrieOracle(g["self_node"])
    for k in g["get_changes"]:
        removed, added = o.get_changes(_subs(k["old"]), _subs(k["new"]))
        assert removed == _ch(k["removed"]) and added == _ch(k["added"]), k
    for k in g["subtract"]:
        removed, _ = o.get_changes(_subs(k["a"]), _subs(k["b"]))
        assert removed == _ch(k["expect"]), k


def test_pattern_pairs_agree_with_naive_matcher():
    """Every transcribed pair also matches under vmq_topic:match/2."""
    for sc in S.load("pattern_matching.json")["scenarios"]:
        f, p = sc["name"][len("pattern "):].split(" ~ ")
        assert O.naive_match(S.topic(p), S.topic(f))


def test_bench_single_lookups():
    g = S.load("reg_trie_bench.json")["single_lookups"]
    o = O.TrieOracle()
    n, mp = g["n"], g["mp"]
    pre = tuple(w.encode() for w in g["topic_prefix"])
    o.apply([("updated", (mp, str(i).encode()), None,
              [(o.self_node, True, [(pre + (str(i).encode(),), 0)])]) for i in range(1, n + 1)])
    res = o.fold_batch([(mp, b"whatever", pre + (str(i).encode(),)) for i in range(1, n + 1)])
    for i, em in enumerate(res, start=1):
        assert em == [("A", (mp, str(i).encode()), "0")]


def test_bench_fanout_subs():
    g = S.load("reg_trie_bench.json")["fanout_subs"]
    o = O.TrieOracle()
    n, mp = g["n"], g["mp"]
    t = tuple(w.encode() for w in g["topic"])
    o.apply([("updated", (mp, str(i).encode()), None, [(o.self_node, True, [(t, 0)])])
             for i in range(1, n + 1)])
    em = o.fold(mp, t)
    assert sorted(em) == sorted(("A", (mp, str(i).encode()), "0") for i in range(1, n + 1))
    o.apply([("deleted", (mp, str(i).encode()), [(o.self_node, True, [(t, 0)])])
             for i in range(1, n + 1)])
    sz = o.sizes()
    assert sz["trie_subs"] == 0 and sz["trie_subs_fanout"] == 0


def test_quirk_q1_table_state():
    """Q1 walk-through of SURVEY.md §8a: after unsubscribing a/+ the nodes
    [a,+], [a], root and the edges ([a],+), (root,a) are gone while a/+/b's
    terminal survives (unreachable)."""
    o = O.TrieOracle()
    sid = ("", b"q1")
    n = o.self_node
    o.apply([("updated", sid, None, [(n, True, [((b"a", b"+", b"b"), 0)])]),
             ("updated", sid, [(n, True, [((b"a", b"+", b"b"), 0)])],
              [(n, True, [((b"a", b"+"), 0), ((b"a", b"+", b"b"), 0)])]),
             ("updated", sid, [(n, True, [((b"a", b"+"), 0), ((b"a", b"+", b"b"), 0)])],
              [(n, True, [((b"a", b"+", b"b"), 0)])])])
    d = o.dump()
    assert 'node ""|["a","+","b"] ec=0 topic=["a","+","b"]' in d
    assert 'trie ""|["a","+"] "b" -> ["a","+","b"]' in d
    assert not any(l.startswith('node ""|root') for l in d)
    assert not any(l.startswith('trie ""|root') for l in d)
