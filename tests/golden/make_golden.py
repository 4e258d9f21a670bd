"""Writes tests/golden/*.json — golden vectors hand-transcribed from the
reference's OWN tests (file:line relative to /root/reference).  These are
data (inputs + expected outputs), not reference source.  Re-run with
``python tests/golden/make_golden.py`` after editing; the JSON is committed.

The reference (Erlang/OTP) cannot run here, so the expected
outputs are the assertions the reference tests make, restated at the matcher
boundary (``vmq_reg_view:fold/4`` emissions):

* an MQTT delivery of a QoS-q message to client C  ⇔  an emission
  ``{SubscriberId, SubInfo}`` (kind "A") in the fold of that topic;
* no delivery ⇔ no emission.

Scenario files whose expectations are NOT asserted by any reference test
(quirks Q1–Q3, multi-node ``$share`` multiplicity) carry ``"pinned": false``
and cite the source lines they were derived from instead.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
N0 = "nonode@nohost"   # node() under eunit / the single-node CT suites


def A(mp, client, si):
    return ["A", [mp, client], si]


def B(node, group, mp, client, si):
    return ["B", node, group, [mp, client], si]


def sub(mp, client, topics, node=N0, old=None, clean=True):
    """{updated, {vmq,subscriber}, SubscriberId, Old, New} for one node."""
    return {"updated": {"sid": [mp, client], "old": old, "new": [[node, clean, topics]]}}


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


# 1. vmq_publish_SUITE.erl:459-481 pattern_matching_test — each pair is run
#    through pattern_test/3 (:483-509): subscribe, publish (delivered),
#    unsubscribe, subscribe again (delivered again, as retained).
PAIRS = [
    ("#", "test/topic"), ("#", "/test/topic"), ("foo/#", "foo/bar/baz"),
    ("foo/+/baz", "foo/bar/baz"), ("foo/+/baz/#", "foo/bar/baz"),
    ("foo/+/baz/#", "foo/bar/baz/bar"), ("foo/foo/baz/#", "foo/foo/baz/bar"),
    ("foo/#", "foo"), ("/#", "/foo"), ("test/topic/", "test/topic/"),
    ("test/topic/+", "test/topic/"),
    ("+/+/+/+/+/+/+/+/+/+/test", "one/two/three/four/five/six/seven/eight/nine/ten/test"),
    ("#", "test////a//topic"), ("#", "/test////a//topic"), ("foo/#", "foo//bar///baz"),
    ("foo/+/baz", "foo//baz"), ("foo/+/baz//", "foo//baz//"), ("foo/+/baz/#", "foo//baz"),
    ("foo/+/baz/#", "foo//baz/bar"), ("foo//baz/#", "foo//baz/bar"),
    ("foo/foo/baz/#", "foo/foo/baz/bar"), ("/#", "////foo///bar"),
]
scen = []
for f, p in PAIRS:
    c = "pattern-sub-test"
    on = [[N0, True, [[f, 0]]]]
    off = [[N0, True, []]]
    scen.append({
        "name": "pattern %s ~ %s" % (f, p), "node": N0,
        "source": "vmq_publish_SUITE.erl:459-509",
        "steps": [
            {"event": sub("", c, [[f, 0]])},
            {"fold": ["", p], "expect": [A("", c, "0")]},
            {"event": {"updated": {"sid": ["", c], "old": on, "new": off}}},
            {"fold": ["", p], "expect": []},
            {"event": {"updated": {"sid": ["", c], "old": off, "new": on}}},
            {"fold": ["", p], "expect": [A("", c, "0")]},
        ]})
write("pattern_matching.json", {"pinned": True, "scenarios": scen})

# 2. vmq_topic.erl:138-201 validate_topic/2 KATs, :203-205 shared, :212-215
#    contains_wildcard.
VT = [
    ("subscribe", "a/b/c", ["a", "b", "c"]), ("subscribe", "/a/b", ["", "a", "b"]),
    ("subscribe", "test/topic/", ["test", "topic", ""]),
    ("subscribe", "test////a//topic", ["test", "", "", "", "a", "", "topic"]),
    ("subscribe", "/test////a//topic", ["", "test", "", "", "", "a", "", "topic"]),
    ("publish", "foo//bar///baz", ["foo", "", "bar", "", "", "baz"]),
    ("publish", "foo//baz//", ["foo", "", "baz", "", ""]),
    ("publish", "foo//baz", ["foo", "", "baz"]),
    ("publish", "foo//baz/bar", ["foo", "", "baz", "bar"]),
    ("publish", "////foo///bar", ["", "", "", "", "foo", "", "", "bar"]),
    ("subscribe", "/+/x", ["", "+", "x"]), ("subscribe", "/a/b/c/#", ["", "a", "b", "c", "#"]),
    ("subscribe", "#", ["#"]), ("subscribe", "foo/#", ["foo", "#"]),
    ("subscribe", "foo/+/baz", ["foo", "+", "baz"]),
    ("subscribe", "foo/+/baz/#", ["foo", "+", "baz", "#"]),
    ("subscribe", "foo/foo/baz/#", ["foo", "foo", "baz", "#"]),
    ("subscribe", "/#", ["", "#"]), ("subscribe", "test/topic/+", ["test", "topic", "+"]),
    ("subscribe", "+/+/+/+/+/+/+/+/+/+/test", ["+"] * 10 + ["test"]),
    ("publish", "test/#-", "no_#_allowed_in_word"), ("publish", "test/+-", "no_+_allowed_in_word"),
    ("publish", "test/+/", "no_+_allowed_in_publish"), ("publish", "test/#", "no_#_allowed_in_publish"),
    ("subscribe", "a/#/c", "no_#_allowed_in_word"), ("subscribe", "#testtopic", "no_#_allowed_in_word"),
    ("subscribe", "testtopic#", "no_#_allowed_in_word"), ("subscribe", "+testtopic", "no_+_allowed_in_word"),
    ("subscribe", "testtopic+", "no_+_allowed_in_word"),
    ("subscribe", "#testtopic/test", "no_#_allowed_in_word"),
    ("subscribe", "testtopic#/test", "no_#_allowed_in_word"),
    ("subscribe", "+testtopic/test", "no_+_allowed_in_word"),
    ("subscribe", "testtopic+/test", "no_+_allowed_in_word"),
    ("subscribe", "/test/#testtopic", "no_#_allowed_in_word"),
    ("subscribe", "/test/testtopic#", "no_#_allowed_in_word"),
    ("subscribe", "/test/+testtopic", "no_+_allowed_in_word"),
    ("subscribe", "/testtesttopic+", "no_+_allowed_in_word"),
    ("subscribe", "$share/mygroup", "invalid_shared_subscription"),
    ("subscribe", "$share/mygroup/a/b", ["$share", "mygroup", "a", "b"]),
    ("publish", "", "no_empty_topic_allowed"),  # :82-83
]
write("topic_validation.json", {
    "pinned": True, "source": "vmq_topic.erl:138-205",
    "cases": [{"type": t, "topic": s, "ok": r} if isinstance(r, list) else
              {"type": t, "topic": s, "error": r} for t, s, r in VT],
    "contains_wildcard": [[["a", "+", "b"], True], [["#"], True], [["a", "b", "c"], False]],
})

# 3. vmq_subscriber.erl:203-303 eunit KATs (topics are atoms there; here the
#    single-word topic [<<"a">>] stands for atom a — only equality/order matter).
def T(x):
    return x
write("subscriber_changes.json", {
    "pinned": True, "source": "vmq_subscriber.erl:203-311", "self_node": N0,
    "subtract": [
        {"a": [["node_a", True, [["a", 0], ["b", 1], ["c", 2]]], ["node_b", True, [["d", 1], ["e", 2]]]],
         "b": [["node_a", True, [["b", 1], ["c", 2]]], ["node_b", True, [["e", 2]]]],
         "expect": [["node_a", [["a", 0]]], ["node_b", [["d", 1]]]]},
        {"a": [["node_a", True, [["a", 0], ["b", 1], ["c", 2]]], ["node_b", True, [["d", 1], ["e", 2]]]],
         "b": [["node_a", True, []], ["node_b", True, []]],
         "expect": [["node_a", [["a", 0], ["b", 1], ["c", 2]]], ["node_b", [["d", 1], ["e", 2]]]]},
        {"a": [["node_a", True, [["a", 0], ["b", 1], ["c", 2]]], ["node_b", True, [["d", 1], ["e", 2]]]],
         "b": [["node_a", True, [["a", 0], ["b", 1], ["c", 2]]], ["node_b", True, [["d", 1], ["e", 2]]]],
         "expect": []},
    ],
    "get_changes": [
        {"old": [["node_a", True, [["a", 1], ["b", 1]]]], "new": [["node_a", True, [["b", 1]]]],
         "removed": [["node_a", [["a", 1]]]], "added": []},
        {"old": [["node_a", True, [["a", 1]]], ["node_b", True, [["b", 1]]]],
         "new": [["node_a", True, [["a", 1]]], ["node_c", True, [["c", 1]]]],
         "removed": [["node_b", [["b", 1]]]], "added": [["node_c", [["c", 1]]]]},
        {"old": [["node_a", True, [["a", 1]]], ["node_b", True, [["b", 1]]], ["node_c", True, [["c", 1]]]],
         "new": [["node_b", True, [["b", 1]]]],
         "removed": [["node_a", [["a", 1]]], ["node_c", [["c", 1]]]], "added": []},
        {"old": [["node_b", True, [["b", 1]]], ["node_c", True, [["c", 1]]]],
         "new": [["node_a", True, [["a", 1]]], ["node_c", True, [["c", 1]]]],
         "removed": [["node_b", [["b", 1]]]], "added": [["node_a", [["a", 1]]]]},
    ],
    "change_node": [
        {"subs": [["node_a", False, [["a", 1], ["b", 1]]], ["node_b", False, [["c", 2]]]],
         "node": "node_a", "new_node": "node_b", "clean": False,
         "expect": [["node_b", False, [["a", 1], ["b", 1], ["c", 2]]]]},
    ],
    "change_node_all": [
        {"subs": [["node_a", False, [["a", 1], ["b", 1]]], ["node_b", False, [["b", 2], ["c", 2]]]],
         "new_node": "node_c", "clean": False,
         "expect": [[["node_c", False, [["a", 1], ["b", 2], ["c", 2]]]], ["node_a", "node_b"]]},
    ],
    "add": [
        {"subs": [[N0, True, []]], "topics": [["a", 1], ["b", 2]],
         "expect": [[[N0, True, [["a", 1], ["b", 2]]]], True]},
        {"subs": [[N0, True, [["a", 1]]]], "topics": [["b", 2]],
         "expect": [[[N0, True, [["a", 1], ["b", 2]]]], True]},
        {"subs": [[N0, True, [["a", 1], ["b", 1]]]], "topics": [["b", 2]],
         "expect": [[[N0, True, [["a", 1], ["b", 2]]]], True]},
        {"subs": [[N0, True, [["a", 1], ["b", 2]]]], "topics": [["b", 2]],
         "expect": [[[N0, True, [["a", 1], ["b", 2]]]], False]},
    ],
    "remove": [
        {"subs": [[N0, True, []]], "topics": ["a"], "expect": [[[N0, True, []]], False]},
        {"subs": [[N0, True, [["a", 1]]]], "topics": ["a"], "expect": [[[N0, True, []]], True]},
        {"subs": [[N0, True, [["a", 1], ["b", 2]]]], "topics": ["a"],
         "expect": [[[N0, True, [["b", 2]]]], True]},
    ],
    "maybe_convert_v0": [
        {"v0": [["a", 0, "node_a"], ["b", 1, "node_b"], ["c", 2, "node_c"]],
         "expect": [["node_a", True, [["a", 0]]], ["node_b", True, [["b", 1]]],
                    ["node_c", True, [["c", 2]]], [N0, False, []]]},
    ],
})

# 4. vmq_reg_trie_bench_SUITE.erl:114-150 bench_single_lookups (each unique
#    topic folds to exactly [{{"a", I}, 0}]) and :152-214 bench_fanout_subs
#    (the fold returns all N; after deleting all, vmq_trie_subs and the fanout
#    table are empty).  N = 1000 is the suite's first size (:98, :153).
write("reg_trie_bench.json", {
    "pinned": True, "source": "vmq_reg_trie_bench_SUITE.erl:97-229",
    "single_lookups": {"n": 1000, "mp": "a", "topic_prefix": ["unique", "topic"], "qos": 0},
    "fanout_subs": {"n": 1000, "mp": "a", "topic": ["some", "topic"], "qos": 0},
})

# 5. vmq_upgrade_SUITE.erl:34-51 — a v0-format record routes as [{SubscriberId, 1}].
write("upgrade.json", {"pinned": True, "source": "vmq_upgrade_SUITE.erl:34-51", "scenarios": [{
    "name": "v0_to_v1_subscriber_format", "node": N0,
    "steps": [
        {"event": {"updated": {"sid": ["", "test-client"], "old": None,
                               "new": {"v0": [["a/b/c", 1, N0]]}}}},
        {"fold": ["", "a/b/c"], "expect": [A("", "test-client", "1")]},
    ]}]})

# 6. vmq_subscribe_SUITE.erl:121-228 subscription_ids: overlapping
#    subscriptions give one emission per matching subscription; :68-109
#    no_local: the matcher still emits (vmq_reg:publish/3 drops it, vmq_reg.erl:327-329).
def v5(qos, sub_id=None, no_local=False):
    o = {"no_local": no_local, "rap": False, "retain_handling": "send_retain"}
    if sub_id is not None:
        o["sub_id"] = sub_id
    return [qos, o]


def v5r(qos, sub_id=None, no_local=False):
    items = ["no_local=>%s" % ("true" if no_local else "false"), "rap=>false",
             "retain_handling=>send_retain"]
    if sub_id is not None:
        items.append("sub_id=>%d" % sub_id)
    return "{%d,#{%s}}" % (qos, ",".join(items))


BT = "subscription_ids_topic"
C = "subscription-ids-client"
topics = [["%s/l1/#" % BT, v5(0, 5)], ["%s/l1/l2" % BT, v5(0, 6)], ["%s/+/t6" % BT, v5(0, 7)],
          ["%s/t5/t6" % BT, v5(0, 7)], ["%s/no-overlap" % BT, v5(0, 8)]]
nl = "subscribe_no_local_test_topic"
write("overlapping_subscriptions.json", {"pinned": True, "scenarios": [
    {"name": "subscription_ids", "node": N0, "source": "vmq_subscribe_SUITE.erl:121-228",
     "steps": [
         {"event": sub("", C, topics)},
         {"fold": ["", BT + "/l1/l2"], "expect": [A("", C, v5r(0, 5)), A("", C, v5r(0, 6))]},
         {"fold": ["", BT + "/l1/notl2"], "expect": [A("", C, v5r(0, 5))]},
         {"fold": ["", BT + "/t5/t6"], "expect": [A("", C, v5r(0, 7)), A("", C, v5r(0, 7))]},
         {"fold": ["", BT + "/nott5/t6"], "expect": [A("", C, v5r(0, 7))]},
         {"fold": ["", BT + "/no-overlap"], "expect": [A("", C, v5r(0, 8))]},
     ]},
    {"name": "subscribe_no_local", "node": N0, "source": "vmq_subscribe_SUITE.erl:68-109",
     "steps": [
         {"event": sub("", "nl-client", [[nl + "/nolocalfalse", v5(0)],
                                         [nl + "/nolocaltrue", v5(0, no_local=True)]])},
         {"fold": ["", nl + "/nolocalfalse"], "expect": [A("", "nl-client", v5r(0))]},
         {"fold": ["", nl + "/nolocaltrue"], "expect": [A("", "nl-client", v5r(0, no_local=True))]},
     ]},
]})

# 7. vmq_publish_SUITE.erl:582-591 drop_dollar_topic_publish (no subscriber:
#    nothing); with subscribers, the MQTT-4.7.2-1 clauses vmq_reg_trie.erl:283-288
#    keep '#' and '+/...' filters away from '$' topics (derived, unpinned part).
write("dollar_topics.json", {"pinned": True, "scenarios": [
    {"name": "drop_dollar_topic_publish", "node": N0, "source": "vmq_publish_SUITE.erl:582-591",
     "steps": [{"fold": ["", "$test/drop"], "expect": []}]},
    {"name": "dollar_rule", "node": N0, "pinned": False,
     "source": "vmq_reg_trie.erl:283-288",
     "steps": [
         {"event": sub("", "d1", [["#", 0], ["+/drop", 0], ["$test/#", 1], ["$test/+", 2],
                                  ["$test/drop", 0], ["+/+", 1]])},
         {"fold": ["", "$test/drop"],
          "expect": [A("", "d1", "1"), A("", "d1", "2"), A("", "d1", "0")]},
         {"fold": ["", "x/drop"], "expect": [A("", "d1", "0"), A("", "d1", "0"), A("", "d1", "1")]},
     ]},
]})

# 8. Shared subscriptions.  vmq_publish_SUITE.erl:653-738: two members of
#    $share/group/shared_sub_topic on one node — the fold yields both (the
#    member choice happens later in vmq_shared_subscriptions).  The cluster
#    cases (vmq_cluster_SUITE.erl:494-608, :662-711) place members on several
#    nodes; that every member is found is pinned, the per-node multiplicity
#    (Q2, vmq_reg_trie.erl:68-72, 301-303) is not.
G = "$share/group/shared_sub_topic"
write("shared_subscriptions.json", {"pinned": True, "scenarios": [
    {"name": "shared_subscription_online_first", "node": N0,
     "source": "vmq_publish_SUITE.erl:690-738",
     "steps": [
         {"event": sub("", "sub-offline", [[G, 1]], clean=False)},
         {"event": sub("", "sub-online", [[G, 1]], clean=False)},
         {"fold": ["", "shared_sub_topic"],
          "expect": [B(N0, "group", "", "sub-offline", "1"), B(N0, "group", "", "sub-online", "1")]},
     ]},
    {"name": "cluster_shared_three_nodes (Q2 multiplicity)", "node": "node1@127.0.0.1",
     "pinned": False, "source": "vmq_cluster_SUITE.erl:494-608; vmq_reg_trie.erl:68-72,301-303",
     "steps": (
         [{"event": sub("", "subscriber-%d" % i, [["$share/share/sharedtopic", 1]],
                        node=["node1@127.0.0.1", "node2@127.0.0.1", "node3@127.0.0.1"][i % 3])}
          for i in range(10)] +
         [{"fold": ["", "sharedtopic"],
           "expect": [B(["node1@127.0.0.1", "node2@127.0.0.1", "node3@127.0.0.1"][i % 3],
                        "share", "", "subscriber-%d" % i, "1")
                      for i in range(10) for _ in range(3)]}])},
    {"name": "routing_table_survives_node_restart", "node": "node1@127.0.0.1",
     "source": "vmq_cluster_SUITE.erl:662-711",
     "steps": [
         {"event": {"updated": {"sid": ["", "restart-node-test-subscriber"], "old": None,
                                "new": [["node2@127.0.0.1", True,
                                         [["$share/group/sharedtopic", 1], ["topic/sub", 1]]]]}}},
         {"fold": ["", "topic/sub"], "expect": [["C", "node2@127.0.0.1"]]},
         {"fold": ["", "sharedtopic"],
          "expect": [B("node2@127.0.0.1", "group", "", "restart-node-test-subscriber", "1")]},
     ]},
]})

# 9. Quirks Q1–Q3 — NOT asserted by any reference test; the
#    expectations are derived by reading vmq_reg_trie.erl (lines cited).
on = lambda ts: [[N0, True, ts]]
write("quirks.json", {"pinned": False, "scenarios": [
    {"name": "Q1 reachability loss under churn", "node": N0,
     "source": "vmq_reg_trie.erl:318-337 (edge_count=0 overwrite), :417-441",
     "steps": [
         {"event": sub("", "q1", [["a/+/b", 0]])},
         {"fold": ["", "a/x/b"], "expect": [A("", "q1", "0")]},
         {"event": {"updated": {"sid": ["", "q1"], "old": on([["a/+/b", 0]]),
                                "new": on([["a/+", 0], ["a/+/b", 0]])}}},
         {"fold": ["", "a/x"], "expect": [A("", "q1", "0")]},
         {"event": {"updated": {"sid": ["", "q1"], "old": on([["a/+", 0], ["a/+/b", 0]]),
                                "new": on([["a/+/b", 0]])}}},
         {"fold": ["", "a/x/b"], "expect": []},
         {"event": sub("", "q1b", [["a/+/b", 1]])},
         {"fold": ["", "a/x/b"], "expect": []},
     ]},
    {"name": "Q2 $share duplication across nodes", "node": N0,
     "source": "vmq_reg_trie.erl:68-72, 253-256, 301-303",
     "steps": [
         {"event": sub("", "m1", [["$share/g/t/+", 1]], node=N0)},
         {"event": sub("", "m2", [["$share/g/t/+", 2]], node="other@host")},
         {"fold": ["", "t/x"], "expect": [B(N0, "g", "", "m1", "1"), B(N0, "g", "", "m1", "1"),
                                          B("other@host", "g", "", "m2", "2"),
                                          B("other@host", "g", "", "m2", "2")]},
     ]},
    {"name": "Q3 value-blind delete of a single subscriber", "node": N0,
     "source": "vmq_reg_trie.erl:494-495",
     "steps": [
         {"event": sub("", "q3", [["x/y", 1]])},
         {"event": {"deleted": {"sid": ["", "q3"], "old": on([["x/y", 2]])}}},
         {"fold": ["", "x/y"], "expect": []},
     ]},
    {"name": "remote exact + remote wildcard dedupe", "node": N0,
     "source": "vmq_reg_trie.erl:78-84, 503-520",
     "steps": [
         {"event": sub("", "r1", [["r/s", 0]], node="n2@h")},
         {"event": sub("", "r2", [["r/+", 0], ["#", 1]], node="n2@h")},
         {"event": sub("", "r3", [["r/#", 0]], node="n3@h")},
         {"fold": ["", "r/s"], "expect": [["C", "n2@h"], ["C", "n3@h"]]},
         {"fold": ["", "q"], "expect": [["C", "n2@h"]]},
     ]},
]})
print("golden fixtures written to", HERE)
