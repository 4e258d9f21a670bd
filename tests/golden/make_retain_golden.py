"""Writes tests/golden/retain.json — golden vectors for the retained-message
store (vmq_retain_srv), hand-transcribed from the reference's OWN tests
(file:line relative to /root/reference).  Data only (inputs + expected
outputs), not reference source.  Re-run with
``python tests/golden/make_retain_golden.py``; the JSON is committed.

The reference (Erlang/OTP) cannot run here, so the expected outputs are what
the reference tests assert, restated at the store boundary
(vmq_retain_srv:match_fold/4): a client subscribing to F receives the
retained message of topic T  <=>  match_fold(F) folds over {T, Payload}.

* pinned   — vmq_publish_SUITE.erl:459-509 (pattern_test/3: after the
  re-subscribe the retained publish of PubTopic is delivered, so
  vmq_topic:match(PubTopic, SubTopic) holds on the retained path for all
  22 pairs) and vmq_retain_SUITE.erl (retain set / repeat / clear /
  wildcard / qos1-then-qos0 replacement).
* unpinned — behaviour read from vmq_retain_srv.erl:63-99, :239-242 and
  vmq_topic.erl:53-65 that no reference test asserts (mountpoint isolation,
  '#' also matching its parent level, no MQTT-4.7.2-1 '$' rule on this path,
  has_wildcard/1 treating a non-final '#' as a literal word).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

PAIRS = [   # vmq_publish_SUITE.erl:459-481, (SubTopic, PubTopic)
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


def ins(t, p, mp=""):
    return {"insert": [mp, t, p]}


def dele(t, mp=""):
    return {"delete": [mp, t]}


def fold(f, expect, mp=""):
    return {"fold": [mp, f], "expect": [list(e) for e in expect]}


scen = []
for f, p in PAIRS:
    scen.append({"name": "pattern %s ~ %s" % (f, p), "pinned": True, "source": "vmq_publish_SUITE.erl:459-509",
                 "steps": [ins(p, "message"), fold(f, [(p, "message")])]})

T = "retain/qos0/test"
scen += [
    {"name": "retain_qos0_test", "pinned": True, "source": "vmq_retain_SUITE.erl:75-89",
     "steps": [ins(T, "retained message"), fold(T, [(T, "retained message")])]},
    {"name": "retain_qos0_repeated_test", "pinned": True, "source": "vmq_retain_SUITE.erl:90-112",
     "steps": [ins("retain/qos0/reptest", "retained message"),
               fold("retain/qos0/reptest", [("retain/qos0/reptest", "retained message")]),
               fold("retain/qos0/reptest", [("retain/qos0/reptest", "retained message")])]},
    # an empty retained payload deletes the key (vmq_reg.erl:274-278)
    {"name": "retain_qos0_clear_test", "pinned": True, "source": "vmq_retain_SUITE.erl:130-158",
     "steps": [ins("retain/clear/test", "retained message"),
               fold("retain/clear/test", [("retain/clear/test", "retained message")]),
               dele("retain/clear/test"), fold("retain/clear/test", [])]},
    {"name": "publish_empty_retained_msg_test", "pinned": True, "source": "vmq_retain_SUITE.erl:178-203",
     "steps": [ins("retain/clear/emptytest", "retained message"),
               fold("retain/clear/emptytest", [("retain/clear/emptytest", "retained message")]),
               dele("retain/clear/emptytest"), fold("retain/clear/emptytest", [])]},
    # the second retained publish replaces the first (ets set)
    {"name": "retain_qos1_qos0_test", "pinned": True, "source": "vmq_retain_SUITE.erl:159-177",
     "steps": [ins("retain/qos1/test", "retained message qos1"), ins("retain/qos1/test", "retained message"),
               fold("retain/qos1/test", [("retain/qos1/test", "retained message")])]},
    {"name": "retain_wildcard_test", "pinned": True, "source": "vmq_retain_SUITE.erl:204-220",
     "steps": [ins("retainwildcard/wildcard/test", "retained message"),
               fold("retainwildcard/+/#", [("retainwildcard/wildcard/test", "retained message")])]},
]

U = "vmq_retain_srv.erl:63-99,239-242; vmq_topic.erl:53-65"
scen += [
    {"name": "mountpoints are separate tables", "pinned": False, "source": U,
     "steps": [ins("a/b", "m0"), ins("a/b", "m1", mp="tenant1"),
               fold("a/#", [("a/b", "m0")]), fold("a/#", [("a/b", "m1")], mp="tenant1"),
               fold("a/b", [("a/b", "m1")], mp="tenant1"), fold("a/b", [], mp="other")]},
    {"name": "'#' matches its parent level and everything below", "pinned": False, "source": U,
     "steps": [ins("a", "p"), ins("a/b", "c1"), ins("a/b/c", "c2"), ins("ab", "x"),
               fold("a/#", [("a", "p"), ("a/b", "c1"), ("a/b/c", "c2")]),
               fold("#", [("a", "p"), ("a/b", "c1"), ("a/b/c", "c2"), ("ab", "x")]),
               fold("a/+", [("a/b", "c1")]), fold("a/+/#", [("a/b", "c1"), ("a/b/c", "c2")])]},
    {"name": "no '$' rule on the retained path", "pinned": False, "source": U,
     "steps": [ins("$SYS/broker/uptime", "u"), ins("t", "t"),
               fold("#", [("$SYS/broker/uptime", "u"), ("t", "t")]),
               fold("+/broker/+", [("$SYS/broker/uptime", "u")])]},
    {"name": "'+' matches an empty level, not a missing one", "pinned": False, "source": U,
     "steps": [ins("a//c", "e"), ins("a/c", "m"), ins("a", "s"),
               fold("a/+/c", [("a//c", "e")]), fold("a/+", [("a/c", "m")]), fold("+", [("a", "s")])]},
    {"name": "a non-final '#' is a literal word (exact lookup)", "pinned": False, "source": U,
     "steps": [ins("a/x", "m"), fold("a/#/x", []), fold("#/a", [])]},
    {"name": "delete, re-insert, replace", "pinned": False, "source": U,
     "steps": [ins("k/1", "v1"), ins("k/2", "v2"), dele("k/1"), fold("k/+", [("k/2", "v2")]),
               ins("k/1", "v3"), ins("k/2", "v4"), fold("k/+", [("k/1", "v3"), ("k/2", "v4")]),
               dele("k/9"), dele("k/1"), dele("k/1"), fold("k/#", [("k/2", "v4")]), fold("k/1", [])]},
    {"name": "exact filters", "pinned": False, "source": U,
     "steps": [ins("x/y/z", "v"), fold("x/y/z", [("x/y/z", "v")]), fold("x/y", []), fold("x/y/z/", []),
               fold("x/y/z/w", [])]},
]

with open(os.path.join(HERE, "retain.json"), "w") as fh:
    json.dump({"scenarios": scen}, fh, indent=1, sort_keys=True)
    fh.write("\n")
