"""Decoding of the golden scenario fixtures (tests/golden/*.json) into the
Python term conventions documented in oracle/oracle.py, and a driver-agnostic
runner: the same scenario runs against the oracle (CPU, checker) and against
the product view (GPU, tests marked gpu)."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def topic(s):
    return tuple(w.encode() for w in s.split("/"))


def subinfo(v):
    if isinstance(v, int):
        return v
    return (v[0], dict(v[1]))


def subs(v):
    if v is None or v == "$deleted":
        return v
    if isinstance(v, dict):
        return ("v0", [(topic(t), subinfo(si), node) for t, si, node in v["v0"]])
    return [(node, clean, [(topic(t), subinfo(si)) for t, si in ts]) for node, clean, ts in v]


def event(ev):
    (kind, body), = ev.items()
    sid = (body["sid"][0], body["sid"][1].encode())
    if kind == "updated":
        return ("updated", sid, subs(body["old"]), subs(body["new"]))
    return ("deleted", sid, subs(body["old"]))


def emission(e):
    if e[0] == "A":
        return ("A", (e[1][0], e[1][1].encode()), e[2])
    if e[0] == "B":
        return ("B", e[1], e[2].encode(), (e[3][0], e[3][1].encode()), e[4])
    return ("C", e[1])


def run_scenario(scen, make_driver):
    """make_driver(node) -> object with apply(events) and fold(mp, topic)."""
    drv = make_driver(scen["node"])
    for i, step in enumerate(scen["steps"]):
        if "event" in step:
            drv.apply([event(step["event"])])
        else:
            mp, t = step["fold"]
            got = sorted(drv.fold(mp, topic(t)))
            want = sorted(emission(e) for e in step["expect"])
            assert got == want, "%s step %d (%s): got %r want %r" % (scen["name"], i, t, got, want)
    return drv
