"""Shared test plumbing: a driver around the product view with the same
interface as the oracle (apply(events) / fold(mp, topic)), dump
normalisation, and deterministic random churn workloads."""
from __future__ import annotations

import random
import re

from oracle import oracle as O


def canon(entry):
    """FoldFun entry term (product) -> canonical emission tuple (oracle.py)."""
    if isinstance(entry, str):
        return ("C", entry)
    if len(entry) == 2:
        return ("A", entry[0], O.subinfo_repr(entry[1]))
    node, group, sid, si = entry
    return ("B", node, group, sid, O.subinfo_repr(si))


class ProductDriver:
    """RegGpuView with the oracle's test interface.  device=-1: host engine only.
    mode "records": vmqg_match_batch (16-B FoldFun records); "ranges":
    vmqg_match_ranges, expanded on the host against vmqg_records."""

    def __init__(self, node: str, device: int = 0, mode: str = "records", word_lists: bool = False, **kw):
        from vernemq_amd.reg_view import RegGpuView
        self.view = RegGpuView(node=node, device=device, **kw)
        self.mode = mode
        # word_lists: publishes prepared by the library (vmqg_prepare_word_lists),
        # the Topic list as fold/4 takes it; else by the Python mirror's prepare
        self.word_lists = word_lists

    def apply(self, events):
        self.view.handle_events(events)

    def fold(self, mp, topic):
        return self.fold_batch([(mp, tuple(topic))])[0]

    def match_arrays(self, pubs, words):
        if self.mode == "ranges":
            rng, offs = self.view.match_ranges(pubs, words)
            return self.view.expand_ranges(rng, offs)
        return self.view.match_arrays(pubs, words)

    def fold_batch(self, pubs):
        v = self.view
        if self.word_lists:
            arr, words = v.prepare_word_lists([(mp, tuple(t)) for mp, t in pubs])
        else:
            arr, words = v.prepare([(mp, t if isinstance(t, (bytes, bytearray)) else tuple(t)) for mp, t in pubs])
        recs, offs = self.match_arrays(arr, words)
        return [[canon(v.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1]))] for i in range(len(arr))]


def _esc(s) -> str:
    if isinstance(s, str):
        s = s.encode()
    out = '"'
    for c in s:
        if 0x20 <= c < 0x7F and c not in (0x22, 0x5C):
            out += chr(c)
        else:
            out += "\\x%02x" % c
    return out + '"'


def _split_top(s: str):
    """Split on top-level commas, respecting "..." and {...}."""
    parts, depth, cur, q = [], 0, "", False
    i = 0
    while i < len(s):
        c = s[i]
        if q:
            cur += c
            if c == "\\":
                cur += s[i + 1]
                i += 1
            elif c == '"':
                q = False
        elif c == '"':
            q = True
            cur += c
        elif c == "{":
            depth += 1
            cur += c
        elif c == "}":
            depth -= 1
            cur += c
        elif c == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += c
        i += 1
    if cur:
        parts.append(cur)
    return parts


def _sort_brackets(line: str) -> str:
    if line.startswith("topic ") or line.startswith("remote "):
        head, _, rest = line.partition(" [")
        inner = rest[:-1]
        return head + " [" + ",".join(sorted(_split_top(inner))) + "]"
    return line


def normalize_product_dump(view) -> list:
    subs, infos, nodes, mps = view.subscribers.terms, view.subinfos.terms, view.nodes.terms, view.mountpoints.terms

    def sub_tok(m):
        mp, cl = subs[int(m.group(1))]
        return "{%s,%s}" % (_esc(mp), _esc(cl))

    out = []
    for line in view.dump_raw().split("\n"):
        if not line:
            continue
        line = re.sub(r"mp#(\d+)", lambda m: _esc(mps[int(m.group(1))]), line)
        line = re.sub(r"node#(\d+)", lambda m: _esc(nodes[int(m.group(1))]), line)
        line = re.sub(r"sub#(\d+)", sub_tok, line)
        line = re.sub(r"info#(\d+)", lambda m: O.subinfo_repr(infos[int(m.group(1))]), line)
        out.append(_sort_brackets(line))
    return sorted(out)


def normalize_oracle_dump(orc) -> list:
    return sorted(_sort_brackets(l) for l in orc.dump())


# ------------------------------------------------------------------ churn
V5_OPTS = [{"no_local": False, "rap": False, "retain_handling": "send_retain"},
           {"no_local": True, "rap": True, "retain_handling": "dont_send"}]


class ChurnWorkload:
    """Random subscriber-store events over a small vocabulary, chosen to hit
    every code path of the delta handlers: wildcard/exact/$share filters,
    remote nodes, QoS changes (delete+add), v5 SubInfos, prefixes of other
    filters (Q1), multi-node groups (Q2) and inconsistent deletes (Q3)."""

    def __init__(self, seed: int, self_node="n0@h", n_nodes=3, n_clients=40, words=("a", "b", "c", ""),
                 depth=4, mps=("", "mp1")):
        self.r = random.Random(seed)
        self.self_node = self_node
        self.nodes = [self_node] + ["n%d@h" % i for i in range(1, n_nodes)]
        self.words = [w.encode() for w in words]
        self.depth = depth
        self.mps = list(mps)
        self.clients = [(self.r.choice(self.mps), b"c%d" % i) for i in range(n_clients)]
        self.state = {sid: None for sid in self.clients}   # sid -> subs or None

    def rand_filter(self):
        r = self.r
        if r.random() < 0.15:
            pre = (b"$share", r.choice([b"g1", b"g2"]))
        else:
            pre = ()
        L = r.randint(1, self.depth)
        t = []
        for i in range(L):
            x = r.random()
            if x < 0.25:
                t.append(b"+")
            elif x < 0.35 and i == L - 1:
                t.append(b"#")
            else:
                t.append(r.choice(self.words))
        if r.random() < 0.05:
            t = [b"$SYS"] + t[1:]
        return tuple(pre) + tuple(t)

    def rand_subinfo(self):
        r = self.r
        if r.random() < 0.5:
            return r.randint(0, 2)
        return (r.randint(0, 2), dict(r.choice(V5_OPTS)))

    def rand_topic(self):
        r = self.r
        L = r.randint(1, self.depth + 1)
        t = [r.choice(self.words) for _ in range(L)]
        if r.random() < 0.1:
            t[0] = b"$SYS"
        return tuple(t)

    def event(self):
        r = self.r
        sid = r.choice(self.clients)
        old = self.state[sid]
        x = r.random()
        if old is not None and x < 0.12:
            self.state[sid] = None
            if r.random() < 0.2:   # Q3: an inconsistent Old value (a QoS that was never stored)
                old = [(n, c, [(t, 2) for t, _ in ns]) for n, c, ns in old]
            return ("deleted", sid, old)
        new = [] if old is None else [(n, c, list(ns)) for n, c, ns in old]
        node = r.choice(self.nodes) if r.random() < 0.4 else self.self_node
        ent = None
        for e in new:
            if e[0] == node:
                ent = e
        if ent is None:
            ent = (node, True, [])
            new.append(ent)
            new.sort(key=lambda e: e[0])
        ns = ent[2]
        if ns and r.random() < 0.35:
            ns.pop(r.randrange(len(ns)))
        else:
            t = self.rand_filter()
            ns[:] = [e for e in ns if e[0] != t] + [(t, self.rand_subinfo())]
            ns.sort(key=lambda e: e[0])
        self.state[sid] = new
        return ("updated", sid, None if old is None or r.random() < 0.05 else old, new)

    def publishes(self, n):
        return [(self.r.choice(self.mps), self.rand_topic()) for _ in range(n)]
