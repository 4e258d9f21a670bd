"""Deterministic synthetic workloads of SURVEY.md §8(d) (configs A-E) and the
reference's own bench shapes (R1/R2, vmq_reg_trie_bench_SUITE.erl:97-214).

A workload is columnar (numpy CSR of word indices), so that million-scale
configs load into the matcher without per-subscription Python work.  The
same columns feed the CPU oracle (test / cpu_baseline infrastructure only)
through oracle/feed.py; this module never imports the oracle.

RNG: splitmix64 (seeded per config), as §8(d) specifies.
"""
from __future__ import annotations

import numpy as np

from . import _lib

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


class SplitMix:
    def __init__(self, seed: int):
        self.state = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)

    def u64(self, n: int) -> np.ndarray:
        with np.errstate(over="ignore"):
            z = self.state + GOLDEN * np.arange(1, n + 1, dtype=np.uint64)
            self.state = self.state + GOLDEN * np.uint64(n)
            z = (z ^ (z >> np.uint64(30))) * M1
            z = (z ^ (z >> np.uint64(27))) * M2
            return z ^ (z >> np.uint64(31))

    def ints(self, n: int, hi) -> np.ndarray:
        return (self.u64(n) % np.asarray(hi, dtype=np.uint64)).astype(np.int64)

    def unif(self, n: int) -> np.ndarray:
        return (self.u64(n) >> np.uint64(11)).astype(np.float64) / float(1 << 53)


V5_OPTS = [{"no_local": nl, "rap": rap, "retain_handling": rh}
           for nl in (False, True) for rap in (False, True) for rh in ("send_retain", "dont_send")]


def std_subinfos():
    """§8(d): 50 % v4 QoS, 50 % v5 {QoS, #{rap, no_local, retain_handling}}."""
    return [0, 1, 2] + [(q, dict(o)) for q in (0, 1, 2) for o in V5_OPTS]


class Workload:
    """Columnar subscriptions + publishes.

    sub_*  : per subscription (load order = initialize_trie fold order)
    topics : CSR (tw_off, tw) of indices into ``words`` (subscription vocab)
    pubs   : CSR (pw_off, pw) of indices into ``pub_words``; pub_mp per publish
    """

    def __init__(self, name, self_node="node0@127.0.0.1"):
        self.name = name
        self.self_node = self_node
        self.nodes = [self_node]
        self.mps = [""]
        self.words: list = []
        self.clients: list = []       # (mp, client bytes)
        self.subinfos: list = []
        self.sub_client = self.sub_info = self.sub_node = None
        self.tw_off = self.tw = None
        self.pub_words: list = []
        self.pub_mp = self.pw_off = self.pw = None
        self.client_mp = None             # lean workloads: MP index per client (clients is None)
        self.notes = {}

    # ------------------------------------------------------------ helpers
    @property
    def n_subs(self):
        return len(self.sub_client)

    @property
    def n_pubs(self):
        return len(self.pub_mp)

    def sub_topic(self, i):
        a, b = self.tw_off[i], self.tw_off[i + 1]
        return tuple(self.words[j] for j in self.tw[a:b])

    def pub_topic(self, i):
        a, b = self.pw_off[i], self.pw_off[i + 1]
        return tuple(self.pub_words[j] for j in self.pw[a:b])

    def pub_slice(self, lo, hi):
        return [(self.mps[self.pub_mp[i]], self.pub_topic(i)) for i in range(lo, hi)]

    # ------------------------------------------------------------ product
    def bind(self, view):
        """Intern this workload's terms in `view`; returns the id maps
        (word, node, mountpoint-of-client, subscriber, subinfo).  A lean
        workload (clients is None: tens of millions of subscribers) uses
        the client index itself as the opaque SubscriberId id and never
        materialises the terms (its records are decoded with client_term)."""
        from .reg_view import _subinfo_key
        wid = view.intern_words(self.words, create=True).astype(np.uint32)
        node_id = np.array([view.nodes.get(n) for n in self.nodes], dtype=np.uint32)
        mp_id = np.array([view.mountpoints.get(m) for m in self.mps], dtype=np.uint32)
        si_id = np.array([view.subinfos.get(s, _subinfo_key(s)) for s in self.subinfos], dtype=np.uint32)
        if self.clients is None:
            return {"wid": wid, "node": node_id, "client_mp": mp_id[self.client_mp],
                    "sid": np.arange(len(self.client_mp), dtype=np.uint32), "si": si_id}
        sid_id = np.array([view.subscribers.get(c) for c in self.clients], dtype=np.uint32)
        mp_index = {m: i for i, m in enumerate(self.mps)}
        client_mp = np.array([mp_index[c[0]] for c in self.clients], dtype=np.int64)
        return {"wid": wid, "node": node_id, "client_mp": mp_id[client_mp], "sid": sid_id, "si": si_id}

    def client_term(self, i: int):
        """SubscriberId term of client i (lean workloads: from client_mp)."""
        if self.clients is not None:
            return self.clients[i]
        return (self.mps[int(self.client_mp[i])], b"c%d" % i)

    def op_arrays(self, ids, idx: np.ndarray, kind: int):
        """OP_DTYPE + word-id arrays for subscriptions `idx` (one op each)."""
        from .reg_view import OP_DTYPE
        idx = np.asarray(idx, dtype=np.int64)
        lens = self.tw_off[idx + 1] - self.tw_off[idx]
        ops = np.zeros(len(idx), dtype=OP_DTYPE)
        ops["kind"] = kind
        ops["mountpoint"] = ids["client_mp"][self.sub_client[idx]]
        woff = np.zeros(len(idx), dtype=np.int64)
        if len(idx):
            woff[1:] = np.cumsum(lens)[:-1]
        ops["word_off"] = woff.astype(np.uint32)
        ops["nwords"] = lens.astype(np.uint32)
        ops["node"] = ids["node"][self.sub_node[idx]]
        ops["subscriber"] = ids["sid"][self.sub_client[idx]]
        ops["subinfo"] = ids["si"][self.sub_info[idx]]
        # gather the word ids of every selected topic
        total = int(lens.sum())
        rep = np.repeat(self.tw_off[idx] - woff, lens)
        words = ids["wid"][self.tw[np.arange(total, dtype=np.int64) + rep]] if total else np.zeros(0, np.uint32)
        return ops, words

    def load_into(self, view, batch: int = 1 << 20, n: int | None = None, progress=None):
        """Bulk initialize_trie of subscriptions [0, n) into a RegGpuView (op
        arrays, no per-subscription Python).  Returns the id maps.
        progress(done, n): called after every batch (long loads log)."""
        ids = self.bind(view)
        n = self.n_subs if n is None else n
        for lo in range(0, n, batch):
            ops, words = self.op_arrays(ids, np.arange(lo, min(n, lo + batch)), _lib.OP_ADD)
            view.apply_op_arrays(ops, words)
            if progress is not None:
                progress(min(n, lo + batch), n)
        return ids

    def publish_arrays(self, view, lo: int = 0, hi: int | None = None):
        """PUB_DTYPE + word-id arrays for publishes [lo, hi) (ids looked up, not created)."""
        pwid = view.intern_words(self.pub_words, create=False).astype(np.uint32)
        mp_id = np.array([view.mountpoints.ids.get(m, _lib.NONE) for m in self.mps], dtype=np.uint32)
        return self.publish_arrays_ids(pwid, mp_id, lo, hi)

    def publish_arrays_ids(self, pwid: np.ndarray, mp_id: np.ndarray, lo: int = 0, hi: int | None = None):
        """Same, from a precomputed pub_words -> word id map (replicas have no dictionary)."""
        from .reg_view import PUB_DTYPE
        hi = self.n_pubs if hi is None else hi
        dollar = np.array([w[:1] == b"$" for w in self.pub_words], dtype=bool)
        base = self.pw_off[lo]
        pubs = np.zeros(hi - lo, dtype=PUB_DTYPE)
        pubs["mountpoint"] = np.asarray(mp_id, dtype=np.uint32)[self.pub_mp[lo:hi]]
        pubs["word_off"] = (self.pw_off[lo:hi] - base).astype(np.uint32)
        pubs["nwords"] = (self.pw_off[lo + 1:hi + 1] - self.pw_off[lo:hi]).astype(np.uint32)
        first = self.pw[self.pw_off[lo:hi]]
        pubs["flags"] = np.where(dollar[first], _lib.PUB_DOLLAR, 0).astype(np.uint32)
        return pubs, np.asarray(pwid, dtype=np.uint32)[self.pw[base:self.pw_off[hi]]]


def _csr(lists):
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(x) for x in lists])
    flat = np.fromiter((w for x in lists for w in x), dtype=np.int64, count=int(off[-1]))
    return off, flat


# ------------------------------------------------------------------ configs
def config_c(n_dev: int = 1_000_000, n_wild: int = 64, n_pubs: int = 1 << 20, dev_range: float = 1.25,
             seed: int = 0xC) -> Workload:
    """Config C (§8d, the headline "1M subs"): devices/{d}/telemetry/# for
    d < n_dev plus n_wild subscribers on devices/+/telemetry/#; publishes
    devices/{d}/telemetry/{m}, d uniform in [0, 1.25 n_dev), m from 16 names."""
    r = SplitMix(seed)
    w = Workload("C")
    n_range = int(n_dev * dev_range)
    dev_words = [b"%d" % d for d in range(n_range)]
    w.words = [b"devices", b"telemetry", b"#", b"+"] + dev_words[:n_dev]
    w.subinfos = std_subinfos()
    w.clients = [("", b"c%d" % d) for d in range(n_dev)] + [("", b"w%d" % i) for i in range(n_wild)]
    n = n_dev + n_wild
    w.sub_client = np.arange(n, dtype=np.int64)
    half = r.unif(n) < 0.5
    w.sub_info = np.where(half, r.ints(n, 3), 3 + r.ints(n, 3 * len(V5_OPTS)))
    w.sub_node = np.zeros(n, dtype=np.int64)
    tw = np.empty((n, 4), dtype=np.int64)
    tw[:, 0], tw[:, 2], tw[:, 3] = 0, 1, 2
    tw[:n_dev, 1] = 4 + np.arange(n_dev)
    tw[n_dev:, 1] = 3
    w.tw_off = np.arange(0, 4 * n + 1, 4, dtype=np.int64)
    w.tw = tw.reshape(-1)
    m_words = [b"m%d" % i for i in range(16)]
    w.pub_words = [b"devices", b"telemetry"] + m_words + dev_words
    d = r.ints(n_pubs, n_range)
    m = r.ints(n_pubs, 16)
    pw = np.empty((n_pubs, 4), dtype=np.int64)
    pw[:, 0], pw[:, 1], pw[:, 2], pw[:, 3] = 0, 18 + d, 1, 2 + m
    w.pw_off = np.arange(0, 4 * n_pubs + 1, 4, dtype=np.int64)
    w.pw = pw.reshape(-1)
    w.pub_mp = np.zeros(n_pubs, dtype=np.int64)
    w.notes = {"n_dev": n_dev, "n_wild": n_wild, "hit_fraction": n_dev / n_range}
    return w


def _instantiate(r: SplitMix, filt, level_vocab):
    out = []
    for i, x in enumerate(filt):
        if x == b"+":
            v = level_vocab[min(i, len(level_vocab) - 1)]
            out.append(v[int(r.ints(1, len(v))[0])])
        elif x == b"#":
            for j in range(int(r.ints(1, 3)[0])):
                v = level_vocab[min(i + j, len(level_vocab) - 1)]
                out.append(v[int(r.ints(1, len(v))[0])])
        else:
            out.append(x)
    return tuple(out) if out else (level_vocab[0][0],)


def _finish(w: Workload, subs, pubs):
    """subs: [(client_idx, topic words, subinfo_idx, node_idx)], pubs: [(mp_idx, words)]."""
    vocab = {}
    for _, t, _, _ in subs:
        for x in t:
            vocab.setdefault(x, len(vocab))
    w.words = list(vocab)
    w.sub_client = np.array([s[0] for s in subs], dtype=np.int64)
    w.sub_info = np.array([s[2] for s in subs], dtype=np.int64)
    w.sub_node = np.array([s[3] for s in subs], dtype=np.int64)
    w.tw_off, w.tw = _csr([[vocab[x] for x in s[1]] for s in subs])
    pv = {}
    for _, t in pubs:
        for x in t:
            pv.setdefault(x, len(pv))
    w.pub_words = list(pv)
    w.pub_mp = np.array([p[0] for p in pubs], dtype=np.int64)
    w.pw_off, w.pw = _csr([[pv[x] for x in p[1]] for p in pubs])
    return w


def config_a(seed: int = 0xA, n_subs: int = 10_000, n_clients: int = 2_000, n_pubs: int = 100_000) -> Workload:
    """Config A (§8d): mixed exact / '+' / '#' / $share subs, 10 % remote."""
    r = SplitMix(seed)
    w = Workload("A")
    w.nodes = [w.self_node, "node1@127.0.0.1", "node2@127.0.0.1", "node3@127.0.0.1"]
    vocab = [[b"w%d_%d" % (k, j) for j in range(16)] for k in range(6)]
    w.subinfos = std_subinfos()
    w.clients = [("", b"c%d" % i) for i in range(n_clients)]
    subs, filts = [], []
    for _ in range(n_subs):
        L = 3 + int(r.ints(1, 3)[0])
        t = [vocab[k][int(r.ints(1, 16)[0])] for k in range(L)]
        x = r.unif(1)[0]
        if x < 0.20:
            for _ in range(1 + int(r.ints(1, 2)[0])):
                t[int(r.ints(1, L)[0])] = b"+"
        elif x < 0.30:
            t = t[:1 + int(r.ints(1, L - 1)[0])] + [b"#"]
        filts.append(tuple(t))
        if r.unif(1)[0] < 0.01:
            t = [b"$share", b"g%d" % int(r.ints(1, 10)[0])] + t
        node = 1 + int(r.ints(1, 3)[0]) if r.unif(1)[0] < 0.10 else 0
        si = int(r.ints(1, len(w.subinfos))[0])
        subs.append((int(r.ints(1, n_clients)[0]), tuple(t), si, node))
    pubs = []
    for _ in range(n_pubs):
        x = r.unif(1)[0]
        if x < 0.50:
            pubs.append((0, _instantiate(r, filts[int(r.ints(1, len(filts))[0])], vocab)))
        elif x < 0.99:
            L = 1 + int(r.ints(1, 6)[0])
            pubs.append((0, tuple(vocab[k][int(r.ints(1, 16)[0])] for k in range(L))))
        else:
            pubs.append((0, (b"$SYS",) + tuple(vocab[k][int(r.ints(1, 16)[0])] for k in range(1, 3))))
    return _finish(w, subs, pubs)


def config_b(seed: int = 0xB, n_subs: int = 100_000, n_pubs: int = 1 << 16) -> Workload:
    """Config B (§8d): 100k subs, 5 levels, 85 % exact / 10 % '+' / 5 % '#'."""
    r = SplitMix(seed)
    w = Workload("B")
    sizes = [8, 32, 128, 512, 2048]
    vocab = [[b"l%d_%d" % (k, j) for j in range(s)] for k, s in enumerate(sizes)]
    w.subinfos = std_subinfos()
    w.clients = [("", b"c%d" % i) for i in range(n_subs)]
    subs, filts = [], []
    for i in range(n_subs):
        t = [vocab[k][int(r.ints(1, sizes[k])[0])] for k in range(5)]
        x = r.unif(1)[0]
        if x < 0.10:
            t[int(r.ints(1, 5)[0])] = b"+"
            if r.unif(1)[0] < 0.2:
                t[int(r.ints(1, 5)[0])] = b"+"
        elif x < 0.15:
            t = t[:1 + int(r.ints(1, 4)[0])] + [b"#"]
        filts.append(tuple(t))
        subs.append((i, tuple(t), int(r.ints(1, len(w.subinfos))[0]), 0))
    pubs = []
    for _ in range(n_pubs):
        if r.unif(1)[0] < 0.5:
            pubs.append((0, _instantiate(r, filts[int(r.ints(1, len(filts))[0])], vocab)))
        else:
            pubs.append((0, tuple(vocab[k][int(r.ints(1, sizes[k])[0])] for k in range(5))))
    return _finish(w, subs, pubs)


def config_r1(n: int = 100_000) -> Workload:
    """R1 = bench_single_lookups (vmq_reg_trie_bench_SUITE.erl:114-150): one
    subscriber per unique topic unique/topic/I, MP "a"; each fold -> [{{"a",I},0}]."""
    w = Workload("R1")
    w.mps = ["a"]
    w.subinfos = [0]
    w.clients = [("a", b"%d" % i) for i in range(1, n + 1)]
    subs = [(i, (b"unique", b"topic", b"%d" % (i + 1)), 0, 0) for i in range(n)]
    pubs = [(0, (b"unique", b"topic", b"%d" % i)) for i in range(1, n + 1)]
    return _finish(w, subs, pubs)


def config_r2(n: int = 100_000) -> Workload:
    """R2 = bench_fanout_subs (vmq_reg_trie_bench_SUITE.erl:152-214): n
    subscribers on some/topic; one fold returns all n."""
    w = Workload("R2")
    w.mps = ["a"]
    w.subinfos = [0]
    w.clients = [("a", b"%d" % i) for i in range(1, n + 1)]
    subs = [(i, (b"some", b"topic"), 0, 0) for i in range(n)]
    pubs = [(0, (b"some", b"topic"))]
    return _finish(w, subs, pubs)


def config_d(scale: float = 1.0, seed: int = 0xD, n_pubs: int = 1 << 20, extra: float = 0.1) -> Workload:
    """Config D (§8d) at `scale` (1.0 = 10M subs):
      8M exact   site/{s}/dev/{d}/state   (s < 1000, d < 8000 at scale 1)
      1M         site/{s}/+/alarm/#       (s uniform)
      1M         $share/g{g}/jobs/{g mod 1000}/+ : 10,000 groups x 100 members,
                 member m on node m mod 4 (so each member is emitted 4 times, Q2)
    plus `extra` x that many not-yet-live subscriptions of the same shapes for
    the churn (1 %/s = 10 batches/s of 10,000 ops at scale 1, 50/50 sub/unsub).
    Publishes: 70 % site/s/dev/d/state, 25 % site/s/x{k}/alarm/z{j}, 5 % jobs/q/x{k}."""
    r = SplitMix(seed)
    w = Workload("D")
    w.nodes = [w.self_node, "node1@127.0.0.1", "node2@127.0.0.1", "node3@127.0.0.1"]
    n_s = max(2, int(1000 * scale))
    n_d = 8000
    n_exact = n_s * n_d
    n_alarm = max(1, int(1_000_000 * scale))
    n_groups = max(1, int(10_000 * scale))
    n_members = 100
    n_jobs = n_groups * n_members
    n_live = n_exact + n_alarm + n_jobs
    n_extra = int(n_live * extra)
    n_q = max(1, min(1000, n_groups))
    words = [b"site", b"dev", b"state", b"+", b"#", b"alarm", b"$share", b"jobs"]
    s_base = len(words)
    words += [b"%d" % i for i in range(max(n_s, n_d, n_q))]
    g_base = len(words)
    words += [b"g%d" % g for g in range(n_groups)]
    w.words = words
    w.subinfos = std_subinfos()
    num = lambda x: s_base + np.asarray(x, dtype=np.int64)
    # --- live subscriptions, then the churn pool of not-yet-live ones
    kinds = []      # (topics [n, L] array, clients, nodes)
    # exact
    i = np.arange(n_exact + n_extra * 8 // 10, dtype=np.int64)
    s_i = np.where(i < n_exact, i // n_d, r.ints(len(i), n_s))
    d_i = np.where(i < n_exact, i % n_d, r.ints(len(i), n_d))
    t = np.stack([np.zeros_like(i), num(s_i), np.ones_like(i), num(d_i), np.full_like(i, 2)], axis=1)
    kinds.append(("e", t, np.zeros_like(i)))
    # alarm
    i = np.arange(n_alarm + n_extra // 10, dtype=np.int64)
    t = np.stack([np.zeros_like(i), num(r.ints(len(i), n_s)), np.full_like(i, 3), np.full_like(i, 5),
                  np.full_like(i, 4)], axis=1)
    kinds.append(("a", t, np.zeros_like(i)))
    # $share jobs
    i = np.arange(n_jobs + n_extra // 10, dtype=np.int64)
    g_i = np.where(i < n_jobs, i // n_members, r.ints(len(i), n_groups))
    m_i = np.where(i < n_jobs, i % n_members, n_members + i)
    t = np.stack([np.full_like(i, 6), g_base + g_i, np.full_like(i, 7), num(g_i % n_q), np.full_like(i, 3)], axis=1)
    kinds.append(("j", t, m_i % 4))
    live_n = [n_exact, n_alarm, n_jobs]
    # order: all live subscriptions first (load order), then the pools
    topics, clients, nodes, live_parts, pool_parts = [], [], [], [], []
    cbase = 0
    for (tag, t, nd), ln in zip(kinds, live_n):
        n = len(t)
        live_parts.append((t[:ln], nd[:ln], cbase, ln))
        pool_parts.append((t[ln:], nd[ln:], cbase + ln, n - ln))
        clients += [("", b"%s%d" % (tag.encode(), k)) for k in range(n)]
        cbase += n
    rows, cl, nod = [], [], []
    for t, nd, c0, n in live_parts + pool_parts:
        rows.append(t)
        cl.append(np.arange(c0, c0 + n, dtype=np.int64))
        nod.append(nd)
    T = np.concatenate(rows)
    w.clients = clients
    w.sub_client = np.concatenate(cl)
    w.sub_node = np.concatenate(nod).astype(np.int64)
    w.sub_info = r.ints(len(T), len(w.subinfos))
    w.tw_off = np.arange(0, 5 * len(T) + 1, 5, dtype=np.int64)
    w.tw = T.reshape(-1)
    w.notes = {"n_live": n_live, "n_pool": len(T) - n_live, "n_s": n_s, "n_d": n_d, "n_q": n_q,
               "groups": n_groups, "members": n_members}
    # publishes
    pw = [b"site", b"dev", b"state", b"alarm", b"jobs"]
    pn_base = len(pw)
    pw += [b"%d" % k for k in range(max(n_s, n_d, n_q))]
    px_base = len(pw)
    pw += [b"x%d" % k for k in range(16)] + [b"z%d" % k for k in range(16)]
    w.pub_words = pw
    u = r.unif(n_pubs)
    a1, a2, a3 = r.ints(n_pubs, n_s), r.ints(n_pubs, n_d), r.ints(n_pubs, 16)
    is_state, is_alarm = u < 0.70, (u >= 0.70) & (u < 0.95)
    rows = np.zeros((n_pubs, 5), dtype=np.int64)
    lens = np.where(is_state | is_alarm, 5, 3)
    rows[:, 0] = np.where(is_state | is_alarm, 0, 4)
    rows[:, 1] = pn_base + np.where(is_state | is_alarm, a1, a1 % n_q)
    rows[:, 2] = np.where(is_state, 1, px_base + a3)
    rows[:, 3] = np.where(is_state, pn_base + a2, 3)
    rows[:, 4] = np.where(is_state, 2, px_base + 16 + a3)
    w.pw_off = np.zeros(n_pubs + 1, dtype=np.int64)
    w.pw_off[1:] = np.cumsum(lens)
    w.pw = rows.reshape(-1)[(np.arange(5)[None, :] < lens[:, None]).reshape(-1)]
    w.pub_mp = np.zeros(n_pubs, dtype=np.int64)
    return w


class Churn:
    """Config D's subscription churn: each batch unsubscribes `n/2` live
    subscriptions chosen uniformly and subscribes `n/2` not-live ones (the
    pool).  Every churn subscriber holds exactly one subscription, so a batch
    is also expressible as subscriber-store events for the oracle."""

    def __init__(self, w: Workload, seed: int = 0xD0):
        self.w = w
        self.r = SplitMix(seed)
        self.live = np.zeros(w.n_subs, dtype=bool)
        self.live[:w.notes["n_live"]] = True

    def batch(self, n: int):
        half = n // 2
        live_idx = np.flatnonzero(self.live)
        dead_idx = np.flatnonzero(~self.live)
        dels = live_idx[np.unique(self.r.ints(half, len(live_idx)))]
        adds = dead_idx[np.unique(self.r.ints(half, len(dead_idx)))] if len(dead_idx) else dead_idx
        self.live[dels] = False
        self.live[adds] = True
        return dels, adds

    def ops(self, ids, dels, adds):
        """Deletes first, then adds (the order handle_event/2 uses within an event)."""
        from .reg_view import OP_DTYPE
        o1, w1 = self.w.op_arrays(ids, dels, _lib.OP_DEL)
        o2, w2 = self.w.op_arrays(ids, adds, _lib.OP_ADD)
        o2["word_off"] += len(w1)
        return np.concatenate([o1, o2]).astype(OP_DTYPE), np.concatenate([w1, w2]).astype(np.uint32)

    def events(self, dels, adds):
        w = self.w
        ev = []
        for i in dels:
            sid = w.clients[w.sub_client[i]]
            ev.append(("deleted", sid, [(w.nodes[w.sub_node[i]], True, [(w.sub_topic(i), w.subinfos[w.sub_info[i]])])]))
        for i in adds:
            sid = w.clients[w.sub_client[i]]
            ev.append(("updated", sid, None, [(w.nodes[w.sub_node[i]], True, [(w.sub_topic(i), w.subinfos[w.sub_info[i]])])]))
        return ev


def config_d_counts(w: Workload, live: np.ndarray, lo: int = 0, hi: int | None = None) -> np.ndarray:
    """Known answer (vectorised) for config D: emissions per publish [lo, hi)
    given the live-subscription mask.  site/s/dev/d/state emits every live
    exact subscriber of (s, d); site/s/x/alarm/z every live site/s/+/alarm/#
    subscriber; jobs/q/x every live member of every group on q, once per
    distinct node hosting a live member of the group (Q2, vmq_reg_trie.erl:
    68-72, 301-303).  Used by bench.py as a size-independent check."""
    hi = w.n_pubs if hi is None else hi
    n_s, n_d, n_q = w.notes["n_s"], w.notes["n_d"], w.notes["n_q"]
    s_base = 8
    T = w.tw.reshape(-1, 5)
    idx = np.flatnonzero(live)
    rows = T[idx]
    is_exact = (rows[:, 0] == 0) & (rows[:, 2] == 1)
    is_alarm = (rows[:, 0] == 0) & (rows[:, 2] == 3)
    is_jobs = rows[:, 0] == 6
    ex = np.bincount((rows[is_exact, 1] - s_base) * n_d + (rows[is_exact, 3] - s_base), minlength=n_s * n_d)
    al = np.bincount(rows[is_alarm, 1] - s_base, minlength=n_s)
    g = rows[is_jobs, 1]
    q = rows[is_jobs, 3] - s_base
    nodes = w.sub_node[idx[is_jobs]]
    g_min = int(g.min()) if len(g) else 0
    G = (g - g_min) if len(g) else g
    n_g = int(G.max()) + 1 if len(G) else 1
    members = np.bincount(G, minlength=n_g)
    node_seen = np.zeros((n_g, 4), dtype=bool)
    node_seen[G, nodes] = True
    distinct = node_seen.sum(axis=1)
    g_q = np.zeros(n_g, dtype=np.int64)
    g_q[G] = q
    jobs = np.bincount(g_q, weights=members * distinct, minlength=n_q).astype(np.int64)
    out = np.zeros(hi - lo, dtype=np.int64)
    pn_base = 5
    a = w.pw_off[lo:hi]
    first = w.pw[a]
    second = w.pw[a + 1] - pn_base
    is_jobs_p = first == 4
    third = np.where(is_jobs_p, 0, w.pw[np.minimum(a + 2, len(w.pw) - 1)])
    is_state = ~is_jobs_p & (third == 1)
    fourth = np.where(is_state, w.pw[np.minimum(a + 3, len(w.pw) - 1)] - pn_base, 0)
    out[is_jobs_p] = jobs[second[is_jobs_p]]
    out[is_state] = ex[second[is_state] * n_d + fourth[is_state]]
    alarm_p = ~is_jobs_p & ~is_state
    out[alarm_p] = al[second[alarm_p]]
    return out


def _zipf_cdf(n: int, s: float) -> np.ndarray:
    p = 1.0 / np.arange(1, n + 1, dtype=np.float64) ** s
    return np.cumsum(p / p.sum())


def config_e(scale: float = 1.0, seed: int = 0xE, n_pubs: int = 1 << 20, n_mps: int = 1000,
             levels: int = 12, vocab: int = 64, n_hot: int = 1_000_000, lean: bool | None = None) -> Workload:
    """Config E (§8d) at `scale` (1.0 = 50M subscriptions): `n_mps`
    mountpoints t{n} with Zipf(1.0) sizes; topics of `levels` words from
    `vocab` words per level; 80 % exact, 15 % with 1-3 '+', 5 % truncated +
    '#'.  Publishes: Zipf(1.1) over `n_hot` hot topics (half instantiate a
    random filter, half random), each in its filter's / a size-weighted MP.
    lean (default above 5M subscriptions): no per-client Python terms (see
    Workload.bind), 16-bit word indexes."""
    r = SplitMix(seed)
    w = Workload("E")
    n = max(1000, int(50_000_000 * scale))
    n_hot = max(100, min(n_hot, n))
    w.mps = ["t%d" % k for k in range(n_mps)]
    mp_cdf = _zipf_cdf(n_mps, 1.0)
    sub_mp = np.searchsorted(mp_cdf, r.unif(n), side="right").clip(0, n_mps - 1)
    lvl = [[b"l%d_%d" % (k, j) for j in range(vocab)] for k in range(levels)]
    w.words = [b"+", b"#"] + [x for lv in lvl for x in lv]
    base = lambda k: 2 + k * vocab
    if lean is None:
        lean = n > 5_000_000
    T = np.empty((n, levels), dtype=np.int16 if lean else np.int64)
    for k in range(levels):
        T[:, k] = base(k) + r.ints(n, vocab)
    u = r.unif(n)
    plus = (u >= 0.80) & (u < 0.95)
    hashed = u >= 0.95
    for _ in range(3):   # 1-3 '+' levels (duplicates collapse)
        pos = r.ints(n, levels)
        sel = plus & (r.unif(n) < 0.75)
        T[sel, pos[sel]] = 0
    first_plus = plus & ~(T == 0).any(axis=1)
    T[first_plus, r.ints(n, levels)[first_plus]] = 0
    cut = 1 + r.ints(n, levels - 1)      # '#' filters: keep 1..L-1 words then '#'
    lens = np.where(hashed, cut + 1, levels)
    T[hashed, cut[hashed]] = 1
    w.tw_off = np.zeros(n + 1, dtype=np.int64)
    w.tw_off[1:] = np.cumsum(lens)
    w.tw = T.reshape(-1)[(np.arange(levels)[None, :] < lens[:, None]).reshape(-1)]
    w.subinfos = std_subinfos()
    w.sub_info = r.ints(n, len(w.subinfos))
    w.sub_node = np.zeros(n, dtype=np.int64)
    if lean:
        w.clients = None
        w.client_mp = sub_mp.astype(np.int32)
    else:
        w.clients = [(w.mps[m], b"c%d" % i) for i, m in enumerate(sub_mp)]
    w.sub_client = np.arange(n, dtype=np.int64)
    # hot topics: half instantiate a filter (same MP), half random (size-weighted MP)
    src = r.ints(n_hot, n)
    inst = r.unif(n_hot) < 0.5
    H = np.empty((n_hot, levels), dtype=np.int64)
    for k in range(levels):
        H[:, k] = base(k) + r.ints(n_hot, vocab)
    hl = np.full(n_hot, levels, dtype=np.int64)
    fl = lens[src]
    ft = T[src]
    # instantiated: copy the filter words, '+' -> random word, '#' -> 0-2 random words
    for k in range(levels):
        keep = inst & (k < fl) & (ft[:, k] > 1)
        H[keep, k] = ft[keep, k]
    has_hash = inst & (ft[np.arange(n_hot), np.minimum(fl - 1, levels - 1)] == 1)
    extra = r.ints(n_hot, 3)
    hl = np.where(inst, np.where(has_hash, np.minimum(fl - 1 + extra, levels), fl), hl)
    hl = np.maximum(hl, 1)
    hot_mp = np.where(inst, sub_mp[src], np.searchsorted(mp_cdf, r.unif(n_hot), side="right").clip(0, n_mps - 1))
    pick = np.searchsorted(_zipf_cdf(n_hot, 1.1), r.unif(n_pubs), side="right").clip(0, n_hot - 1)
    plen = hl[pick]
    w.pub_words = w.words
    w.pw_off = np.zeros(n_pubs + 1, dtype=np.int64)
    w.pw_off[1:] = np.cumsum(plen)
    w.pw = H[pick].reshape(-1)[(np.arange(levels)[None, :] < plen[:, None]).reshape(-1)]
    w.pub_mp = hot_mp[pick]
    w.notes = {"n_subs": n, "n_mps": n_mps, "levels": levels, "vocab": vocab, "n_hot": n_hot}
    return w


CONFIGS = {"A": config_a, "B": config_b, "C": config_c, "D": config_d, "E": config_e,
           "R1": config_r1, "R2": config_r2}


def algorithmic_bytes_c(w: Workload, lo: int = 0, hi: int | None = None, part: str = "all") -> int:
    """Σ B_p over publishes [lo, hi) of a config-C workload, with SURVEY.md
    §8(d)'s B_p = 8(L_p+1) + 16 S_p + 32 R_p and the reference's lookup counts
    for this shape (validated against the oracle's counters in
    tests/test_workloads.py):
      hit  (d < n_dev): S_p = 26 (20 trie_match + 2 match/4 + 4 fold), R_p = 65
      miss (d >= n_dev): S_p = 17 (13 + 1 + 3),                       R_p = 64
    part: "all" = B_p; "lookup" = 8(L_p+1) + 16 S_p (the walk, COUNT kernel);
    "emit" = 32 R_p (record read + write, EMIT kernel);
    "lookup_tx" = the transaction-granular form of "lookup" (SURVEY §8(d)):
    every logical lookup charged a whole 64-B line, 8(L_p+1) + 64 S_p;
    "emit_compulsory" = the bytes EMIT cannot avoid moving through HBM:
    16 R_p written + 40 B per publish read (32-B key cache, its offset) +
    16 B per DISTINCT record of the batch (the 64 shared wildcard records
    once, each hit publish's own device record).  32 R_p charges a 16-B HBM
    read for every emission although 64 of a publish's 65 records are the
    same L2-resident list, so it can exceed what any kernel moves.
    """
    hi = w.n_pubs if hi is None else hi
    d = w.pw[4 * lo + 1:4 * hi:4] - 18
    n_hit = int(np.count_nonzero(d < w.notes["n_dev"]))
    n_miss = (hi - lo) - n_hit
    look_hit, look_miss = 8 * 5 + 16 * 26, 8 * 5 + 16 * 17
    emit_hit, emit_miss = 32 * (w.notes["n_wild"] + 1), 32 * w.notes["n_wild"]
    look = n_hit * look_hit + n_miss * look_miss
    emit = n_hit * emit_hit + n_miss * emit_miss
    if part == "emit_compulsory":
        distinct = int(np.unique(d[d < w.notes["n_dev"]]).size) + w.notes["n_wild"]
        writes = 16 * (n_hit * (w.notes["n_wild"] + 1) + n_miss * w.notes["n_wild"])
        return writes + 40 * (hi - lo) + 16 * distinct
    if part == "lookup_tx":
        return n_hit * (8 * 5 + 64 * 26) + n_miss * (8 * 5 + 64 * 17)
    return {"all": look + emit, "lookup": look, "emit": emit}[part]


class RetainWorkload:
    """Retained-store workload RT: the retained
    messages of config C's device fleet and a burst of subscriptions folding
    over them (vmq_reg:deliver_retained/5 -> vmq_retain_srv:match_fold/4).

    Store: ``devices/{d}/telemetry/{m}`` for d < n_dev, m < 16 (one retained
    message per topic, message id = row).  Filters (splitmix64 seed 0x7E7):
      50 % ``devices/{d}/telemetry/#``   -> 16 messages
      20 % ``devices/{d}/+/{m}``         -> 1
      25 % ``devices/{d}/telemetry/{m}`` -> 1 (exact ets:lookup)
       5 % ``devices/{d'}/telemetry/#`` with d' >= n_dev (no retained topic) -> 0
      plus ``n_heavy`` x ``devices/+/telemetry/{m}`` -> n_dev each (the
      reference scans the whole table for it; the product walks the position
      list {m, 3}).
    Columns: word strings in ``vocab``; topics/filters as (n, 4) index arrays.
    """

    def __init__(self, n_dev: int = 62_500, n_filters: int = 1 << 18, n_heavy: int = 16, seed: int = 0x7E7):
        self.n_dev, self.n_filters, self.n_heavy = n_dev, n_filters, n_heavy
        self.n_topics = 16 * n_dev
        self.vocab = [b"devices", b"telemetry", b"+", b"#"] + [b"m%d" % m for m in range(16)] + \
                     [b"%d" % d for d in range(n_dev)]
        self.V_DEV, self.V_TEL, self.V_PLUS, self.V_HASH, self.V_M0, self.V_D0 = 0, 1, 2, 3, 4, 20
        i = np.arange(self.n_topics, dtype=np.int64)
        self.topics = np.stack([np.zeros_like(i), self.V_D0 + i // 16, np.full_like(i, self.V_TEL),
                                self.V_M0 + i % 16], axis=1)
        r = SplitMix(seed)
        n_reg = n_filters - n_heavy
        kind = r.ints(n_reg, 100)
        d = r.ints(n_reg, n_dev)
        m = r.ints(n_reg, 16)
        f = np.empty((n_reg, 4), dtype=np.int64)
        f[:, 0] = self.V_DEV
        f[:, 1] = self.V_D0 + d
        f[:, 2] = self.V_TEL
        f[:, 3] = self.V_M0 + m
        wild = kind < 50
        f[wild, 3] = self.V_HASH
        plus = (kind >= 50) & (kind < 70)
        f[plus, 2] = self.V_PLUS
        unk = kind >= 95
        f[unk, 1] = -1 - d[unk]            # a device id no retained topic has (word "x{d}")
        f[unk, 3] = self.V_HASH
        heavy = np.empty((n_heavy, 4), dtype=np.int64)
        heavy[:, 0], heavy[:, 1], heavy[:, 2] = self.V_DEV, self.V_PLUS, self.V_TEL
        heavy[:, 3] = self.V_M0 + np.arange(n_heavy) % 16
        # heavy filters spread through the batch
        pos = np.linspace(0, n_filters - 1, n_heavy).astype(np.int64) if n_heavy else np.zeros(0, np.int64)
        is_heavy = np.zeros(n_filters, dtype=bool)
        is_heavy[pos] = True
        self.filters = np.empty((n_filters, 4), dtype=np.int64)
        self.filters[is_heavy] = heavy
        self.filters[~is_heavy] = f
        per = np.where(wild, 16, np.where(unk, 0, 1))
        self.matches = np.empty(n_filters, dtype=np.int64)
        self.matches[is_heavy] = n_dev
        self.matches[~is_heavy] = per
        # rows of the list each filter walks (the shortest its literal words
        # select): pair list {devices, d} = 16 rows; devices/+/telemetry/{m}
        # -> position list {m, 3} = n_dev rows; exact -> 1 row (the plan's
        # probe); unknown word -> none
        self.rows_visited = np.empty(n_filters, dtype=np.int64)
        self.rows_visited[is_heavy] = n_dev
        self.rows_visited[~is_heavy] = np.where(wild, 16, np.where(plus, 16, np.where(unk, 0, 1)))
        self.exact = np.zeros(n_filters, dtype=bool)
        self.exact[~is_heavy] = (kind >= 70) & (kind < 95)

    def word(self, v: int) -> bytes:
        return self.vocab[v] if v >= 0 else b"x%d" % (-1 - v)

    def topic(self, i: int):
        return tuple(self.word(int(v)) for v in self.topics[i])

    def filter(self, i: int):
        return tuple(self.word(int(v)) for v in self.filters[i])

    def load_into(self, srv, batch: int = 1 << 20):
        """Bulk insert/3 of every retained topic (message id = row)."""
        from .retain import ROP_DTYPE
        vid = srv.intern_words(self.vocab, create=True).astype(np.int64)
        for lo in range(0, self.n_topics, batch):
            hi = min(self.n_topics, lo + batch)
            n = hi - lo
            ops = np.zeros(n, dtype=ROP_DTYPE)
            ops["kind"] = _lib.ROP_INSERT
            ops["word_off"] = 4 * np.arange(n)
            ops["nwords"] = 4
            ops["msg"] = np.arange(lo, hi)
            srv.apply_op_arrays(ops, vid[self.topics[lo:hi]].reshape(-1).astype(np.uint32))
        return vid

    def filter_arrays(self, vid: np.ndarray):
        """(PUB_DTYPE filters, word ids): unknown device words -> WORD_UNKNOWN."""
        from .reg_view import PUB_DTYPE
        n = self.n_filters
        arr = np.zeros(n, dtype=PUB_DTYPE)
        arr["word_off"] = 4 * np.arange(n)
        arr["nwords"] = 4
        f = self.filters
        words = np.where(f >= 0, vid[np.maximum(f, 0)], np.int64(_lib.WORD_UNKNOWN)).astype(np.uint32)
        return arr, words.reshape(-1)

    def algorithmic_bytes(self, part: str = "walk") -> int:
        """Bytes one match batch must move, per the walk over each filter's
        list: per visited candidate its 32-B list entry (row id, message id,
        length, the topic's first 4 words); per filter its 16-B descriptor +
        16-B words + 8-B offset; per match one 4-B message id written.
        part "walk": the one-pass walk kernel; "batch": plus the plan (per
        filter its descriptor and words again, the plan entry and row count
        written: 56 B)."""
        rows = int(self.rows_visited.sum())
        walk = 32 * rows + 4 * int(self.matches.sum()) + 40 * self.n_filters
        if part == "walk":
            return walk
        return walk + 56 * self.n_filters


class AclWorkload:
    """ACL-check workload AC: config C's device
    fleet publishing through vmq_acl's auth_on_publish / auth_on_subscribe
    (apps/vmq_acl/src/vmq_acl.erl:78-93).

    ACL (``lines()``): 32 ``topic read sys/{k}/#`` + 32 ``topic write
    public/{k}/+`` (the `all` tables, never matching a device topic);
    ``n_users`` users ``u{k}`` with ``topic write devices/{4k+j}/cmd/#``
    (j < 4); patterns ``pattern write devices/%c/telemetry/+``, ``pattern
    read devices/%c/cmd/#``, ``pattern write %m/%u/#`` and 5 ``pattern write
    tenants/%m/%c/x{j}``.
    Requests (splitmix64 seed 0xAC), client id = the device id string d,
    user ``u{d // 4}``:
      80 % write devices/{d}/telemetry/{m}          -> allowed (pattern %c)
      10 % write devices/{d}/telemetry/{m}, client d+1 -> denied (every list walked)
       5 % read  devices/{d}/cmd/#                  -> allowed (pattern read %c)
       5 % write devices/{d}/cmd/x                  -> allowed (user table)
    """

    def __init__(self, n_dev: int = 62_500, n_reqs: int = 1 << 20, seed: int = 0xAC):
        self.n_dev, self.n_reqs = n_dev, n_reqs
        self.n_users = (n_dev + 3) // 4
        r = SplitMix(seed)
        kind = r.ints(n_reqs, 100)
        self.d = r.ints(n_reqs, n_dev)
        self.m = r.ints(n_reqs, 16)
        self.kind = np.where(kind < 80, 0, np.where(kind < 90, 1, np.where(kind < 95, 2, 3)))
        self.expect = (self.kind != 1).astype(np.uint8)

    def lines(self):
        out = [b"# workload AC\n"]
        out += [b"topic read sys/%d/#\n" % k for k in range(32)]
        out += [b"topic write public/%d/+\n" % k for k in range(32)]
        for k in range(self.n_users):
            out.append(b"user u%d\n" % k)
            out += [b"topic write devices/%d/cmd/#\n" % (4 * k + j) for j in range(4)]
        out += [b"pattern write devices/%c/telemetry/+\n", b"pattern read devices/%c/cmd/#\n",
                b"pattern write %m/%u/#\n"]
        out += [b"pattern write tenants/%%m/%%c/x%d\n" % j for j in range(5)]
        return out

    def vocab(self):
        return [b"devices", b"telemetry", b"cmd", b"x", b"#", b""] + [b"m%d" % m for m in range(16)] + \
               [b"%d" % d for d in range(self.n_dev + 1)] + [b"u%d" % k for k in range(self.n_users)]

    def request(self, i: int):
        """Request i as (type, topic words, user, mountpoint, client id)."""
        d, m, k = int(self.d[i]), int(self.m[i]), int(self.kind[i])
        user = b"u%d" % (d // 4)
        if k in (0, 1):
            return ("write", (b"devices", b"%d" % d, b"telemetry", b"m%d" % m), user, "",
                    b"%d" % (d + k))
        if k == 2:
            return ("read", (b"devices", b"%d" % d, b"cmd", b"#"), user, "", b"%d" % d)
        return ("write", (b"devices", b"%d" % d, b"cmd", b"x"), user, "", b"%d" % d)

    def arrays(self, acl):
        """(REQ_DTYPE requests, word ids) for the whole batch, vectorised;
        `acl` interns the vocabulary (real words of the workload)."""
        from .acl import REQ_DTYPE
        v = self.vocab()
        ids = acl.intern_words(v, create=True).astype(np.int64)
        DEV, TEL, CMD, X, HASH, EMPTY = ids[:6]
        M0 = 6
        D0 = M0 + 16
        U0 = D0 + self.n_dev + 1
        n = self.n_reqs
        reqs = np.zeros(n, dtype=REQ_DTYPE)
        reqs["type"] = np.where(self.kind == 2, _lib.A_READ, _lib.A_WRITE)
        reqs["user"] = ids[U0 + self.d // 4]
        reqs["client"] = ids[D0 + self.d + (self.kind == 1)]
        reqs["mountpoint"] = EMPTY
        reqs["word_off"] = 4 * np.arange(n)
        reqs["nwords"] = 4
        w = np.empty((n, 4), dtype=np.int64)
        w[:, 0] = DEV
        w[:, 1] = ids[D0 + self.d]
        w[:, 2] = np.where(self.kind >= 2, CMD, TEL)
        w[:, 3] = np.where(self.kind == 2, HASH, np.where(self.kind == 3, X, ids[M0 + self.m]))
        return reqs, w.reshape(-1).astype(np.uint32)

    def algorithmic_bytes(self) -> int:
        """Per request its 24-B descriptor, 16-B topic words read and a 1-B
        verdict written (the rules are an L2-resident table shared by all)."""
        return 41 * self.n_reqs
