"""TEST / BASELINE INFRASTRUCTURE ONLY — encodes a columnar
vernemq_amd.workloads.Workload into the oracle's input records
(initialize_trie/2 tuples and publish batches)."""
import struct

from .oracle import subinfo_repr


def _enc(b: bytes) -> bytes:
    return struct.pack("<I", len(b)) + b


def init_bytes(w, lo: int = 0, hi=None, idx=None) -> bytes:
    """initialize_trie/2 tuples (vmq_reg_trie.erl:305-316), record type 3,
    for subscriptions [lo, hi) or the index list `idx`."""
    hi = w.n_subs if hi is None else hi
    idx = range(lo, hi) if idx is None else idx
    wenc = [_enc(x) for x in w.words]
    ienc = [_enc(subinfo_repr(s).encode()) for s in w.subinfos]
    nenc = [_enc(n.encode()) for n in w.nodes]
    cache = {}

    def cenc(c):
        e = cache.get(c)
        if e is None:
            mp, cl = w.client_term(c)
            e = cache[c] = (_enc(mp.encode()), _enc(cl))
        return e

    out = []
    for i in idx:
        a, b = w.tw_off[i], w.tw_off[i + 1]
        mp, cl = cenc(int(w.sub_client[i]))
        out.append(b"\x03" + mp + cl + struct.pack("<I", b - a) + b"".join(wenc[j] for j in w.tw[a:b]) +
                   ienc[w.sub_info[i]] + nenc[w.sub_node[i]])
    return b"".join(out)


def publish_bytes(w, lo: int, hi: int, client: bytes = b"publisher", idx=None) -> bytes:
    """A publish batch: publishes [lo, hi) or the index list `idx`."""
    idx = range(lo, hi) if idx is None else idx
    wenc = [_enc(x) for x in w.pub_words]
    mpenc = [_enc(m.encode()) for m in w.mps]
    cl = _enc(client)
    out = [struct.pack("<I", len(idx))]
    for i in idx:
        a, b = w.pw_off[i], w.pw_off[i + 1]
        out.append(mpenc[w.pub_mp[i]] + cl + struct.pack("<I", b - a) + b"".join(wenc[j] for j in w.pw[a:b]))
    return b"".join(out)


def load(w):
    """A TrieOracle holding workload w's subscriptions."""
    from .oracle import TrieOracle
    o = TrieOracle(w.self_node)
    o.apply_raw(init_bytes(w))
    return o


def load_prefix(w, n: int):
    """A TrieOracle holding workload w's first n subscriptions."""
    from .oracle import TrieOracle
    o = TrieOracle(w.self_node)
    o.apply_raw(init_bytes(w, 0, n))
    return o
