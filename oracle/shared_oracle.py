"""TEST INFRASTRUCTURE ONLY — CPU restatement of VerneMQ's shared-subscription
dispatch (vmq_reg.erl:341-346, 373-378 + vmq_shared_subscriptions.erl:18-106),
the checker for libvmqgpu's include/vmqs.h.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module, and only as the checker.

Two restatements that must agree: ``publish_groups`` (pure Python, clause for
clause, for small cases and fixtures) and ``select`` (the C++ one in
oracle/vmq_shared_oracle.cpp, for batch sizes).  rand:uniform() is replaced by
the counter-based key of vmqs.h (``sel_key``), see the C++ header.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import oracle as _o

M64 = (1 << 64) - 1
NOT_FOUND, ONLINE, OFFLINE, DRAINING = 0, 1, 2, 3
POLICIES = {"random": 0, "prefer_local": 1, "local_only": 2}


def mix64(x: int) -> int:
    x &= M64
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & M64
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & M64
    x ^= x >> 33
    return x


def sel_key(seed: int, q: int, p: int) -> int:
    h = mix64((mix64(seed ^ ((q * 0x9E3779B97F4A7C15) & M64)) + p * 0xD1B54A32D192ED03) & M64)
    return (h & ~0xFFFFFF & M64) | (p & 0xFFFFFF)


# ---- pure-Python restatement --------------------------------------------------
def filter_subscribers(subs, policy, local):
    """vmq_shared_subscriptions.erl:90-106; subs = [(node, sub, pos)]."""
    if policy == "random":
        return subs
    loc = [s for s in subs if s[0] == local]
    if policy == "prefer_local" and not loc:
        return subs
    return loc


def publish_groups(groups, policy, local, state, seed, q):
    """publish/3 (:18-36) over SubscriberGroups = {group: [(node, sub, pos)]}
    (as add_to_subscriber_group built it, vmq_reg.erl:373-378).  Returns
    ({group: chosen (node, sub, pos) or None}) -- None is {error, no_subscribers}."""
    out = {}
    for g, members in groups.items():
        subs = filter_subscribers(members, policy, local)
        ordered = [s for _, s in sorted(((sel_key(seed, q, s[2]), s) for s in subs), key=lambda t: t[0])]
        out[g] = publish_to_group(ordered, state)
    return out


def publish_to_group(ordered, state):
    """:38-73: publish_online in order, then publish_any over the not-online
    members in the order publish_online's fold accumulated them (reversed)."""
    acc = []
    for s in ordered:
        st = state(s[1])
        if st == ONLINE:
            return s            # throw(done)
        if st in (OFFLINE, DRAINING):
            acc.insert(0, s)    # [Subscriber|Acc]
    for s in acc:
        if state(s[1]) != NOT_FOUND:
            return s            # publish_(.., any) -> ok
    return None


def dispatch(records, policy, local, states, seed, q):
    """One publish: records = [(kind, node, group, sub, subinfo)] in emission
    order.  Returns (chosen flags, failed count)."""
    groups = {}
    for p, (kind, node, group, sub, _info) in enumerate(records):
        if kind == 2:
            groups.setdefault(group, []).insert(0, (node, sub, p))
    state = (lambda s: int(states[s]) if s < len(states) else ONLINE)
    res = publish_groups(groups, policy, local, state, seed, q)
    chosen = [0] * len(records)
    failed = 0
    for g, s in res.items():
        if s is None:
            failed += 1
        else:
            chosen[s[2]] = 1
    return chosen, failed


# ---- C++ restatement ----------------------------------------------------------
def _lib():
    L = _o._load()
    if not getattr(L, "_shared_bound", False):
        L.shared_oracle_key.restype = ctypes.c_uint64
        L.shared_oracle_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.shared_oracle_select.restype = None
        L.shared_oracle_select.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.shared_oracle_select_timed.restype = ctypes.c_longlong
        L.shared_oracle_select_timed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L._shared_bound = True
    return L


def _as_records(emits) -> np.ndarray:
    a = np.ascontiguousarray(emits)
    if a.dtype.names is None:
        a = np.ascontiguousarray(a, dtype=np.uint32).reshape(-1, 4)
    return a


def select(emits, offsets, policy: str, seed: int, pub_seq: int, states, local_node: int):
    """Batch form over vmqg_emit records (structured EMIT_DTYPE or [n, 4] u32)
    and offsets[0..npub].  Returns (chosen u8 per record, failed u32 per publish)."""
    e = _as_records(emits)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    st = np.ascontiguousarray(states, dtype=np.uint8)
    npub = len(off) - 1
    chosen = np.zeros(max(int(off[-1]) if npub >= 0 else 0, 1), dtype=np.uint8)
    failed = np.zeros(max(npub, 1), dtype=np.uint32)
    _lib().shared_oracle_select(e.ctypes.data, off.ctypes.data, npub, POLICIES[policy], seed, pub_seq,
                                st.ctypes.data, len(st), local_node, chosen.ctypes.data, failed.ctypes.data)
    return chosen[:int(off[-1])], failed[:npub]


def select_timed(emits, offsets, policy: str, seed: int, states, local_node: int, reps: int, threads: int) -> float:
    """CPU baseline: seconds for `reps` passes on `threads` threads."""
    e = _as_records(emits)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    st = np.ascontiguousarray(states, dtype=np.uint8)
    chosen = np.zeros(max(int(off[-1]), 1), dtype=np.uint8)
    ns = _lib().shared_oracle_select_timed(e.ctypes.data, off.ctypes.data, len(off) - 1, POLICIES[policy], seed,
                                           st.ctypes.data, len(st), local_node, chosen.ctypes.data, reps, threads)
    return ns * 1e-9
