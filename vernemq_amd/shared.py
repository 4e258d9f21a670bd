"""``SharedGpu`` — host-side mirror of VerneMQ's shared-subscription dispatch
backed by the MI355X dispatcher (libvmqgpu, include/vmqs.h).

Interface (apps/vmq_server/src/vmq_shared_subscriptions.erl and the fold fun
of vmq_reg.erl that feeds it):

* ``set_states({subscriber_id: state})`` — the queue state each member's
  publish_/3 meets (:75-88): "online", "offline", "draining", "not_found".
  Members never set are "online".
* ``select_batch(records, offsets, policy, seed, pub_seq)`` — publish/3
  (:18-36) for every publish of a match batch at once: for each group of
  each publish, the member that takes the message (chosen byte per record)
  and the groups that reached nobody (``{error, no_subscribers}``).
  ``policy`` is the ``shared_subscription_policy`` atom: "random",
  "prefer_local" (the default, vmq_server.app.src:91) or "local_only".
* ``route_batch(view, pubs, policy, seed, pub_seq)`` — vmq_reg:publish/5
  (vmq_reg.erl:257-261) end to end on the device: match, then dispatch; per
  publish, the local deliveries (kind A entries after the no_local rule,
  :333-335), the remote nodes (kind C) and one member per shared group.

rand:uniform() is replaced by the counter-based element key of vmqs.h, so
a choice is a pure function of (records, states, policy, seed, publish
number): parity with the CPU restatement is bit-exact and the distribution
is the reference's (uniform over the collected entries).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

POLICIES = {"random": _lib.S_RANDOM, "prefer_local": _lib.S_PREFER_LOCAL, "local_only": _lib.S_LOCAL_ONLY}
STATES = {"not_found": _lib.S_NOT_FOUND, "online": _lib.S_ONLINE, "offline": _lib.S_OFFLINE,
          "draining": _lib.S_DRAINING}


class SharedGpu:
    def __init__(self, device: int = 0, local_node: int = 0):
        """local_node: the node id that plays node() (RegGpuView interns node() as 0)."""
        self._L = _lib.lib()
        cfg = _lib.SConfig(device=device, local_node=local_node)
        err = ctypes.c_int(0)
        self._h = self._L.vmqs_create(ctypes.byref(cfg), ctypes.byref(err))
        if not self._h:
            raise _lib.VmqgError(err.value, "vmqs_create")
        self.device = device
        self.local_node = local_node

    def close(self):
        if getattr(self, "_h", None):
            self._L.vmqs_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def handle(self):
        return self._h

    def set_state_ids(self, ids, states):
        """Queue states by subscriber id (uint32) -> state code (VMQS_*)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        st = np.ascontiguousarray(states, dtype=np.uint8)
        if ids.shape != st.shape:
            raise ValueError("ids and states differ in length")
        _lib.check(self._L.vmqs_set_states(self._h, ids.ctypes.data, st.ctypes.data, len(ids)), "vmqs_set_states")

    def set_states(self, view, states: dict):
        """{subscriber_id term: "online" | "offline" | "draining" | "not_found"}."""
        ids = [view.subscribers.get(sid) for sid in states]
        self.set_state_ids(ids, [STATES[s] for s in states.values()])

    def select_batch(self, records, offsets, policy: str = "prefer_local", seed: int = 0, pub_seq: int = 0):
        """records: EMIT_DTYPE array, offsets: uint64[npub + 1] (match_arrays'
        output).  Returns (chosen uint8 per record, failed uint32 per publish)."""
        recs = np.ascontiguousarray(records)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        if len(offs) == 0:
            raise ValueError("offsets must hold npub + 1 entries (got an empty array)")
        npub = len(offs) - 1
        total = int(offs[-1]) if npub >= 0 else 0
        chosen = np.zeros(max(total, 1), dtype=np.uint8)
        failed = np.zeros(max(npub, 1), dtype=np.uint32)
        _lib.check(self._L.vmqs_select_batch(self._h, recs.ctypes.data, offs.ctypes.data, npub, POLICIES[policy],
                                             seed, pub_seq, chosen.ctypes.data, failed.ctypes.data),
                   "vmqs_select_batch")
        return chosen[:total], failed[:npub]

    # ------------------------------------------------------------ device path
    def select_device(self, d_records: int, d_offsets: int, npub: int, policy: str, seed: int, pub_seq: int,
                      d_chosen: int, d_failed: int = 0, stream: int = 0):
        _lib.check(self._L.vmqs_select_device(self._h, d_records, d_offsets, npub, POLICIES[policy], seed, pub_seq,
                                              d_chosen, d_failed or None, stream or None), "vmqs_select_device")

    def select_status(self, stream: int = 0) -> int:
        return self._L.vmqs_select_status(self._h, stream or None)

    def set_timing(self, on: bool):
        _lib.check(self._L.vmqs_set_timing(self._h, 1 if on else 0), "vmqs_set_timing")

    def kernel_times(self):
        """(average select ns, timed launches, publishes of the last checked call in tier 2)."""
        ns, n, d = ctypes.c_double(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        _lib.check(self._L.vmqs_kernel_times(self._h, ctypes.byref(ns), ctypes.byref(n), ctypes.byref(d)),
                   "vmqs_kernel_times")
        return ns.value, n.value, d.value

    # ------------------------------------------------------------ vmq_reg:publish/5
    def route_batch(self, view, pubs, policy: str = "prefer_local", seed: int = 0, pub_seq: int = 0):
        """pubs: [(publisher subscriber_id, topic)] with the MP taken from the
        subscriber id (vmq_reg.erl:257-261).  Returns per publish a dict
        {"local": [(sid, subinfo)], "remote": [node], "shared": {group: (node, sid, subinfo) | None}}."""
        arr, words = view.prepare([(sid[0], topic) for sid, topic in pubs])
        recs, offs = view.match_arrays(arr, words)
        chosen, _failed = self.select_batch(recs, offs, policy, seed, pub_seq)
        out = []
        for i, (sid, _topic) in enumerate(pubs):
            d = {"local": [], "remote": [], "shared": {}}
            for j in range(int(offs[i]), int(offs[i + 1])):
                e = view.decode(recs[j])
                kind = int(recs[j]["kind_node"]) >> 24
                if kind == _lib.EMIT_LOCAL:
                    s, info = e
                    # publish({SubscriberId, {_, #{no_local := true}}}, SubscriberId, Acc) (vmq_reg.erl:333-335)
                    if s == sid and isinstance(info, tuple) and info[1].get("no_local") is True:
                        continue
                    d["local"].append(e)
                elif kind == _lib.EMIT_GROUP:
                    node, group, s, info = e
                    d["shared"].setdefault(group, None)
                    if chosen[j]:
                        d["shared"][group] = (node, s, info)
                else:
                    d["remote"].append(e)
            out.append(d)
        return out
