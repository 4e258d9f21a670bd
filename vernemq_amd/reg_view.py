"""``RegGpuView`` — the host-side mirror of a ``vmq_reg_view`` module backed by
the MI355X matcher (libvmqgpu).

It exposes the reference's view interface for the hot path:

* ``fold(subscriber_id, topic, fold_fun, acc)`` — ``vmq_reg_view`` callback
  (apps/vmq_server/src/vmq_reg_view.erl:20-27; vmq_reg_trie.erl:59-98): the
  fold fun is called as ``fold_fun(entry, subscriber_id, acc)`` once per
  emission, entry being ``(subscriber_id, subinfo)``,
  ``(node, group, subscriber_id, subinfo)`` or ``node`` exactly as in
  vmq_reg_trie.erl:83, :97.
* ``handle_event(event)`` — what the view's gen_server does with a
  subscriber-store event (vmq_reg_trie.erl:198-251).
* ``initialize(tuples)`` — ``initialize_trie/2`` bulk load (:305-316).
* ``stats()`` — ``{NrOfSubs + NrOfRemoteSubs, Memory}`` (:101-112).

Batches are the native unit: ``fold_batch`` / ``match_arrays`` match many
publishes in one device call, which is how a batching ``vmq_reg_gpu_view``
gen_server serves concurrent ``fold/4`` callers.

Erlang terms are interned here: mountpoints, nodes, SubscriberIds and
SubInfos become dense uint32 ids; topic words go through the library's own
dictionary so filters and publishes share one id space.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from . import subscriber as vsub
from .topic import validate_topic

OP_DTYPE = np.dtype([(n, "<u4") for n in
                     ("kind", "mountpoint", "word_off", "nwords", "node", "subscriber", "subinfo", "reserved")])
PUB_DTYPE = np.dtype([(n, "<u4") for n in ("mountpoint", "word_off", "nwords", "flags")])
EMIT_DTYPE = np.dtype([(n, "<u4") for n in ("kind_node", "group", "subscriber", "subinfo")])
RANGE_DTYPE = np.dtype([("off", "<u4"), ("count", "<u4")])


def _subinfo_key(si):
    if isinstance(si, int):
        return si
    qos, opts = si
    return (qos, tuple(sorted(opts.items())))


class Interner:
    """Dense ids for hashable terms (id -> term kept for decoding)."""

    def __init__(self, first=()):
        self.ids, self.terms = {}, []
        for t in first:
            self.get(t)

    def get(self, term, key=None):
        k = term if key is None else key
        i = self.ids.get(k)
        if i is None:
            i = len(self.terms)
            self.ids[k] = i
            self.terms.append(term)
        return i

    def __len__(self):
        return len(self.terms)


class RegGpuView:
    def __init__(self, node: str = "nonode@nohost", device: int = 0, nodes=(), max_mountpoints: int = 1024,
                 hints: dict | None = None, replica: bool = False):
        self._L = _lib.lib()
        self.node = node
        self.nodes = Interner([node] + [n for n in nodes if n != node])   # node() is id 0
        self.mountpoints = Interner([""])
        self.subscribers = Interner()
        self.subinfos = Interner()
        self._words: dict = {b"+": _lib.WORD_PLUS, b"#": _lib.WORD_HASH, b"$share": _lib.WORD_SHARE}
        self._word_text: dict = {v: k for k, v in self._words.items()}
        cfg = _lib.Config()
        cfg.device = device
        cfg.local_node = 0
        cfg.max_nodes = _lib.MAX_NODES
        cfg.max_mountpoints = max_mountpoints
        cfg.flags = _lib.CFG_REPLICA if replica else 0
        for k, v in (hints or {}).items():
            setattr(cfg, "hint_" + k, int(v))
        err = ctypes.c_int(0)
        h = self._L.vmqg_create(ctypes.byref(cfg), ctypes.byref(err))
        if not h:
            raise _lib.VmqgError(err.value, "vmqg_create")
        self._h = h
        self.device = device
        # the initial root range only: a new mountpoint past it grows the
        # roots (vmq_reg_trie has no mountpoint limit); an unknown mountpoint
        # is prepared as NONE, an id no root ever takes
        self.max_mountpoints = max_mountpoints

    def close(self):
        if getattr(self, "_h", None):
            self._L.vmqg_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ words
    def intern_words(self, words, create: bool = True) -> np.ndarray:
        """Word bytes -> library word ids (unseen words: created, or UNKNOWN)."""
        words = list(words)
        out = np.empty(len(words), dtype=np.uint32)
        todo = [i for i, w in enumerate(words) if w not in self._words]
        for i, w in enumerate(words):
            v = self._words.get(w)
            if v is not None:
                out[i] = v
        if todo:
            if not create:
                out[todo] = _lib.WORD_UNKNOWN
                return out
            blob = b"".join(words[i] for i in todo)
            offs = np.zeros(len(todo) + 1, dtype=np.uint64)
            offs[1:] = np.cumsum([len(words[i]) for i in todo])
            ids = np.empty(len(todo), dtype=np.uint32)
            _lib.check(self._L.vmqg_intern_words(self._h, blob, offs.ctypes.data, len(todo), 1,
                                                 ids.ctypes.data), "vmqg_intern_words")
            for j, i in enumerate(todo):
                self._words[words[i]] = int(ids[j])
                self._word_text[int(ids[j])] = words[i]
                out[i] = ids[j]
        return out

    def word_text(self, wid: int) -> bytes:
        return self._word_text[wid]

    def reclaim_words(self) -> int:
        """Drops the words no subscription holds any more (vmqg_dict_grace_token +
        vmqg_dict_release: this mirror has no concurrent readers, so the grace
        period is over at once); their ids may be reused, so the word -> id
        cache starts afresh.  Returns the words released so far."""
        tok = self._L.vmqg_dict_grace_token(self._h)
        _lib.check(self._L.vmqg_dict_release(self._h, tok), "vmqg_dict_release")
        self._words = {b"+": _lib.WORD_PLUS, b"#": _lib.WORD_HASH, b"$share": _lib.WORD_SHARE}
        return self.stats_raw()["words_released"]

    # ------------------------------------------------------------ deltas
    def _ops_array(self, ops):
        """ops: iterable of (kind 'add'|'del', subscriber_id, topic, subinfo, node)."""
        ops = list(ops)
        arr = np.zeros(len(ops), dtype=OP_DTYPE)
        allw = []
        off = 0
        for i, (kind, sid, topic, si, node) in enumerate(ops):
            mp = sid[0]
            arr[i] = (_lib.OP_ADD if kind == "add" else _lib.OP_DEL, self.mountpoints.get(mp), off,
                      len(topic), self.nodes.get(node), self.subscribers.get(sid),
                      self.subinfos.get(si, _subinfo_key(si)), 0)
            allw.extend(topic)
            off += len(topic)
        if len(self.nodes) > _lib.MAX_NODES:
            raise _lib.VmqgError(_lib.E_LIMIT, "nodes")
        return arr, self.intern_words(allw, create=True)

    def apply_op_arrays(self, ops: np.ndarray, words: np.ndarray) -> int:
        """Low-level: apply an OP_DTYPE array whose ids are already interned."""
        ops = np.ascontiguousarray(ops, dtype=OP_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint32)
        ep = ctypes.c_uint64(0)
        _lib.check(self._L.vmqg_apply_ops(self._h, ops.ctypes.data, len(ops), words.ctypes.data, len(words),
                                          ctypes.byref(ep)), "vmqg_apply_ops")
        return ep.value

    def apply_ops(self, ops) -> int:
        arr, words = self._ops_array(ops)
        return self.apply_op_arrays(arr, words)

    def handle_event(self, event) -> int:
        """One {updated|deleted, {vmq,subscriber}, ...} event (vmq_reg_trie.erl:240-251)."""
        return self.handle_events([event])

    def handle_events(self, events) -> int:
        ops = []
        for ev in events:
            ops.extend(vsub.event_ops(ev, self.node))
        return self.apply_ops(ops)

    def initialize(self, tuples) -> int:
        """initialize_trie/2 (vmq_reg_trie.erl:305-316) over
        (mountpoint, topic, (subscriber_id, subinfo, node)) tuples."""
        return self.apply_ops(("add", sid, topic, si, node) for _mp, topic, (sid, si, node) in tuples)

    # ------------------------------------------------------------ publishes
    def prepare(self, pubs):
        """pubs: iterable of (mountpoint, topic) with topic a word tuple or the
        raw topic bytes -> (PUB_DTYPE array, word id array)."""
        pubs = list(pubs)
        arr = np.zeros(len(pubs), dtype=PUB_DTYPE)
        allw = []
        off = 0
        for i, (mp, topic) in enumerate(pubs):
            if isinstance(topic, (bytes, bytearray)):
                st, words = validate_topic("publish", bytes(topic))
                if st != "ok":
                    raise ValueError("invalid publish topic %r: %s" % (topic, words))
                topic = words
            mid = self.mountpoints.ids.get(mp, _lib.NONE)   # unknown MP: matches nothing
            flags = _lib.PUB_DOLLAR if topic and topic[0][:1] == b"$" else 0
            arr[i] = (mid, off, len(topic), flags)
            allw.extend(topic)
            off += len(topic)
        return arr, self.intern_words(allw, create=False)

    def prepare_word_lists(self, pubs):
        """pubs: iterable of (mountpoint, word tuple) -> (PUB_DTYPE array, word
        id array) through the library's vmqg_prepare_word_lists: the Topic list
        exactly as fold/4 receives it (vmq_reg_trie.erl:59-66) — no split, no
        validation; "+" / "#" words are the literal words, any word no filter
        has (one holding a '/', say) is UNKNOWN, an empty list has no words."""
        pubs = list(pubs)
        n = len(pubs)
        mps = np.array([self.mountpoints.ids.get(mp, _lib.NONE) for mp, _ in pubs], dtype=np.uint32)
        counts = np.array([len(t) for _, t in pubs], dtype=np.uint32)
        flat = [bytes(w) for _, t in pubs for w in t]
        nw = len(flat)
        bufs = [ctypes.create_string_buffer(w, max(1, len(w))) for w in flat]
        ptrs = (ctypes.c_void_p * max(1, nw))(*[ctypes.addressof(b) for b in bufs])
        lens = np.array([len(w) for w in flat] or [0], dtype=np.uint64)
        arr = np.zeros(max(1, n), dtype=PUB_DTYPE)
        words = np.zeros(max(1, nw), dtype=np.uint32)
        got = ctypes.c_size_t(0)
        _lib.check(self._L.vmqg_prepare_word_lists(self._h, n, mps.ctypes.data, counts.ctypes.data, ptrs,
                                                   lens.ctypes.data, arr.ctypes.data, words.ctypes.data, nw,
                                                   ctypes.byref(got)), "vmqg_prepare_word_lists")
        assert got.value == nw
        return arr[:n], words[:nw]

    def match_arrays(self, pubs: np.ndarray, words: np.ndarray, out_cap: int | None = None):
        """Device match of a prepared batch -> (EMIT_DTYPE records, uint64 offsets[n+1])."""
        pubs = np.ascontiguousarray(pubs, dtype=PUB_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint32)
        offs = np.zeros(len(pubs) + 1, dtype=np.uint64)
        cap = out_cap if out_cap is not None else max(1024, 8 * len(pubs))
        while True:
            out = np.zeros(cap, dtype=EMIT_DTYPE)
            n = ctypes.c_size_t(0)
            rc = self._L.vmqg_match_batch(self._h, pubs.ctypes.data, len(pubs), words.ctypes.data, len(words),
                                          out.ctypes.data, cap, ctypes.byref(n), offs.ctypes.data)
            if rc == _lib.E_OVERFLOW and n.value > cap:
                cap = int(n.value)
                continue
            _lib.check(rc, "vmqg_match_batch")
            return out[: n.value], offs

    def match_ranges(self, pubs: np.ndarray, words: np.ndarray, out_cap: int | None = None):
        """Range-mode match (vmqg_match_ranges) -> (RANGE_DTYPE entries,
        uint64 offsets[n+1]).  count > 0: records [off, off + count) of
        records(); count == 0: remote node `off`."""
        pubs = np.ascontiguousarray(pubs, dtype=PUB_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint32)
        offs = np.zeros(len(pubs) + 1, dtype=np.uint64)
        cap = out_cap if out_cap is not None else max(1024, 2 * len(pubs))
        while True:
            out = np.zeros(cap, dtype=RANGE_DTYPE)
            n = ctypes.c_size_t(0)
            rc = self._L.vmqg_match_ranges(self._h, pubs.ctypes.data, len(pubs), words.ctypes.data, len(words),
                                           out.ctypes.data, cap, ctypes.byref(n), offs.ctypes.data)
            if rc == _lib.E_OVERFLOW and n.value > cap:
                cap = int(n.value)
                continue
            _lib.check(rc, "vmqg_match_ranges")
            return out[: n.value], offs

    def epoch(self) -> int:
        """The table epoch a match queued now sees (vmqg_epoch)."""
        e = ctypes.c_uint64()
        _lib.check(self._L.vmqg_epoch(self._h, ctypes.byref(e)), "vmqg_epoch")
        return e.value

    def records(self, epoch: int | None = None) -> np.ndarray:
        """Host view (copy) of the record table that ranges index
        (vmqg_records); with `epoch`, the table for range results of that
        epoch (vmqg_records_at: raises VmqgError E_STATE when a later apply
        rewrote record slots)."""
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        if epoch is None:
            _lib.check(self._L.vmqg_records(self._h, ctypes.byref(p), ctypes.byref(n)), "vmqg_records")
        else:
            _lib.check(self._L.vmqg_records_at(self._h, epoch, ctypes.byref(p), ctypes.byref(n)), "vmqg_records_at")
        if not n.value:
            return np.zeros(0, dtype=EMIT_DTYPE)
        buf = (ctypes.c_uint8 * (n.value * 16)).from_address(p.value)
        return np.frombuffer(buf, dtype=EMIT_DTYPE).copy()

    def expand_ranges(self, rng: np.ndarray, offs: np.ndarray, recs: np.ndarray | None = None):
        """Range entries -> (EMIT_DTYPE records, offsets): the FoldFun
        arguments in the order the ranges give them (host-side expansion, as
        the NIF does it)."""
        recs = self.records() if recs is None else recs
        cnt = rng["count"].astype(np.int64)
        per = np.where(cnt > 0, cnt, 1)
        starts = np.concatenate([[0], np.cumsum(per)])
        out = np.zeros(int(starts[-1]), dtype=EMIT_DTYPE)
        idx = np.repeat(rng["off"].astype(np.int64), per) + (np.arange(int(starts[-1])) - np.repeat(starts[:-1], per))
        isrec = np.repeat(cnt > 0, per)
        out[isrec] = recs[idx[isrec]]
        rem = out[~isrec]
        rem["kind_node"] = (_lib.EMIT_REMOTE << 24) | np.repeat(rng["off"], per)[~isrec]
        rem["group"] = rem["subscriber"] = rem["subinfo"] = _lib.NONE
        out[~isrec] = rem
        n_ent = np.diff(offs.astype(np.int64))
        sums = np.zeros(len(n_ent), dtype=np.int64)
        np.add.at(sums, np.repeat(np.arange(len(n_ent)), n_ent), per)
        eoffs = np.concatenate([[0], np.cumsum(sums)])
        return out, eoffs.astype(np.uint64)

    def decode(self, rec, sub_term=None) -> object:
        """One 16-B record -> the FoldFun entry term.  sub_term(id): the
        SubscriberId term of an id the caller chose itself (a lean workload's
        client index, workloads.Workload.client_term); default: this view's
        subscriber interner."""
        kind, node = int(rec["kind_node"]) >> 24, int(rec["kind_node"]) & 0xFFFFFF
        sub = sub_term or self.subscribers.terms.__getitem__
        if kind == _lib.EMIT_LOCAL:
            return (sub(int(rec["subscriber"])), self.subinfos.terms[rec["subinfo"]])
        if kind == _lib.EMIT_GROUP:
            return (self.nodes.terms[node], self._word_text[int(rec["group"])],
                    sub(int(rec["subscriber"])), self.subinfos.terms[rec["subinfo"]])
        return self.nodes.terms[node]

    def fold_batch(self, pubs):
        """Match (mountpoint, topic) publishes -> list of FoldFun entry lists."""
        arr, words = self.prepare(pubs)
        recs, offs = self.match_arrays(arr, words)
        return [[self.decode(recs[j]) for j in range(int(offs[i]), int(offs[i + 1]))] for i in range(len(arr))]

    def fold(self, subscriber_id, topic, fold_fun, acc):
        """vmq_reg_view fold/4 (vmq_reg_view.erl:20-27 / vmq_reg_trie.erl:59-66)."""
        for entry in self.fold_batch([(subscriber_id[0], tuple(topic))])[0]:
            acc = fold_fun(entry, subscriber_id, acc)
        return acc

    # ------------------------------------------------------------ device path
    def match_device(self, d_pubs: int, npub: int, d_words: int, d_out: int, out_cap: int, d_offsets: int,
                     stream: int = 0):
        _lib.check(self._L.vmqg_match_device(self._h, d_pubs, npub, d_words, d_out, out_cap, d_offsets,
                                             stream or None), "vmqg_match_device")

    def match_status(self, stream: int = 0) -> int:
        return self._L.vmqg_match_status(self._h, stream or None)

    def release_stream(self, stream: int):
        """Before destroying a stream passed to this view (vmqg_release_stream)."""
        _lib.check(self._L.vmqg_release_stream(self._h, stream or None), "vmqg_release_stream")

    def set_option(self, name: str, value: int):
        """Kernel tuning knob (vmqg_set_option): "fast_g" 1|2|4, "nt_stores" 0|1, "count_bpc" / "emit_bpc"."""
        _lib.check(self._L.vmqg_set_option(self._h, name.encode(), int(value)), "vmqg_set_option")

    def set_timing(self, on: bool):
        _lib.check(self._L.vmqg_set_timing(self._h, 1 if on else 0), "vmqg_set_timing")

    def kernel_times(self):
        c, e, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        _lib.check(self._L.vmqg_kernel_times(self._h, ctypes.byref(c), ctypes.byref(e), ctypes.byref(n)),
                   "vmqg_kernel_times")
        return c.value, e.value, n.value

    STAGES = ("count", "count_wave", "scan", "emit", "emit_wave")

    def stage_times(self) -> dict:
        """Average ns per launch of all five kernels of a match call
        (vmqg_kernel_times_ex), keyed by STAGES, plus "launches"."""
        ns, n = (ctypes.c_double * len(self.STAGES))(), ctypes.c_uint64()
        _lib.check(self._L.vmqg_kernel_times_ex(self._h, ns, ctypes.byref(n)), "vmqg_kernel_times_ex")
        out = {k: ns[i] for i, k in enumerate(self.STAGES)}
        out["launches"] = n.value
        return out

    # ------------------------------------------------------------ replication
    def arena(self):
        p, b = ctypes.c_void_p(), ctypes.c_uint64()
        lay = (ctypes.c_uint8 * _lib.LAYOUT_BYTES)()
        _lib.check(self._L.vmqg_arena(self._h, ctypes.byref(p), ctypes.byref(b), lay), "vmqg_arena")
        return p.value or 0, b.value, bytes(lay)

    def export_image(self) -> "np.ndarray":
        """Host copy of the arena image (primary): what replicas receive."""
        _, nbytes, _ = self.arena()
        img = np.empty(nbytes, dtype=np.uint8)
        _lib.check(self._L.vmqg_export_image(self._h, img.ctypes.data, nbytes), "vmqg_export_image")
        return img

    def replica_load(self, layout: bytes, d_src: int, stream: int = 0):
        lay = (ctypes.c_uint8 * _lib.LAYOUT_BYTES).from_buffer_copy(layout)
        _lib.check(self._L.vmqg_replica_load(self._h, lay, d_src, stream or None), "vmqg_replica_load")

    def last_patches(self):
        p, b, full = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int()
        _lib.check(self._L.vmqg_last_patches(self._h, ctypes.byref(p), ctypes.byref(b), ctypes.byref(full)),
                   "vmqg_last_patches")
        data = ctypes.string_at(p.value, b.value) if b.value else b""
        return data, bool(full.value)

    def replica_sync_layout(self, layout: bytes):
        lay = (ctypes.c_uint8 * _lib.LAYOUT_BYTES).from_buffer_copy(layout)
        _lib.check(self._L.vmqg_replica_sync_layout(self._h, lay), "vmqg_replica_sync_layout")

    def match_ranges_device(self, d_pubs: int, npub: int, d_words: int, d_out: int, out_cap: int, d_offsets: int,
                            stream: int = 0):
        _lib.check(self._L.vmqg_match_ranges_device(self._h, d_pubs, npub, d_words, d_out, out_cap, d_offsets,
                                                    stream or None), "vmqg_match_ranges_device")

    def apply_patches_device(self, d_patches: int, nbytes: int, stream: int = 0):
        _lib.check(self._L.vmqg_apply_patches_device(self._h, d_patches, nbytes, stream or None),
                   "vmqg_apply_patches_device")

    # ------------------------------------------------------------ introspection
    def stats_raw(self) -> dict:
        s = _lib.Stats()
        _lib.check(self._L.vmqg_stats(self._h, ctypes.byref(s)), "vmqg_stats")
        return {k: getattr(s, k) for k, _ in _lib.Stats._fields_}

    def stats(self):
        """stats/0 (vmq_reg_trie.erl:101-112): (NrOfSubs + NrOfRemoteSubs, bytes)."""
        s = self.stats_raw()
        return s["subs"], s["device_bytes"]

    def dump_raw(self) -> str:
        p, n = ctypes.c_char_p(), ctypes.c_size_t()
        _lib.check(self._L.vmqg_dump(self._h, ctypes.byref(p), ctypes.byref(n)), "vmqg_dump")
        return ctypes.string_at(p, n.value).decode()
