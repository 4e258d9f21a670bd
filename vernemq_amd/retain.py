"""``RetainGpuSrv`` — host-side mirror of ``vmq_retain_srv`` backed by the
MI355X retained-message matcher (libvmqgpu, include/vmqr.h).

Interface (apps/vmq_server/src/vmq_retain_srv.erl):

* ``insert(mp, routing_key, message)`` — insert/3 (:68-71): the retained
  message of ``{MP, RoutingKey}``; an existing key takes the new message.
* ``delete(mp, routing_key)`` — delete/2 (:63-66).
* ``match_fold(fold_fun, acc, mp, topic)`` — match_fold/4 (:75-99): the fold
  fun is called as ``fold_fun((routing_key, message), acc)`` for every
  retained message the subscription ``topic`` receives — vmq_topic:match/2
  over the whole store for a wildcard filter, the one exact key otherwise.
* ``stats()`` — ``{Size, Memory}`` (:101-113).

Batches are the native unit (``match_fold_batch``, ``match_arrays``): a
subscribe burst (e.g. reconnecting clients, vmq_reg:deliver_retained/5)
becomes one device call.  Messages stay on the host: the device holds a
message id per retained key.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .reg_view import Interner, PUB_DTYPE

ROP_DTYPE = np.dtype([(n, "<u4") for n in ("kind", "mountpoint", "word_off", "nwords", "msg", "reserved")])


class RetainGpuSrv:
    def __init__(self, device: int = 0, max_mountpoints: int = 1024, hint_topics: int = 0):
        self._L = _lib.lib()
        cfg = _lib.RConfig()
        cfg.device = device
        cfg.max_mountpoints = max_mountpoints
        cfg.hint_topics = hint_topics
        err = ctypes.c_int(0)
        self._h = self._L.vmqr_create(ctypes.byref(cfg), ctypes.byref(err))
        if not self._h:
            raise _lib.VmqgError(err.value, "vmqr_create")
        self.device = device
        self.max_mountpoints = max_mountpoints
        self.mountpoints = Interner([""])
        self._words: dict = {b"+": _lib.WORD_PLUS, b"#": _lib.WORD_HASH, b"$share": _lib.WORD_SHARE}
        self._msgs: list = []        # msg id -> (routing_key, message) | None
        self._free: list = []
        self._key_msg: dict = {}     # (mp, routing_key) -> msg id of its live entry

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.vmqr_destroy(h)
            self._h = None

    # ------------------------------------------------------------ words
    def intern_words(self, words, create: bool) -> np.ndarray:
        """Word ids (create=False: unseen words -> WORD_UNKNOWN)."""
        out = np.empty(len(words), dtype=np.uint32)
        todo = []
        for i, w in enumerate(words):
            j = self._words.get(w)
            if j is None:
                todo.append(i)
            else:
                out[i] = j
        if todo:
            blob = b"".join(words[i] for i in todo)
            offs = np.zeros(len(todo) + 1, dtype=np.uint64)
            offs[1:] = np.cumsum([len(words[i]) for i in todo])
            ids = np.empty(len(todo), dtype=np.uint32)
            _lib.check(self._L.vmqr_intern_words(self._h, blob, offs.ctypes.data, len(todo), 1 if create else 0,
                                                 ids.ctypes.data), "vmqr_intern_words")
            for k, i in enumerate(todo):
                out[i] = ids[k]
                if create or ids[k] != _lib.WORD_UNKNOWN:
                    self._words[words[i]] = int(ids[k])
        return out

    def _mp(self, mp: str, create: bool) -> int:
        if create:   # a new mountpoint past the initial range grows the library's lists
            return self.mountpoints.get(mp)
        return self.mountpoints.ids.get(mp, _lib.NONE)   # unknown: holds nothing

    # ------------------------------------------------------------ deltas
    def apply_op_arrays(self, ops: np.ndarray, words: np.ndarray):
        ops = np.ascontiguousarray(ops, dtype=ROP_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint32)
        _lib.check(self._L.vmqr_apply(self._h, ops.ctypes.data, len(ops), words.ctypes.data, len(words)),
                   "vmqr_apply")

    def _new_msg(self, routing_key, message) -> int:
        if self._free:
            i = self._free.pop()
            self._msgs[i] = (routing_key, message)
        else:
            i = len(self._msgs)
            self._msgs.append((routing_key, message))
        return i

    def apply(self, ops):
        """ops: [("insert", mp, routing_key, message) | ("delete", mp, routing_key)],
        applied in order (one device patch upload)."""
        rows, flat = [], []
        for op in ops:
            kind, mp, rk = op[0], op[1], tuple(op[2])
            ids = self.intern_words(list(rk), create=True)
            old = self._key_msg.pop((mp, rk), None)   # replaced / deleted: its id is free again
            if old is not None:
                self._msgs[old] = None
                self._free.append(old)
            msg = 0
            if kind == "insert":
                msg = self._new_msg(rk, op[3])
                self._key_msg[(mp, rk)] = msg
            rows.append((_lib.ROP_INSERT if kind == "insert" else _lib.ROP_DELETE, self._mp(mp, True),
                         len(flat), len(ids), msg, 0))
            flat.extend(int(x) for x in ids)
        arr = np.array(rows, dtype=ROP_DTYPE) if rows else np.zeros(0, ROP_DTYPE)
        self.apply_op_arrays(arr, np.array(flat, dtype=np.uint32))

    def insert(self, mp: str, routing_key, message):
        self.apply([("insert", mp, routing_key, message)])

    def delete(self, mp: str, routing_key):
        self.apply([("delete", mp, routing_key)])

    # ------------------------------------------------------------ matching
    def prepare(self, filters):
        """[(mp, filter words)] -> (PUB_DTYPE array, word ids)."""
        arr = np.zeros(len(filters), dtype=PUB_DTYPE)
        flat = []
        for i, (mp, f) in enumerate(filters):
            ids = self.intern_words(list(f), create=False)
            arr[i] = (self._mp(mp, False), len(flat), len(ids), 0)
            flat.extend(int(x) for x in ids)
        return arr, np.array(flat, dtype=np.uint32)

    def match_arrays(self, filters: np.ndarray, words: np.ndarray, out_cap: int | None = None):
        """vmqr_match_batch: (message ids uint32, offsets uint64[n+1])."""
        filters = np.ascontiguousarray(filters, dtype=PUB_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint32)
        n = len(filters)
        cap = out_cap if out_cap is not None else max(1024, 4 * n)
        offs = np.zeros(n + 1, dtype=np.uint64)
        while True:
            out = np.empty(cap, dtype=np.uint32)
            got = ctypes.c_size_t(0)
            rc = self._L.vmqr_match_batch(self._h, filters.ctypes.data, n, words.ctypes.data, len(words),
                                          out.ctypes.data, cap, ctypes.byref(got), offs.ctypes.data)
            if rc == _lib.E_OVERFLOW:
                cap = int(got.value) + 1024
                continue
            _lib.check(rc, "vmqr_match_batch")
            return out[: got.value], offs

    def match_device(self, d_filters: int, n: int, d_words: int, d_out: int, out_cap: int, d_offsets: int,
                     stream: int = 0):
        _lib.check(self._L.vmqr_match_device(self._h, d_filters, n, d_words, d_out, out_cap, d_offsets,
                                             stream or None), "vmqr_match_device")

    def match_status(self, stream: int = 0) -> int:
        return self._L.vmqr_match_status(self._h, stream or None)

    def match_fold_batch(self, filters):
        """[(mp, filter)] -> per filter the [(routing_key, message)] match_fold folds over."""
        arr, words = self.prepare(filters)
        ids, offs = self.match_arrays(arr, words)
        return [[self._msgs[j] for j in ids[offs[i]:offs[i + 1]]] for i in range(len(filters))]

    def match_fold(self, fold_fun, acc, mp: str, topic):
        """vmq_retain_srv:match_fold/4 (FoldFun({T, Payload}, Acc))."""
        for entry in self.match_fold_batch([(mp, tuple(topic))])[0]:
            acc = fold_fun(entry, acc)
        return acc

    # ------------------------------------------------------------ introspection
    def stats_raw(self) -> dict:
        st = _lib.RStats()
        _lib.check(self._L.vmqr_stats(self._h, ctypes.byref(st)), "vmqr_stats")
        return {n: int(getattr(st, n)) for n, _ in _lib.RStats._fields_}

    def stats(self):
        """{Size, Memory} (vmq_retain_srv.erl:101-113; memory = device bytes)."""
        s = self.stats_raw()
        return s["retained"], s["device_bytes"]

    def dump(self) -> str:
        p = ctypes.c_char_p()
        n = ctypes.c_size_t()
        _lib.check(self._L.vmqr_dump(self._h, ctypes.byref(p), ctypes.byref(n)), "vmqr_dump")
        return ctypes.string_at(p, n.value).decode("latin-1")

    def set_option(self, name: str, value: int):
        """Tuning knob (vmqr_set_option): "walk_rows_hint" = rows the first
        look-back allocation of the walk covers (results unchanged)."""
        _lib.check(self._L.vmqr_set_option(self._h, name.encode(), int(value)), "vmqr_set_option")

    def set_timing(self, on: bool):
        _lib.check(self._L.vmqr_set_timing(self._h, 1 if on else 0), "vmqr_set_timing")

    def kernel_times(self):
        c, e, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        _lib.check(self._L.vmqr_kernel_times(self._h, ctypes.byref(c), ctypes.byref(e), ctypes.byref(n)),
                   "vmqr_kernel_times")
        return c.value, e.value, n.value
