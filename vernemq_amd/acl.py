"""``AclGpu`` — host-side mirror of VerneMQ's file-based ACL plugin
``vmq_acl`` backed by the MI355X ACL checker (libvmqgpu, include/vmqa.h).

Interface (apps/vmq_acl/src/vmq_acl.erl):

* ``load_from_list(lines)`` — load_from_list/1 (:128-144): age the six
  tables, parse the lines (parse_acl_line/2, :146-177; in/3, :219-231),
  delete what was not re-inserted.  A line no clause takes raises
  ``AclLoadCrash`` with the tables as far as the load got (the reference's
  function_clause: del_aged_entries never runs) — the device holds exactly
  that state too.  ``load_from_file(path)`` (:114-126) reads the lines.
* ``check(type, topic, user, subscriber_id)`` — check/4 (:179-188):
  ``type`` "read" | "write", ``user`` bytes or None (``undefined``),
  ``subscriber_id`` = (mountpoint str, client id bytes).
* ``auth_on_subscribe(user, sid, [(topic, qos)])`` / ``auth_on_publish(user,
  sid, topic, ...)`` — the hooks (:78-93): "ok" or "next".

The batch (``check_batch`` / ``check_arrays``) is the native unit: the
checks of a publish burst become one device call.  Topic words, user names,
client ids and mountpoints are word ids: interned ones from the context's
dictionary, others batch-local ids >= VMQA_EPHEMERAL (equal ids <=> equal
strings within the batch).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .topic import validate_topic

RULE_DTYPE = np.dtype([(n, "<u4") for n in ("type", "table", "user", "word_off", "nwords", "reserved")])
REQ_DTYPE = np.dtype([(n, "<u4") for n in ("type", "user", "client", "mountpoint", "word_off", "nwords")])
TYPES = {"read": _lib.A_READ, "write": _lib.A_WRITE}


_ALL, _PATTERN = object(), object()   # the parse-time atoms `all` and `pattern`


class AclLoadCrash(Exception):
    """The reference's parse_acl_line/2 (or in/3) would crash on this line."""


class AclGpu:
    def __init__(self, device: int = 0):
        self._L = _lib.lib()
        cfg = _lib.AConfig()
        cfg.device = device
        err = ctypes.c_int(0)
        self._h = self._L.vmqa_create(ctypes.byref(cfg), ctypes.byref(err))
        if not self._h:
            raise _lib.VmqgError(err.value, "vmqa_create")
        self.device = device
        self._words = {b"+": _lib.WORD_PLUS, b"#": _lib.WORD_HASH, b"$share": _lib.WORD_SHARE,
                       b"%u": _lib.A_WORD_USER, b"%c": _lib.A_WORD_CLIENT, b"%m": _lib.A_WORD_MOUNTPOINT}
        # the six ets sets: (type, table) -> {key: 1 fresh | 2 aged}; key =
        # topic words (all, pattern) or (user, topic words) (user)
        self.tables = {(t, k): {} for t in ("read", "write") for k in ("all", "user", "pattern")}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.vmqa_destroy(h)
            self._h = None

    # ------------------------------------------------------------ words
    def intern_words(self, words, create: bool) -> np.ndarray:
        """Dictionary ids (create=False: unseen words -> WORD_UNKNOWN)."""
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
            _lib.check(self._L.vmqa_intern_words(self._h, blob, offs.ctypes.data, len(todo), 1 if create else 0,
                                                 ids.ctypes.data), "vmqa_intern_words")
            for k, i in enumerate(todo):
                out[i] = ids[k]
                if create or ids[k] != _lib.WORD_UNKNOWN:
                    self._words[words[i]] = int(ids[k])
        return out

    # ------------------------------------------------------------ loading
    def _in(self, ty: str, user, topic: bytes):
        """in/3 (:219-231): the last byte is dropped (newline or not), the rest
        validated as a subscription; invalid topics are skipped (a warning)."""
        if len(topic) == 0:
            raise AclLoadCrash("empty topic")          # TopicLen = -1: badmatch
        ok, words = validate_topic("subscribe", topic[:-1])
        if ok != "ok":
            return
        if user is _PATTERN:
            self.tables[(ty, "pattern")][words] = 1
        elif user is _ALL:
            self.tables[(ty, "all")][words] = 1
        else:
            self.tables[(ty, "user")][(user, words)] = 1

    def _parse(self, lines):
        """parse_acl_line/2 (:146-177), clause order kept.  `user` is the
        atom ``all`` until a "user" line."""
        user = _ALL
        for line in lines:
            if line.startswith(b"#"):                                     # :146-148
                continue
            for prefix, types in ((b"topic read ", ("read",)), (b"topic write ", ("write",)),
                                  (b"topic ", ("read", "write"))):
                if line.startswith(prefix):                               # :149-158
                    for ty in types:
                        self._in(ty, user, line[len(prefix):])
                    break
            else:
                if line.startswith(b"user "):                             # :159-162
                    rest = line[5:]
                    if len(rest) == 0:
                        raise AclLoadCrash("user line without a name")    # UserLen = -1: badmatch
                    user = rest[:-1]
                    continue
                for prefix, types in ((b"pattern read ", ("read",)), (b"pattern write ", ("write",)),
                                      (b"pattern ", ("read", "write"))):
                    if line.startswith(prefix):                           # :163-172
                        for ty in types:
                            self._in(ty, _PATTERN, line[len(prefix):])
                        break
                else:
                    if line == b"\n":                                     # :173-174
                        continue
                    raise AclLoadCrash("no parse_acl_line clause for %r" % line[:64])

    def load_from_list(self, lines):
        for t in self.tables.values():                                    # age_entries/0 (:268-271)
            for k in t:
                t[k] = 2
        try:
            self._parse(list(lines))
        except AclLoadCrash:
            self._push()        # the device holds the partial state the reference keeps
            raise
        for key, t in self.tables.items():                                # del_aged_entries/0 (:273-276)
            self.tables[key] = {k: v for k, v in t.items() if v != 2}
        self._push()

    def load_from_file(self, path):
        with open(path, "rb") as f:
            self.load_from_list(f.readlines())

    def _push(self):
        """The six tables -> vmqa_load (one device image)."""
        rows, flat = [], []
        for (ty, table), t in self.tables.items():
            for key in t:
                user, words = (key if table == "user" else (None, key))
                uid = int(self.intern_words([user], create=True)[0]) if table == "user" else 0
                ids = self.intern_words(list(words), create=True)
                rows.append((TYPES[ty], {"all": _lib.A_TABLE_ALL, "user": _lib.A_TABLE_USER,
                                         "pattern": _lib.A_TABLE_PATTERN}[table], uid, len(flat), len(ids), 0))
                flat.extend(int(x) for x in ids)
        arr = np.array(rows, dtype=RULE_DTYPE) if rows else np.zeros(0, RULE_DTYPE)
        words = np.array(flat, dtype=np.uint32)
        _lib.check(self._L.vmqa_load(self._h, arr.ctypes.data, len(arr), words.ctypes.data, len(words)), "vmqa_load")

    # ------------------------------------------------------------ checking
    def prepare(self, reqs):
        """[(type, topic words, user | None, mountpoint, client id)] ->
        (REQ_DTYPE array, word ids); strings outside the dictionary get
        batch-local ids."""
        eph: dict = {}

        def wid(b: bytes) -> int:
            j = self._words.get(b)
            if j is None:
                j = int(self.intern_words([b], create=False)[0])
                if j == _lib.WORD_UNKNOWN:
                    j = eph.setdefault(b, _lib.A_EPHEMERAL + len(eph))
            return j

        arr = np.zeros(len(reqs), dtype=REQ_DTYPE)
        flat = []
        for i, (ty, topic, user, mp, client) in enumerate(reqs):
            mpb = mp.encode() if isinstance(mp, str) else mp
            arr[i] = (TYPES[ty], _lib.A_NO_USER if user is None else wid(user), wid(client), wid(mpb),
                      len(flat), len(topic))
            flat.extend(wid(w) for w in topic)
        return arr, np.array(flat, dtype=np.uint32)

    def check_arrays(self, reqs: np.ndarray, words: np.ndarray) -> np.ndarray:
        """vmqa_check_batch: uint8 verdict per request."""
        reqs = np.ascontiguousarray(reqs, dtype=REQ_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint32)
        out = np.zeros(len(reqs), dtype=np.uint8)
        _lib.check(self._L.vmqa_check_batch(self._h, reqs.ctypes.data, len(reqs), words.ctypes.data, len(words),
                                            out.ctypes.data), "vmqa_check_batch")
        return out

    def check_batch(self, reqs) -> np.ndarray:
        if any(len(r[1]) == 0 for r in reqs):
            raise ValueError("check/4 has no clause for an empty topic")
        if not reqs:
            return np.zeros(0, dtype=np.uint8)
        return self.check_arrays(*self.prepare(reqs))

    def check_device(self, d_reqs: int, n: int, d_words: int, d_out: int, stream: int = 0):
        _lib.check(self._L.vmqa_check_device(self._h, d_reqs, n, d_words, d_out, stream or None),
                   "vmqa_check_device")

    def check_status(self, stream: int = 0) -> int:
        return self._L.vmqa_check_status(self._h, stream or None)

    def check(self, ty: str, topic, user, subscriber_id) -> bool:
        mp, client = subscriber_id
        return bool(self.check_batch([(ty, tuple(topic), user, mp, client)])[0])

    def auth_on_subscribe(self, user, subscriber_id, topics) -> str:
        """:78-85 — every topic must pass a read check."""
        if not topics:
            return "ok"
        mp, client = subscriber_id
        res = self.check_batch([("read", tuple(t), user, mp, client) for t, _qos in topics])
        return "ok" if bool(np.all(res == 1)) else "next"

    def auth_on_publish(self, user, subscriber_id, topic, *_rest) -> str:
        """:87-93 (QoS, payload and retain flag do not enter the check)."""
        return "ok" if self.check("write", topic, user, subscriber_id) else "next"

    # ------------------------------------------------------------ introspection
    def dump(self):
        """The six tables, one sorted line per row ("read all [a,b]",
        "write user u [x,#]", "read pattern [%u]")."""
        lines = []
        for (ty, table), t in self.tables.items():
            for key in t:
                user, words = (key if table == "user" else (None, key))
                show = "[" + ",".join(w.decode("latin-1") for w in words) + "]"
                if table == "user":
                    lines.append("%s user %s %s" % (ty, user.decode("latin-1"), show))
                else:
                    lines.append("%s %s %s" % (ty, table, show))
        return sorted(lines)

    def stats_raw(self) -> dict:
        st = _lib.AStats()
        _lib.check(self._L.vmqa_stats(self._h, ctypes.byref(st)), "vmqa_stats")
        return {n: int(getattr(st, n)) for n, _ in _lib.AStats._fields_}

    def set_timing(self, on: bool):
        _lib.check(self._L.vmqa_set_timing(self._h, 1 if on else 0), "vmqa_set_timing")

    def kernel_times(self):
        c, n = ctypes.c_double(), ctypes.c_uint64()
        _lib.check(self._L.vmqa_kernel_times(self._h, ctypes.byref(c), ctypes.byref(n)), "vmqa_kernel_times")
        return c.value, n.value
