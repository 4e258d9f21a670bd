"""TEST INFRASTRUCTURE ONLY — ctypes wrapper around the CPU restatement of
``vmq_retain_srv`` (oracle/vmq_retain_oracle.cpp).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module, and only as the checker.  The product package
(``vernemq_amd``) never imports it.

Terms: mountpoint ``str``; topic / filter = tuple of ``bytes`` words
(``vmq_topic:validate_topic`` output); payload = opaque ``int`` id.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from . import oracle as _o


def _lib():
    L = _o._load()
    if not getattr(L, "_retain_bound", False):
        L.retain_oracle_new.restype = ctypes.c_void_p
        L.retain_oracle_free.argtypes = [ctypes.c_void_p]
        L.retain_oracle_size.restype = ctypes.c_uint64
        L.retain_oracle_size.argtypes = [ctypes.c_void_p]
        L.retain_oracle_apply.restype = ctypes.c_int
        L.retain_oracle_apply.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.retain_oracle_match.restype = ctypes.c_long
        L.retain_oracle_match.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
        L.retain_oracle_out.restype = ctypes.POINTER(ctypes.c_uint32)
        L.retain_oracle_out.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
        L.retain_oracle_match_timed.restype = ctypes.c_longlong
        L.retain_oracle_match_timed.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_ulonglong)]
        L.retain_oracle_topic_match.restype = ctypes.c_int
        L.retain_oracle_topic_match.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.retain_oracle_has_wildcard.restype = ctypes.c_int
        L.retain_oracle_has_wildcard.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L._retain_bound = True
    return L


def _str(b) -> bytes:
    if isinstance(b, str):
        b = b.encode()
    return struct.pack("<I", len(b)) + b


def _words(ws) -> bytes:
    return struct.pack("<I", len(ws)) + b"".join(_str(w) for w in ws)


def topic_match(topic, filt) -> bool:
    """vmq_topic:match(Topic, Filter) (vmq_topic.erl:53-65)."""
    buf = _words(topic) + _words(filt)
    return _lib().retain_oracle_topic_match(buf, len(buf)) == 1


def has_wildcard(filt) -> bool:
    """vmq_retain_srv:has_wildcard/1 (vmq_retain_srv.erl:239-242)."""
    buf = _words(filt)
    return _lib().retain_oracle_has_wildcard(buf, len(buf)) == 1


class RetainOracle:
    """The ?RETAIN_CACHE ets set + match_fold/4 (vmq_retain_srv.erl:52-99)."""

    def __init__(self):
        self._L = _lib()
        self._h = self._L.retain_oracle_new()

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.retain_oracle_free(self._h)
            self._h = None

    def apply(self, ops):
        """ops: [("insert", mp, topic, payload) | ("delete", mp, topic)]."""
        parts = [struct.pack("<I", len(ops))]
        for op in ops:
            if op[0] == "insert":
                parts.append(b"\x01" + _str(op[1]) + _words(op[2]) + struct.pack("<I", op[3]))
            else:
                parts.append(b"\x02" + _str(op[1]) + _words(op[2]) + struct.pack("<I", 0))
        buf = b"".join(parts)
        if self._L.retain_oracle_apply(self._h, buf, len(buf)) != 0:
            raise ValueError("malformed retain ops")

    def size(self) -> int:
        return int(self._L.retain_oracle_size(self._h))

    @staticmethod
    def filters_bytes(filters) -> bytes:
        return struct.pack("<I", len(filters)) + b"".join(_str(mp) + _words(f) for mp, f in filters)

    def match_batch(self, filters):
        """[(mp, filter)] -> per filter the list of payload ids match_fold folds over."""
        buf = self.filters_bytes(filters)
        offs = (ctypes.c_uint64 * (len(filters) + 1))()
        n = self._L.retain_oracle_match(self._h, buf, len(buf), offs, len(filters) + 1)
        if n < 0:
            raise ValueError("malformed filters")
        cnt = ctypes.c_size_t()
        p = self._L.retain_oracle_out(self._h, ctypes.byref(cnt))
        out = np.ctypeslib.as_array(p, shape=(cnt.value,)).copy() if cnt.value else np.zeros(0, np.uint32)
        return [out[offs[i]:offs[i + 1]].tolist() for i in range(len(filters))]

    def match_timed(self, filters, reps: int):
        """(ns for `reps` passes over the batch, payloads folded per pass)."""
        buf = self.filters_bytes(filters)
        m = ctypes.c_ulonglong()
        ns = self._L.retain_oracle_match_timed(self._h, buf, len(buf), reps, ctypes.byref(m))
        if ns < 0:
            raise ValueError("malformed filters")
        return int(ns), int(m.value)
