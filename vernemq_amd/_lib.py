"""ctypes binding of libvmqgpu (include/vmqg.h, include/vmqr.h) and its in-tree build.

The library is the product: there is no Python or CPU fallback for matching.
If ``libvmqgpu.so`` is missing, :func:`lib` raises ``ImportError`` (call
:func:`build` first, or ``python -c "import __graft_entry__ as g; g.build()"``).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libvmqgpu.so")
HEADER = os.path.join(ROOT, "include", "vmqg.h")
HEADERS = [HEADER, os.path.join(ROOT, "include", "vmqr.h"), os.path.join(ROOT, "include", "vmqa.h"),
           os.path.join(ROOT, "include", "vmqs.h")]
SOURCES = [os.path.join(HERE, "csrc", f) for f in
           ("vmqg_engine.cpp", "vmqg_abi.cpp", "vmqg_kernels.hip",
            "vmqr_engine.cpp", "vmqr_abi.cpp", "vmqr_kernels.hip",
            "vmqa_engine.cpp", "vmqa_abi.cpp", "vmqa_kernels.hip",
            "vmqs_abi.cpp", "vmqs_kernels.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", f) for f in
                  ("vmqg_common.h", "vmqg_engine.h", "vmqg_kernels.h", "vmqg_lookback.h", "vmqg_chain.h",
                   "vmqg_nullorder.h",
                   "vmqr_engine.h", "vmqa_engine.h", "vmqs_engine.h")] + HEADERS

# ---- status codes / constants (vmqg.h)
OK, E_INVAL, E_OVERFLOW, E_NOMEM, E_DEVICE, E_FRONTIER, E_LIMIT, E_STATE = 0, -1, -2, -3, -4, -5, -6, -7
ERRORS = {E_INVAL: "VMQG_E_INVAL", E_OVERFLOW: "VMQG_E_OVERFLOW", E_NOMEM: "VMQG_E_NOMEM",
          E_DEVICE: "VMQG_E_DEVICE", E_FRONTIER: "VMQG_E_FRONTIER", E_LIMIT: "VMQG_E_LIMIT",
          E_STATE: "VMQG_E_STATE"}
WORD_PLUS, WORD_HASH, WORD_SHARE, WORD_UNKNOWN = 0, 1, 2, 0xFFFFFFFF
NONE = 0xFFFFFFFF
OP_ADD, OP_DEL = 1, 2
PUB_DOLLAR = 1
PUB_UNKNOWN = 2
EMIT_LOCAL, EMIT_GROUP, EMIT_REMOTE = 1, 2, 3
CFG_REPLICA = 1
LAYOUT_BYTES = 256
MAX_NODES = 4096


class VmqgError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        super().__init__("%s failed: %s (%d)" % (what, ERRORS.get(rc, "?"), rc))
        self.rc = rc


class Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("local_node", ctypes.c_uint32),
                ("max_nodes", ctypes.c_uint32), ("max_mountpoints", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("hint_edges", ctypes.c_uint64), ("hint_paths", ctypes.c_uint64),
                ("hint_keys", ctypes.c_uint64), ("hint_records", ctypes.c_uint64),
                ("hint_exact", ctypes.c_uint64)]


class Op(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in
                ("kind", "mountpoint", "word_off", "nwords", "node", "subscriber", "subinfo", "reserved")]


class Pub(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("mountpoint", "word_off", "nwords", "flags")]


class Emit(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("kind_node", "group", "subscriber", "subinfo")]


class Range(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("off", "count")]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("subs", "device_bytes", "trie_edges", "trie_nodes", "trie_topics", "subs_objects",
                 "fanout_objects", "remote_keys", "epoch", "rebuilds", "paths", "words",
                 "deferred_tier1", "deferred_tier2", "ops_applied", "apply_host_ns", "apply_upload_ns", "apply_wait_ns", "patch_bytes",
                 "image_bytes", "max_depth", "many_key", "retried", "wave_entries", "wide_entries",
                 "dedup", "dedup_walked", "error_bits", "reader_waits", "reader_wait_ns",
                 "keys", "topics", "words_retired", "words_released", "host_bytes")]


class RConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_mountpoints", ctypes.c_uint32), ("hint_topics", ctypes.c_uint64)]


class ROp(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("kind", "mountpoint", "word_off", "nwords", "msg", "reserved")]


class RStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("retained", "device_bytes", "partitions", "epoch", "rebuilds", "words")]


ROP_INSERT, ROP_DELETE = 1, 2


class AConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


class AStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("rules", "users", "device_bytes", "loads", "words")]


# vmqa.h constants
A_READ, A_WRITE = 1, 2
A_TABLE_ALL, A_TABLE_USER, A_TABLE_PATTERN = 0, 1, 2
A_WORD_USER, A_WORD_CLIENT, A_WORD_MOUNTPOINT = 3, 4, 5
A_NO_USER, A_EPHEMERAL = 0xFFFFFFFE, 0x80000000
# vmqs.h constants
S_RANDOM, S_PREFER_LOCAL, S_LOCAL_ONLY = 0, 1, 2
S_NOT_FOUND, S_ONLINE, S_OFFLINE, S_DRAINING = 0, 1, 2, 3
S_MAX_SEGMENT = 1 << 24


class SConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("local_node", ctypes.c_uint32)]


# (name, restype, argtypes) for every entry point declared in include/vmqg.h, vmqr.h and vmqa.h
_P = ctypes.c_void_p
_U32, _U64, _SZ = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
SIGNATURES = [
    ("vmqg_abi_version", ctypes.c_int, []),
    ("vmqg_replica_follow", ctypes.c_int, [_P, _P]),
    ("vmqg_dict_grace_token", _U64, [_P]),
    ("vmqg_dict_release", ctypes.c_int, [_P, _U64]),
    ("vmqg_released_ids", ctypes.c_int, [_P, _U32, ctypes.POINTER(_P), ctypes.POINTER(_SZ)]),
    ("vmqg_arena_digest", ctypes.c_int, [_P, ctypes.POINTER(_U64)]),
    ("vmqg_build_id", ctypes.c_char_p, []),
    ("vmqg_create", _P, [ctypes.POINTER(Config), ctypes.POINTER(ctypes.c_int)]),
    ("vmqg_destroy", None, [_P]),
    ("vmqg_intern_words", ctypes.c_int, [_P, _P, _P, _U32, ctypes.c_int, _P]),
    ("vmqg_prepare_publish", ctypes.c_int, [_P, _U32, ctypes.c_char_p, _SZ, _P, _U32, ctypes.POINTER(Pub)]),
    ("vmqg_prepare_publishes", ctypes.c_int, [_P, _SZ, _P, _P, _P, _P, _P, _P, _SZ, ctypes.POINTER(_SZ)]),
    ("vmqg_prepare_word_lists", ctypes.c_int, [_P, _SZ, _P, _P, _P, _P, _P, _P, _SZ, ctypes.POINTER(_SZ)]),
    ("vmqg_dict_generation", _U64, [_P]),
    ("vmqg_hbatch_new", _P, [_P]),
    ("vmqg_hbatch_free", None, [_P]),
    ("vmqg_hbatch_inputs", ctypes.c_int, [_P, _SZ, _SZ, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    ("vmqg_hbatch_submit", ctypes.c_int, [_P, _P, _SZ, _SZ, ctypes.c_int]),
    ("vmqg_hbatch_offsets", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    ("vmqg_hbatch_entries", ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    ("vmqg_apply_ops", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, ctypes.POINTER(_U64)]),
    ("vmqg_apply_stage", ctypes.c_int, [_P, _P, _SZ, _P, _SZ]),
    ("vmqg_apply_commit", ctypes.c_int, [_P, ctypes.POINTER(_U64)]),
    ("vmqg_match_batch", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, _P, _SZ, ctypes.POINTER(_SZ), _P]),
    ("vmqg_match_device", ctypes.c_int, [_P, _P, _U32, _P, _P, _U64, _P, _P]),
    ("vmqg_match_status", ctypes.c_int, [_P, _P]),
    ("vmqg_match_ranges", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, _P, _SZ, ctypes.POINTER(_SZ), _P]),
    ("vmqg_match_ranges_device", ctypes.c_int, [_P, _P, _U32, _P, _P, _U64, _P, _P]),
    ("vmqg_records", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_U64)]),
    ("vmqg_release_stream", ctypes.c_int, [_P, _P]),
    ("vmqr_release_stream", ctypes.c_int, [_P, _P]),
    ("vmqa_release_stream", ctypes.c_int, [_P, _P]),
    ("vmqs_release_stream", ctypes.c_int, [_P, _P]),
    ("vmqg_epoch", ctypes.c_int, [_P, ctypes.POINTER(_U64)]),
    ("vmqg_records_at", ctypes.c_int, [_P, _U64, ctypes.POINTER(_P), ctypes.POINTER(_U64)]),
    ("vmqg_records_pin", ctypes.c_int, [_P, _U64, ctypes.POINTER(_P), ctypes.POINTER(_U64), ctypes.POINTER(ctypes.c_uint32)]),
    ("vmqg_records_unpin", None, [_P, ctypes.c_uint32]),
    ("vmqg_replica_sync_layout", ctypes.c_int, [_P, _P]),
    ("vmqg_stats", ctypes.c_int, [_P, ctypes.POINTER(Stats)]),
    ("vmqg_dump", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_SZ)]),
    ("vmqg_set_option", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int64]),
    ("vmqg_set_timing", ctypes.c_int, [_P, ctypes.c_int]),
    ("vmqg_kernel_times", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
    ("vmqg_kernel_times_ex", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
    ("vmqg_arena", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_U64), _P]),
    ("vmqg_export_image", ctypes.c_int, [_P, _P, _U64]),
    ("vmqg_replica_load", ctypes.c_int, [_P, _P, _P, _P]),
    ("vmqg_last_patches", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_U64),
                                         ctypes.POINTER(ctypes.c_int)]),
    ("vmqg_apply_patches_device", ctypes.c_int, [_P, _P, _U64, _P]),
    # retained-message matcher (include/vmqr.h)
    ("vmqr_create", _P, [ctypes.POINTER(RConfig), ctypes.POINTER(ctypes.c_int)]),
    ("vmqr_destroy", None, [_P]),
    ("vmqr_intern_words", ctypes.c_int, [_P, _P, _P, _U32, ctypes.c_int, _P]),
    ("vmqr_apply", ctypes.c_int, [_P, _P, _SZ, _P, _SZ]),
    ("vmqr_match_batch", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, _P, _SZ, ctypes.POINTER(_SZ), _P]),
    ("vmqr_match_device", ctypes.c_int, [_P, _P, _U32, _P, _P, _U64, _P, _P]),
    ("vmqr_match_status", ctypes.c_int, [_P, _P]),
    ("vmqr_stats", ctypes.c_int, [_P, ctypes.POINTER(RStats)]),
    ("vmqr_dump", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_SZ)]),
    ("vmqr_set_option", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int64]),
    # ACL checker (include/vmqa.h)
    ("vmqa_create", _P, [ctypes.POINTER(AConfig), ctypes.POINTER(ctypes.c_int)]),
    ("vmqa_destroy", None, [_P]),
    ("vmqa_intern_words", ctypes.c_int, [_P, _P, _P, _U32, ctypes.c_int, _P]),
    ("vmqa_load", ctypes.c_int, [_P, _P, _SZ, _P, _SZ]),
    ("vmqa_check_batch", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, _P]),
    ("vmqa_check_device", ctypes.c_int, [_P, _P, _U32, _P, _P, _P]),
    ("vmqa_check_status", ctypes.c_int, [_P, _P]),
    ("vmqa_stats", ctypes.c_int, [_P, ctypes.POINTER(AStats)]),
    ("vmqa_set_timing", ctypes.c_int, [_P, ctypes.c_int]),
    ("vmqa_kernel_times", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
    # shared-subscription dispatcher (include/vmqs.h)
    ("vmqs_create", _P, [ctypes.POINTER(SConfig), ctypes.POINTER(ctypes.c_int)]),
    ("vmqs_destroy", None, [_P]),
    ("vmqs_set_states", ctypes.c_int, [_P, _P, _P, _SZ]),
    ("vmqs_select_batch", ctypes.c_int, [_P, _P, _P, _SZ, _U32, _U64, _U64, _P, _P]),
    ("vmqs_select_device", ctypes.c_int, [_P, _P, _P, _U32, _U32, _U64, _U64, _P, _P, _P]),
    ("vmqs_select_status", ctypes.c_int, [_P, _P]),
    ("vmqs_key", _U64, [_U64, _U64, _U32]),
    ("vmqs_set_timing", ctypes.c_int, [_P, ctypes.c_int]),
    ("vmqs_kernel_times", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64),
                                         ctypes.POINTER(_U64)]),
    ("vmqr_set_timing", ctypes.c_int, [_P, ctypes.c_int]),
    ("vmqr_kernel_times", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
]

_lib = None


FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-value", "-Wno-unused-result"]


def source_id() -> str:
    """Build id of the current sources: sha256 over every source and header
    the library is compiled from, plus the compile flags (16 hex digits).
    Embedded in the library (vmqg_build_id), recorded in every profile
    summary, and compared by bench.py before a PMC figure is reported."""
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for p in sorted(DEPS):
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    with open(LIB_PATH, "rb") as f:
        return ("vmqg-build:" + source_id()).encode() not in f.read()


def build_id() -> str:
    """Build id embedded in the loaded library."""
    return lib().vmqg_build_id().decode().split(":", 1)[-1]


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile libvmqgpu.so for gfx950 with hipcc (in-tree)."""
    if not force and not _stale():
        return LIB_PATH
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc] + FLAGS + ['-DVMQG_BUILD_ID="vmqg-build:%s"' % source_id(),
                             "-o", LIB_PATH + ".tmp"] + SOURCES
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n%s" % (r.stderr if not verbose else ""))
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


def _share_torch_hip_runtime():
    """PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7) and
    fails to initialise if the system runtime was loaded into the process
    first.  Loading torch's copy first makes our DT_NEEDED libamdhip64.so.7
    resolve to it, so the process has ONE HIP runtime and torch tensors,
    streams and RCCL buffers are shared with libvmqgpu."""
    try:
        import torch  # noqa: F401
    except Exception:   # no torch: the system runtime is used (e.g. an Erlang NIF host)
        pass


def lib():
    """Load libvmqgpu.so; raises ImportError when the native library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("VMQG_LIB_PATH", LIB_PATH)   # A/B runs of kernel variants (tools/)
    if not os.path.exists(path):
        raise ImportError("libvmqgpu.so not built (%s); run vernemq_amd._lib.build()" % path)
    _share_torch_hip_runtime()
    L = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        if path != LIB_PATH and not hasattr(L, name):
            continue   # an A/B build of an older revision (VMQG_LIB_PATH): the entry points it has
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != OK:
        raise VmqgError(rc, what)
