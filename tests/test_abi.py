"""CPU checks of the C ABI boundary (include/vmqg.h, vmqr.h, vmqa.h, vmqs.h): the library loads,
exports every declared entry point, its structs have the header's layout,
and a host-only context fails loudly on match calls (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from vernemq_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vmqg.h")
HEADERS = [HEADER] + [os.path.join(ROOT, "include", h) for h in ("vmqr.h", "vmqa.h", "vmqs.h")]


def declared_functions():
    out = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        out |= set(re.findall(r"^\s*[\w\s\*]+?\b(vmq[gras]_\w+)\s*\(", src, flags=re.M))
    return sorted(out)


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    decl = declared_functions()
    assert len(decl) >= 30
    missing = [f for f in decl if not hasattr(L, f)]
    assert not missing, missing
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(decl) == bound, set(decl) ^ bound
    assert L.vmqg_abi_version() == 7


def test_struct_layouts_match_header(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "vmqg.h"\n'
                    'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %u\\n", sizeof(vmqg_config),'
                    ' sizeof(vmqg_op), sizeof(vmqg_pub), sizeof(vmqg_emit), sizeof(vmqg_stats_t),'
                    ' offsetof(vmqg_config, hint_edges), offsetof(vmqg_op, subinfo), sizeof(vmqg_range),'
                    ' VMQG_MAX_NODES);return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(prog),
                    "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(_lib.Config), ctypes.sizeof(_lib.Op), ctypes.sizeof(_lib.Pub), ctypes.sizeof(_lib.Emit),
            ctypes.sizeof(_lib.Stats), _lib.Config.hint_edges.offset, _lib.Op.subinfo.offset,
            ctypes.sizeof(_lib.Range), _lib.MAX_NODES]
    assert got == want
    from vernemq_amd.reg_view import EMIT_DTYPE, OP_DTYPE, PUB_DTYPE, RANGE_DTYPE
    assert (OP_DTYPE.itemsize, PUB_DTYPE.itemsize, EMIT_DTYPE.itemsize, RANGE_DTYPE.itemsize) == \
        (got[1], got[2], got[3], got[7])


def test_acl_struct_layouts_match_header(tmp_path):
    prog = tmp_path / "sza.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "vmqa.h"\n'
                    'int main(void){printf("%zu %zu %zu %zu %zu\\n", sizeof(vmqa_config), sizeof(vmqa_rule),'
                    ' sizeof(vmqa_req), sizeof(vmqa_stats_t), offsetof(vmqa_req, nwords));return 0;}\n')
    exe = tmp_path / "sza"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(prog),
                    "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    from vernemq_amd.acl import REQ_DTYPE, RULE_DTYPE
    assert got == [ctypes.sizeof(_lib.AConfig), RULE_DTYPE.itemsize, REQ_DTYPE.itemsize, ctypes.sizeof(_lib.AStats),
                   REQ_DTYPE.fields["nwords"][1]]


def test_shared_struct_layouts_match_header(tmp_path):
    prog = tmp_path / "szs.c"
    prog.write_text('#include <stdio.h>\n#include "vmqs.h"\n'
                    'int main(void){printf("%zu %u %u %u\\n", sizeof(vmqs_config), VMQS_POLICY_LOCAL_ONLY,'
                    ' VMQS_DRAINING, VMQS_MAX_SEGMENT);return 0;}\n')
    exe = tmp_path / "szs"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(prog),
                    "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [ctypes.sizeof(_lib.SConfig), _lib.S_LOCAL_ONLY, _lib.S_DRAINING, _lib.S_MAX_SEGMENT]


def test_shared_key_matches_oracle():
    """vmqs_key (the element order of a shared group) is host-callable and
    equals the oracle's restatement of it bit for bit."""
    from oracle import shared_oracle as SO
    L = _lib.lib()
    for seed, q, p in [(0, 0, 0), (1, 2, 3), (0xDEADBEEF, 1 << 40, (1 << 24) - 1), (7, 12345, 4095)]:
        k = L.vmqs_key(seed, q, p)
        assert k == SO.sel_key(seed, q, p)
        assert k & 0xFFFFFF == p


def test_shared_context_needs_a_device():
    err = ctypes.c_int(0)
    cfg = _lib.SConfig(device=-1, local_node=0)
    assert _lib.lib().vmqs_create(ctypes.byref(cfg), ctypes.byref(err)) is None
    assert err.value == _lib.E_DEVICE


def test_acl_host_context_refuses_checks():
    """device = -1: tables only; a check fails loudly (no CPU fallback)."""
    cfg = _lib.AConfig()
    cfg.device = -1
    err = ctypes.c_int(0)
    L = _lib.lib()
    h = L.vmqa_create(ctypes.byref(cfg), ctypes.byref(err))
    assert h and err.value == 0
    req = np.zeros(6, dtype=np.uint32)
    req[0], req[5] = 2, 1
    words = np.zeros(1, dtype=np.uint32)
    out = np.zeros(1, dtype=np.uint8)
    assert L.vmqa_check_batch(h, req.ctypes.data, 1, words.ctypes.data, 1, out.ctypes.data) == _lib.E_DEVICE
    L.vmqa_destroy(h)


def test_retain_struct_layouts_match_header(tmp_path):
    prog = tmp_path / "szr.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "vmqr.h"\n'
                    'int main(void){printf("%zu %zu %zu %zu\\n", sizeof(vmqr_config), sizeof(vmqr_op),'
                    ' sizeof(vmqr_stats_t), offsetof(vmqr_op, msg));return 0;}\n')
    exe = tmp_path / "szr"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(prog),
                    "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [ctypes.sizeof(_lib.RConfig), ctypes.sizeof(_lib.ROp), ctypes.sizeof(_lib.RStats),
                   _lib.ROp.msg.offset]
    from vernemq_amd.retain import ROP_DTYPE
    assert ROP_DTYPE.itemsize == got[1]


def test_host_only_retain_context_refuses_to_match():
    from vernemq_amd.retain import RetainGpuSrv
    r = RetainGpuSrv(device=-1)
    r.insert("", (b"a",), "m")
    with pytest.raises(_lib.VmqgError) as ei:
        r.match_fold_batch([("", (b"#",))])
    assert ei.value.rc == _lib.E_DEVICE


def test_host_only_context_refuses_to_match():
    from vernemq_amd.reg_view import RegGpuView
    v = RegGpuView(device=-1)
    v.handle_event(("updated", ("", b"c"), None, [("nonode@nohost", True, [((b"a",), 0)])]))
    with pytest.raises(_lib.VmqgError) as ei:
        v.fold_batch([("", (b"a",))])
    assert ei.value.rc == _lib.E_DEVICE
    with pytest.raises(_lib.VmqgError) as ei:
        v.match_ranges(*v.prepare([("", (b"a",))]))
    assert ei.value.rc == _lib.E_DEVICE
    # the record table the ranges index is the host mirror
    recs = v.records()
    assert len(recs) > 0 and (recs["kind_node"] >> 24 == _lib.EMIT_LOCAL).sum() == 1


def test_create_rejects_bad_config():
    L = _lib.lib()
    cfg = _lib.Config()
    cfg.device = -1
    cfg.local_node = 70
    cfg.max_nodes = 64
    err = ctypes.c_int(0)
    assert not L.vmqg_create(ctypes.byref(cfg), ctypes.byref(err))
    assert err.value == _lib.E_LIMIT
    cfg.local_node, cfg.max_nodes = 0, _lib.MAX_NODES + 1
    assert not L.vmqg_create(ctypes.byref(cfg), ctypes.byref(err))
    assert err.value == _lib.E_LIMIT
    assert not L.vmqg_create(None, ctypes.byref(err))
    assert err.value == _lib.E_INVAL


def test_prepare_publish_follows_validate_topic():
    """vmqg_prepare_publish splits and rejects exactly like
    vmq_topic:validate_topic(publish, _) on the reference KATs."""
    from tests import scenarios as S
    from vernemq_amd.reg_view import RegGpuView
    v = RegGpuView(device=-1)
    v.intern_words([b"foo", b"baz"], create=True)
    L = _lib.lib()
    for c in S.load("topic_validation.json")["cases"]:
        if c["type"] != "publish":
            continue
        t = c["topic"].encode()
        words = np.zeros(64, dtype=np.uint32)
        pub = _lib.Pub()
        rc = L.vmqg_prepare_publish(v.handle, 0, t, len(t), words.ctypes.data, 64, ctypes.byref(pub))
        if "ok" in c:
            assert rc == 0 and pub.nwords == len(c["ok"]), c
            for i, w in enumerate(c["ok"]):
                want = v._words.get(w.encode(), _lib.WORD_UNKNOWN)
                assert words[i] == want, (c, i)
        else:
            assert rc == _lib.E_INVAL, c
    t = b"$SYS/x"
    assert L.vmqg_prepare_publish(v.handle, 0, t, len(t), words.ctypes.data, 64, ctypes.byref(pub)) == 0
    assert pub.flags == _lib.PUB_DOLLAR | _lib.PUB_UNKNOWN and pub.nwords == 2
    t = b"foo/baz"
    assert L.vmqg_prepare_publish(v.handle, 0, t, len(t), words.ctypes.data, 64, ctypes.byref(pub)) == 0
    assert pub.flags == 0


def test_batched_prepare_equals_the_single_form():
    """vmqg_prepare_publishes (the pipelined dictionary probes) gives, topic
    for topic, what vmqg_prepare_publish gives: same rejections, same words,
    same flags — on the validate_topic KATs, long words (> 16 bytes, verified
    beyond the slot's inline prefix), empty levels, many blocks."""
    from tests import scenarios as S
    from vernemq_amd.reg_view import PUB_DTYPE, RegGpuView
    v = RegGpuView(device=-1)
    known = [b"foo", b"baz", b"a" * 16, b"a" * 17, b"b" * 40, b"", b"w%d" % 7]
    v.intern_words(known + [b"x%d" % i for i in range(3000)], create=True)
    L = _lib.lib()
    topics = [c["topic"].encode() for c in S.load("topic_validation.json")["cases"] if c["type"] == "publish"]
    topics += [b"a" * 16 + b"/" + b"a" * 17, b"a" * 17 + b"/" + b"a" * 16 + b"x", b"b" * 40 + b"/b" * 3,
               b"b" * 39 + b"c", b"/foo//baz/", b"$SYS/foo", b"w7/+", b"#"]
    topics += [b"x%d/foo/y%d" % (i, i % 5) for i in range(700)]
    n = len(topics)
    ptrs = (ctypes.c_char_p * n)(*topics)
    lens = np.array([len(t) for t in topics], dtype=np.uint64)
    mps = np.arange(n, dtype=np.uint32) % 3
    pubs = np.zeros(n, dtype=PUB_DTYPE)
    rcs = np.zeros(n, dtype=np.int32)
    cap = int((lens + 1).sum())
    words = np.zeros(cap, dtype=np.uint32)
    nw = ctypes.c_size_t(0)
    assert L.vmqg_prepare_publishes(v.handle, n, mps.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data,
                                    pubs.ctypes.data, rcs.ctypes.data, words.ctypes.data, cap, ctypes.byref(nw)) == 0
    one = np.zeros(64, dtype=np.uint32)
    total = 0
    for i, t in enumerate(topics):
        pub = _lib.Pub()
        rc = L.vmqg_prepare_publish(v.handle, int(mps[i]), t, len(t), one.ctypes.data, 64, ctypes.byref(pub))
        assert rc == rcs[i], (t, rc, rcs[i])
        if rc:
            continue
        p = pubs[i]
        assert (p["mountpoint"], p["nwords"], p["flags"]) == (pub.mountpoint, pub.nwords, pub.flags), t
        assert list(words[p["word_off"]:p["word_off"] + p["nwords"]]) == list(one[:pub.nwords]), t
        total += pub.nwords
    assert total == nw.value
    # too small a word buffer is refused, not overrun
    assert L.vmqg_prepare_publishes(v.handle, n, mps.ctypes.data, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data,
                                    pubs.ctypes.data, rcs.ctypes.data, words.ctypes.data, 10, ctypes.byref(nw)) == \
        _lib.E_OVERFLOW
    g0 = L.vmqg_dict_generation(v.handle)
    v.intern_words([b"brand-new"], create=True)
    assert L.vmqg_dict_generation(v.handle) == g0 + 1


def test_intern_reserved_words():
    from vernemq_amd.reg_view import RegGpuView
    v = RegGpuView(device=-1)
    L = _lib.lib()
    blob = b"+#$sharefoo"
    offs = np.array([0, 1, 2, 8, 11], dtype=np.uint64)
    ids = np.zeros(4, dtype=np.uint32)
    assert L.vmqg_intern_words(v.handle, blob, offs.ctypes.data, 4, 0, ids.ctypes.data) == 0
    assert list(ids) == [_lib.WORD_PLUS, _lib.WORD_HASH, _lib.WORD_SHARE, _lib.WORD_UNKNOWN]
    assert L.vmqg_intern_words(v.handle, blob, offs.ctypes.data, 4, 1, ids.ctypes.data) == 0
    assert ids[3] == 3


def test_prepare_split_matches_a_plain_split():
    """The prepare's word split (8 bytes at a time) and word keys (16-byte
    loads that never cross into the next page past the topic) against a
    plain bytes.split(b"/") + dictionary lookup: random topics over an
    alphabet heavy in '/', '+', '#', NUL, 0x01 and 0x80+ bytes (the
    zero-byte trick's false-positive cases), every length 1..80, and each
    topic also placed so that it ends exactly at a page boundary."""
    import random
    from vernemq_amd.reg_view import RegGpuView
    v = RegGpuView(device=-1)
    r = random.Random(11)
    alphabet = [b"/", b"/", b"/", b"a", b"b", b"\x00", b"\x01", b"\x2e", b"\x30", b"\x80", b"\xff", b"+", b"#"]
    topics = []
    for n in range(1, 81):
        for _ in range(12):
            t = b"".join(r.choice(alphabet) for _ in range(n))
            if r.random() < 0.5:
                t = t.replace(b"+", b"c").replace(b"#", b"d")
            topics.append(t)
    words = sorted({w for t in topics for w in t.split(b"/")})
    v.intern_words(words[::2], create=True)   # half the words known
    L = _lib.lib()
    page = 4096
    buf = np.zeros(4 * page, dtype=np.uint8)
    base = (buf.ctypes.data + page - 1) // page * page
    out = np.zeros(128, dtype=np.uint32)
    for t in topics:
        want_rc = _lib.E_INVAL if (b"+" in t or b"#" in t) else 0
        parts = t.split(b"/")
        want = v.intern_words(parts, create=False) if not want_rc else None
        for where in ("heap", "page_end"):
            if where == "heap":
                ptr = ctypes.c_char_p(t)
            else:
                at = base + page - len(t)   # the topic's last byte is the page's last
                ctypes.memmove(at, t, len(t))
                ptr = ctypes.cast(ctypes.c_void_p(at), ctypes.c_char_p)
            pub = _lib.Pub()
            rc = L.vmqg_prepare_publish(v.handle, 0, ptr, len(t), out.ctypes.data, 128, ctypes.byref(pub))
            assert rc == want_rc, (t, where, rc)
            if rc:
                continue
            assert pub.nwords == len(parts), (t, where)
            assert list(out[:pub.nwords]) == list(want), (t, where)
            assert bool(pub.flags & _lib.PUB_DOLLAR) == t.startswith(b"$")
