"""GPU parity of the pipelined match (vmqg_match_submit / _submit_ranges /
vmqg_match_flush, include/vmqg.h): batch k's COUNT runs in the same launches
as batch k-1's EMIT, so every batch's output must equal, byte for byte, what
the unpipelined vmqg_match_batch / vmqg_match_ranges writes for it (itself
checked against the oracle by tests/test_gpu_parity.py) — across batch sizes,
deferred publishes, table changes between submits, stream and mode changes,
and latched errors."""
import itertools

import numpy as np
import pytest

from oracle import oracle as O
from tests import harness as H

pytestmark = pytest.mark.gpu

MODES = ["records", "ranges"]


def _torch():
    import torch
    return torch, torch.device("cuda:0")


class Batch:
    """Device buffers of one submitted batch (kept alive until flushed)."""

    def __init__(self, v, pubs, words, mode, cap):
        torch, dev = _torch()
        self.n = len(pubs)
        self.mode = mode
        self.d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
        self.d_words = torch.from_numpy(np.asarray(words).astype(np.int32).reshape(-1) if len(words)
                                        else np.zeros(1, np.int32)).to(dev)
        esz = 4 if mode == "records" else 2
        self.cap = cap
        self.d_out = torch.full((max(cap, 1) * esz,), -1, dtype=torch.int32, device=dev)
        self.d_offs = torch.full((self.n + 1,), -1, dtype=torch.int64, device=dev)

    def submit(self, v, stream):
        f = v.match_submit if self.mode == "records" else v.match_submit_ranges
        f(self.d_pubs.data_ptr(), self.n, self.d_words.data_ptr(), self.d_out.data_ptr(), self.cap,
          self.d_offs.data_ptr(), stream)

    def result(self):
        offs = self.d_offs.cpu().numpy().astype(np.uint64)
        w = 4 if self.mode == "records" else 2
        out = self.d_out.cpu().numpy().view(np.uint32).reshape(-1, w)[: int(offs[-1])]
        return offs, out


def _reference(v, pubs, words, mode):
    """The unpipelined host-buffer path's bytes for the same batch."""
    if mode == "records":
        recs, offs = v.match_arrays(pubs, words)
        return np.asarray(offs, dtype=np.uint64), np.asarray(recs).view(np.uint32).reshape(-1, 4)
    rng, offs = v.match_ranges(pubs, words)
    return np.asarray(offs, dtype=np.uint64), np.asarray(rng).view(np.uint32).reshape(-1, 2)


def _check(b, ref, ctx):
    offs, out = b.result()
    assert np.array_equal(offs, ref[0]), "%s: offsets differ" % ctx
    assert np.array_equal(out, ref[1]), "%s: entries differ" % ctx


def _hot_workload(node="n@h"):
    """n/{j} topics matched by one filter each, plus h/x/y/z matched by 31
    filters (more keys than the fast tier's lists: the wave tier walks it)."""
    prod = H.ProductDriver(node, device=0)
    evs = []
    hot = (b"h", b"x", b"y", b"z")
    filters = set()
    for combo in itertools.product([0, 1], repeat=4):
        t = tuple(b"+" if c else hot[i] for i, c in enumerate(combo))
        filters.add(t)
        for k in range(4):
            filters.add(t[:k] + (b"#",))
    for i, t in enumerate(sorted(filters)):
        evs.append(("updated", ("", b"f%d" % i), None, [(node, True, [(t, i % 3)])]))
    for j in range(0, 1000, 2):
        evs.append(("updated", ("", b"n%d" % j), None, [(node, True, [((b"n", b"%d" % j), 1)])]))
    # a fan-out key and a remote node, as in config C
    for k in range(40):
        evs.append(("updated", ("", b"w%d" % k), None, [(node, True, [((b"n", b"+"), 0)])]))
    evs.append(("updated", ("", b"r"), None, [("m@h", True, [((b"n", b"#"), 0)])]))
    prod.apply(evs)
    topics = [("", (b"n", b"%d" % j)) for j in range(1000)] + [("", hot), ("", (b"q",))]
    return prod, evs, topics


@pytest.mark.parametrize("mode", MODES)
def test_pipelined_batches_equal_unpipelined(mode):
    """Five batches of different sizes (incl. 1 publish and deferral-heavy
    ones) submitted back to back on torch's stream, one flush."""
    torch, dev = _torch()
    prod, _, topics = _hot_workload()
    v = prod.view
    arr, words = v.prepare(topics)
    rng = np.random.default_rng(5)
    sizes = [4096, 1, 37, 70_000, 4096]
    batches, refs = [], []
    for k, n in enumerate(sizes):
        idx = rng.integers(0, len(topics), n)
        if k == 3:
            idx[::23] = 1000      # h/x/y/z: deferred to the wave tier all over the batch
        ref = _reference(v, arr[idx], words, mode)
        refs.append(ref)
        batches.append(Batch(v, arr[idx], words, mode, int(ref[0][-1]) + 8))
    s = torch.cuda.current_stream().cuda_stream
    for b in batches:
        b.submit(v, s)
    v.match_flush()
    assert v.match_status(s) == 0
    for k, (b, ref) in enumerate(zip(batches, refs)):
        _check(b, ref, "batch %d (%d publishes)" % (k, sizes[k]))
    assert int(refs[3][0][-1]) > 70_000


def test_pipeline_is_ordered_against_table_changes():
    """A table change between two submits lands after the pending batch's
    EMIT: batch A sees the tables before it, batch B after."""
    torch, dev = _torch()
    node = "n@h"
    prod, evs, topics = _hot_workload(node)
    v = prod.view
    orc = O.TrieOracle(node)
    orc.apply(evs)
    arr, words = v.prepare(topics)
    idx = np.arange(len(topics)).repeat(3)
    ref_a = _reference(v, arr[idx], words, "records")
    s = torch.cuda.current_stream().cuda_stream
    a = Batch(v, arr[idx], words, "records", int(ref_a[0][-1]) + 8)
    a.submit(v, s)
    # delete half the filters and the fan-out key (moves / frees records)
    dels = [("deleted", e[1], e[3]) for e in evs[::2]] + [("deleted", e[1], e[3]) for e in evs if e[1][1][:1] == b"w"]
    prod.apply(dels)
    orc.apply(dels)
    ref_b = _reference(v, arr[idx], words, "records")
    b = Batch(v, arr[idx], words, "records", int(ref_b[0][-1]) + 8)
    b.submit(v, s)
    v.match_flush()
    assert v.match_status(s) == 0
    _check(a, ref_a, "batch before the deletes")
    _check(b, ref_b, "batch after the deletes")
    assert int(ref_b[0][-1]) < int(ref_a[0][-1])
    # and the post-delete reference is the oracle's
    want = orc.fold_batch([(mp, b"pub", t) for mp, t in topics])
    offs, out = b.result()
    for i in range(len(topics)):
        j = 3 * i
        got = sorted(H.canon(v.decode({"kind_node": r[0], "group": r[1], "subscriber": r[2], "subinfo": r[3]}))
                     for r in out[int(offs[j]): int(offs[j + 1])])
        assert got == sorted(want[i]), topics[i]


def test_pipeline_stream_and_mode_changes():
    """Records, then ranges, then records on another stream, then the NULL
    stream: each change flushes the pending batch; all outputs exact."""
    torch, dev = _torch()
    prod, _, topics = _hot_workload()
    v = prod.view
    arr, words = v.prepare(topics)
    rng = np.random.default_rng(9)
    plan = [("records", "cur"), ("ranges", "cur"), ("ranges", "cur"), ("records", "side"), ("records", "side"),
            ("records", "null"), ("ranges", "null")]
    side = torch.cuda.Stream()
    batches, refs = [], []
    for mode, _ in plan:
        idx = rng.integers(0, len(topics), 3000)
        ref = _reference(v, arr[idx], words, mode)
        refs.append(ref)
        batches.append(Batch(v, arr[idx], words, mode, int(ref[0][-1]) + 8))
    torch.cuda.synchronize()
    for (mode, where), b in zip(plan, batches):
        if where == "side":
            with torch.cuda.stream(side):
                b.submit(v, side.cuda_stream)
        elif where == "null":
            b.submit(v, 0)
        else:
            b.submit(v, torch.cuda.current_stream().cuda_stream)
    assert v.match_status(0) == 0          # flushes the last batch (NULL stream)
    torch.cuda.synchronize()
    for k, (b, ref) in enumerate(zip(batches, refs)):
        _check(b, ref, "batch %d %r" % (k, plan[k]))


def test_pipeline_errors_are_latched():
    """An overflowing batch in a pipeline is reported by the status after a
    later clean one; the clean one's output is exact."""
    torch, dev = _torch()
    prod = H.ProductDriver("n@h", device=0)
    v = prod.view
    v.handle_events([("updated", ("", b"c%d" % i), None, [("n@h", True, [((b"t",), 0)])]) for i in range(100)])
    pubs, words = v.prepare([("", (b"t",))] * 4)
    ref = _reference(v, pubs, words, "records")
    s = torch.cuda.current_stream().cuda_stream
    bad = Batch(v, pubs, words, "records", 10)
    good = Batch(v, pubs, words, "records", 400)
    bad.submit(v, s)
    good.submit(v, s)
    from vernemq_amd import _lib
    assert v.match_status(s) == _lib.E_OVERFLOW
    _check(good, ref, "clean batch after an overflow")
    good.submit(v, s)
    assert v.match_status(s) == 0


def test_pipelined_config_c_counts():
    """Config C shape (100k devices, 2^18 publishes per batch) through four
    pipelined submits with alternating publish sets: every publish's count is
    the known answer and the records equal the unpipelined ones."""
    torch, dev = _torch()
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    w = W.config_c(n_dev=100_000, n_pubs=1 << 18, seed=3)
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    d_idx = w.pw[1::4] - 18
    want = np.where(d_idx < 100_000, w.notes["n_wild"] + 1, w.notes["n_wild"])
    ref = _reference(v, pubs, words, "records")
    assert np.array_equal(np.diff(ref[0].astype(np.int64)), want)
    rev = np.arange(len(pubs))[::-1].copy()
    ref_r = _reference(v, pubs[rev], words, "records")
    batches = [Batch(v, pubs if k % 2 == 0 else pubs[rev], words, "records", int(ref[0][-1]) + 8) for k in range(4)]
    s = torch.cuda.current_stream().cuda_stream
    v.set_timing(True)
    for b in batches:
        b.submit(v, s)
    assert v.match_status(s) == 0
    mixed_ns, nmixed, count_ns, emit_ns = v.pipeline_times()
    v.set_timing(False)
    assert nmixed == 3 and mixed_ns > 0 and count_ns > 0 and emit_ns > 0
    for k, b in enumerate(batches):
        _check(b, ref if k % 2 == 0 else ref_r, "config C batch %d" % k)
