"""Shared-subscription dispatch (vmq_shared_subscriptions:publish/3,
include/vmqs.h).

CPU: the two oracle restatements agree; the reference's dispatch tests
(tests/golden/shared_dispatch.json) hold on the oracle pipeline (trie fold ->
dispatch); the element keys give the reference's distribution (uniform over
collected entries, so proportional to the Q2 multiplicity).
GPU (marked): the HIP dispatcher against the oracle, byte for byte, on the
fixtures end to end (match + dispatch on the device), random record batches
covering both tiers and the limits, and the config-D match output.
"""
import ctypes
import random
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from oracle import shared_oracle as SO
from tests import scenarios as S

SCEN = S.load("shared_dispatch.json")["scenarios"]
STATE_CODE = {"not_found": 0, "online": 1, "offline": 2, "draining": 3}


def _words(t: str):
    return tuple(w.encode() for w in t.split("/"))


def _events(sc):
    evs = []
    for client, node, filt, qos in sc["subs"]:
        evs.append(("updated", ("", client.encode()), None, [(node, True, [(_words(filt), qos)])]))
    return evs


class Ids:
    def __init__(self, first=()):
        self.m = {}
        for t in first:
            self.get(t)

    def get(self, t):
        return self.m.setdefault(t, len(self.m))


def oracle_records(sc, n_pub):
    """Fold the scenario's publishes on the trie oracle and encode the
    emissions as vmqg_emit records (node() = id 0)."""
    orc = O.TrieOracle(sc["node"])
    orc.apply(_events(sc))
    folds = orc.fold_batch([("", sc["publisher"].encode(), _words(sc["topic"]))] * n_pub)
    nodes, groups, subs = Ids([sc["node"]]), Ids(), Ids()
    recs, offs = [], [0]
    for f in folds:
        for e in f:
            if e[0] == "B":
                recs.append((2 << 24 | nodes.get(e[1]), groups.get(e[2]), subs.get(e[3][1].decode()), 0))
            elif e[0] == "A":
                recs.append((1 << 24, 0xFFFFFFFF, subs.get(e[1][1].decode()), 0))
            else:
                recs.append((3 << 24 | nodes.get(e[1]), 0xFFFFFFFF, 0, 0))
        offs.append(len(recs))
    states = np.ones(max(len(subs.m), 1), dtype=np.uint8)
    for c, st in sc["states"].items():
        if c in subs.m:
            states[subs.m[c]] = STATE_CODE[st]
    return np.array(recs, dtype=np.uint32).reshape(-1, 4), np.array(offs, dtype=np.uint64), states, groups, subs


def check_expectation(sc, per_pub):
    """per_pub: list of {group bytes: chosen client str | None}."""
    for i, got in enumerate(per_pub):
        assert set(got) == {g.encode() for g in sc["expect"]}, (sc["name"], i, got)
        for g, allowed in sc["expect"].items():
            c = got[g.encode()]
            if allowed is None:
                assert c is None, (sc["name"], i, g, c)
            else:
                assert c in allowed, (sc["name"], i, g, c)


def _decode_choice(recs, offs, chosen, groups, subs):
    gname = {v: k for k, v in groups.m.items()}
    sname = {v: k for k, v in subs.m.items()}
    out = []
    for i in range(len(offs) - 1):
        d = {}
        for j in range(int(offs[i]), int(offs[i + 1])):
            if recs[j][0] >> 24 == 2:
                g = gname[int(recs[j][1])]
                d.setdefault(g, None)
                if chosen[j]:
                    assert d[g] is None, "two receivers for one group"
                    d[g] = sname[int(recs[j][2])]
        out.append(d)
    return out


# ---------------------------------------------------------------- CPU
@pytest.mark.parametrize("sc", SCEN, ids=[s["name"] for s in SCEN])
def test_golden_dispatch_on_oracle(sc):
    recs, offs, states, groups, subs = oracle_records(sc, sc["n_publishes"])
    for seed in (0, 1, 0xC0FFEE):
        chosen, failed = SO.select(recs, offs, sc["policy"], seed, 0, states, 0)
        per_pub = _decode_choice(recs, offs, chosen, groups, subs)
        check_expectation(sc, per_pub)
        assert list(failed) == [sum(1 for v in d.values() if v is None) for d in per_pub]


def _random_batch(r: random.Random, npub, max_seg=40, n_groups=4, n_nodes=3, n_subs=20):
    recs, offs = [], [0]
    for _ in range(npub):
        for _ in range(r.randint(0, max_seg)):
            k = r.choice((1, 2, 2, 2, 3))
            recs.append((k << 24 | r.randrange(n_nodes), r.randrange(n_groups) if k == 2 else 0xFFFFFFFF,
                         r.randrange(n_subs), r.randrange(5)))
        offs.append(len(recs))
    return (np.array(recs, dtype=np.uint32).reshape(-1, 4), np.array(offs, dtype=np.uint64))


def test_python_and_cpp_restatements_agree():
    r = random.Random(7)
    for t in range(120):
        recs, offs = _random_batch(r, r.randint(1, 6))
        st = np.array([r.randrange(4) for _ in range(15)], dtype=np.uint8)   # ids >= 15: online
        pol = ("random", "prefer_local", "local_only")[t % 3]
        seed = r.getrandbits(64)
        chosen, failed = SO.select(recs, offs, pol, seed, 1000, st, 0)
        for i in range(len(offs) - 1):
            seg = [(int(x[0]) >> 24, int(x[0]) & 0xFFFFFF, int(x[1]), int(x[2]), int(x[3]))
                   for x in recs[int(offs[i]):int(offs[i + 1])]]
            c2, f2 = SO.dispatch(seg, pol, 0, st, seed, 1000 + i)
            assert list(chosen[int(offs[i]):int(offs[i + 1])]) == c2 and failed[i] == f2


def test_key_distribution_is_the_references():
    """rand:uniform() per entry (:27-28): every collected entry equally likely
    to come first, so a member emitted k times (Q2) wins k times as often."""
    # members a (x1), b (x2), c (x3) of one group, all online
    seg = [(2, 0, 0, s, 0) for s in (0, 1, 1, 2, 2, 2)]
    wins = np.zeros(3)
    n = 30000
    for q in range(n):
        c, _ = SO.dispatch(seg, "random", 0, np.ones(3, np.uint8), 0x5EED, q)
        wins[seg[c.index(1)][3]] += 1
    expect = np.array([1, 2, 3]) / 6 * n
    chi2 = float(((wins - expect) ** 2 / expect).sum())
    assert chi2 < 13.8, (wins, chi2)   # p = 0.001 at 2 dof
    # publish_any picks uniformly among offline entries too (reverse order of a uniform order)
    st = np.full(3, 2, np.uint8)
    wins[:] = 0
    for q in range(n):
        c, _ = SO.dispatch(seg, "random", 0, st, 0xF00, q)
        wins[seg[c.index(1)][3]] += 1
    chi2 = float(((wins - expect) ** 2 / expect).sum())
    assert chi2 < 13.8, (wins, chi2)


def test_policies_filter_as_reference():
    # group g: local (node 0) member 0 offline, remote members 1, 2 online
    seg = [(2, 0, 7, 0, 0), (2, 1, 7, 1, 0), (2, 2, 7, 2, 0)]
    st = np.array([2, 1, 1], np.uint8)
    for q in range(50):
        c, f = SO.dispatch(seg, "prefer_local", 0, st, 1, q)
        assert c == [1, 0, 0] and f == 0        # the local member, via publish_any
        c, f = SO.dispatch(seg, "local_only", 0, st, 1, q)
        assert c == [1, 0, 0] and f == 0
        c, f = SO.dispatch(seg, "random", 0, st, 1, q)
        assert c[0] == 0 and sum(c) == 1        # an online member first
    seg_remote = seg[1:]
    c, f = SO.dispatch(seg_remote, "local_only", 0, st, 1, 0)
    assert c == [0, 0] and f == 1
    c, f = SO.dispatch(seg_remote, "prefer_local", 0, st, 1, 0)
    assert sum(c) == 1 and f == 0


# ---------------------------------------------------------------- GPU
def _gpu_select(sel, recs, offs, policy, seed, pub_seq):
    from vernemq_amd.reg_view import EMIT_DTYPE
    e = np.ascontiguousarray(recs, dtype=np.uint32).view(EMIT_DTYPE).reshape(-1)
    return sel.select_batch(e, offs, policy, seed, pub_seq)


@pytest.fixture(scope="module")
def sel():
    from vernemq_amd.shared import SharedGpu
    s = SharedGpu(device=0, local_node=0)
    yield s
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sc", SCEN, ids=[s["name"] for s in SCEN])
def test_golden_dispatch_end_to_end_on_gpu(sc):
    """Subscriptions into the GPU matcher, publishes matched and dispatched
    on the device (SharedGpu.route_batch = vmq_reg:publish/5)."""
    from vernemq_amd.reg_view import RegGpuView
    from vernemq_amd.shared import SharedGpu
    view = RegGpuView(node=sc["node"], device=0, nodes=sc["nodes"])
    view.handle_events(_events(sc))
    s = SharedGpu(device=0, local_node=0)
    s.set_states(view, {("", c.encode()): st for c, st in sc["states"].items()})
    pubs = [(("", sc["publisher"].encode()), _words(sc["topic"]))] * sc["n_publishes"]
    for seed in (0, 1, 0xC0FFEE):
        routes = s.route_batch(view, pubs, sc["policy"], seed)
        per_pub = [{g: (None if c is None else c[1][1].decode()) for g, c in d["shared"].items()} for d in routes]
        check_expectation(sc, per_pub)
    s.close()
    view.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sc", SCEN, ids=[s["name"] for s in SCEN])
def test_golden_records_bit_exact_on_gpu(sel, sc):
    recs, offs, states, _g, _s = oracle_records(sc, sc["n_publishes"])
    _all_online(sel)
    sel.set_state_ids(np.arange(len(states)), states)
    for seed in (0, 99):
        want = SO.select(recs, offs, sc["policy"], seed, 5, states, 0)
        got = _gpu_select(sel, recs, offs, sc["policy"], seed, 5)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["small", "long_segments", "many_groups", "ragged"])
def test_random_batches_bit_exact(sel, shape):
    r = random.Random(zlib.crc32(shape.encode()))   # reproducible across processes
    kw = {"small": dict(max_seg=40, n_groups=4),
          "long_segments": dict(max_seg=9000, n_groups=6),        # > kWaveMax: tier 2
          "many_groups": dict(max_seg=600, n_groups=300),         # > 64 groups: tier 2
          "ragged": dict(max_seg=5000, n_groups=80, n_nodes=5, n_subs=3000)}[shape]
    npub = {"small": 3000, "long_segments": 60, "many_groups": 200, "ragged": 300}[shape]
    recs, offs = _random_batch(r, npub, **kw)
    _all_online(sel)
    st = np.array([r.randrange(4) for _ in range(kw.get("n_subs", 20) - 3)], np.uint8)
    sel.set_state_ids(np.arange(len(st)), st)
    full = np.ones(kw.get("n_subs", 20), np.uint8)
    full[:len(st)] = st
    for pol in ("random", "prefer_local", "local_only"):
        seed = r.getrandbits(64)
        want = SO.select(recs, offs, pol, seed, 77, full, 0)
        got = _gpu_select(sel, recs, offs, pol, seed, 77)
        assert np.array_equal(got[1], want[1]), pol
        assert np.array_equal(got[0], want[0]), pol


def _all_online(sel, n=4096):
    sel.set_state_ids(np.arange(n), np.ones(n, np.uint8))


@pytest.mark.gpu
def test_offsets_not_starting_at_zero_and_empty(sel):
    _all_online(sel)
    r = random.Random(3)
    recs, offs = _random_batch(r, 50)
    sub = offs[10:31]   # publishes 10..29 only; records outside are untouched
    want = SO.select(recs, offs, "random", 5, 0, np.ones(20, np.uint8), 0)
    got_c, got_f = _gpu_select(sel, recs, sub, "random", 5, 10)
    assert np.array_equal(got_c[int(sub[0]):], want[0][int(sub[0]):int(sub[-1])])
    assert np.array_equal(got_f, want[1][10:30])
    c, f = _gpu_select(sel, recs[:0], np.zeros(5, np.uint64), "random", 1, 0)   # 4 empty publishes
    assert len(c) == 0 and list(f) == [0, 0, 0, 0]


@pytest.mark.gpu
def test_group_table_limit_is_loud(sel):
    from vernemq_amd import _lib
    _all_online(sel)
    # one publish with 3000 distinct groups > the tier-2 table: VMQG_E_LIMIT, not a wrong answer
    recs = np.array([(2 << 24, g, g, 0) for g in range(3000)], dtype=np.uint32)
    offs = np.array([0, 3000], dtype=np.uint64)
    with pytest.raises(_lib.VmqgError) as ei:
        _gpu_select(sel, recs, offs, "random", 1, 0)
    assert ei.value.rc == _lib.E_LIMIT
    # the context stays usable
    c, f = _gpu_select(sel, recs[:100], np.array([0, 100], np.uint64), "random", 1, 0)
    assert c.sum() == 100 and f[0] == 0


@pytest.mark.gpu
def test_config_d_match_output_dispatch():
    """Config D (scaled): the GPU's own match output (Q2: each member 4x)
    dispatched on the device, against the oracle on the same records."""
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    from vernemq_amd.shared import SharedGpu
    w = W.config_d(scale=0.01, n_pubs=1 << 14)
    view = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(view)
    arr, words = w.publish_arrays(view)
    recs, offs = view.match_arrays(arr, words)
    s = SharedGpu(device=0, local_node=0)
    n_sub = int(max(recs["subscriber"].max(), 1)) + 1
    st = np.array([(i * 7) % 4 for i in range(n_sub)], np.uint8)
    s.set_state_ids(np.arange(n_sub), st)
    raw = recs.view(np.uint32).reshape(-1, 4)
    assert (raw[:, 0] >> 24 == 2).sum() > 0
    for pol in ("random", "prefer_local", "local_only"):
        want = SO.select(raw, offs, pol, 0xD, 0, st, 0)
        got = s.select_batch(recs, offs, pol, 0xD, 0)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), pol
    s.close()
    view.close()


@pytest.mark.gpu
def test_device_entry_point_with_torch_buffers():
    import torch
    from vernemq_amd.shared import SharedGpu
    r = random.Random(11)
    recs, offs = _random_batch(r, 500, max_seg=100, n_groups=8)
    s = SharedGpu(device=0, local_node=0)
    d_r = torch.from_numpy(recs.astype(np.int32)).cuda()
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_c = torch.full((len(recs),), 7, dtype=torch.uint8, device="cuda")
    d_f = torch.zeros(500, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    s.select_device(d_r.data_ptr(), d_o.data_ptr(), 500, "prefer_local", 42, 9, d_c.data_ptr(), d_f.data_ptr(),
                    stream)
    assert s.select_status(stream) == 0
    want = SO.select(recs, offs, "prefer_local", 42, 9, np.ones(20, np.uint8), 0)
    assert np.array_equal(d_c.cpu().numpy(), want[0])
    assert np.array_equal(d_f.cpu().numpy().astype(np.uint32), want[1])
    s.close()


@pytest.mark.gpu
def test_single_group_chunks_bit_exact(sel):
    """Runs of >= 64 records of one group inside one tier-1 segment take the
    wave-wide group reduction (vmqs_kernels.hip); mixed chunks take the
    per-lane path.  One group spans both kinds of chunk; members are local
    and remote, online, offline, draining and without a queue; every policy
    against the restatement."""
    r = random.Random(64)
    n_subs = 500
    st = np.array([r.choice([0, 1, 1, 1, 2, 3]) for _ in range(n_subs)], np.uint8)
    sel.set_state_ids(np.arange(n_subs), st)
    recs, offs = [], [0]

    def member(g):
        node = r.choice([0, 0, 1, 2])
        return (2 << 24 | node, g, r.randrange(n_subs), r.randrange(3))

    for p in range(40):
        seg = [member(7) for _ in range(64 + 64 * (p % 3))]                 # whole single-group chunks
        seg += [member(r.choice([7, 8, 9])) for _ in range(48 + p)]         # group 7 again, in mixed chunks
        seg += [member(8) for _ in range(130)]                              # another group's run
        if p % 5 == 0:
            seg += [(1 << 24, 0xFFFFFFFF, r.randrange(n_subs), 0), (3 << 24 | 2, 0xFFFFFFFF, 0, 0)]
        recs += seg
        offs.append(len(recs))
    recs = np.array(recs, dtype=np.uint32).reshape(-1, 4)
    offs = np.array(offs, dtype=np.uint64)
    for pol in ("random", "prefer_local", "local_only"):
        for seed in (1, 2):
            want = SO.select(recs, offs, pol, seed, 3, st, 0)
            got = _gpu_select(sel, recs, offs, pol, seed, 3)
            assert np.array_equal(got[1], want[1]), (pol, seed)
            assert np.array_equal(got[0], want[0]), (pol, seed)
