"""The pure-C half of the vmq_reg_gpu_view NIF (integration/c_src/vmqg_batch.c):
compiled with gcc against include/vmqg.h and libvmqgpu.so, and run over a
host-engine-only context (no GPU): interners, subscription ops from filter
strings, publish batches (vmq_topic:validate_topic splitting, rejection,
growth, merging per-thread batches), the fold over records and over ranges,
and the loud refusal to match without a device."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_batch_layer_unit(tmp_path):
    from vernemq_amd import _lib
    lib_dir = os.path.dirname(_lib.LIB_PATH)
    exe = tmp_path / "test_batch"
    subprocess.run(["gcc", "-std=c99", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "integration", "c_src"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "c", "test_batch.c"),
                    os.path.join(ROOT, "integration", "c_src", "vmqg_batch.c"),
                    "-L", lib_dir, "-l:libvmqgpu.so", "-Wl,-rpath," + lib_dir], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


def test_nif_sources_are_present():
    """The Erlang drop-in and its NIF glue ship as files (OTP is not in this
    image: they are not compiled here; their C core above is)."""
    erl = open(os.path.join(ROOT, "integration", "src", "vmq_reg_gpu_view.erl")).read()
    nif = open(os.path.join(ROOT, "integration", "c_src", "vmqg_nif.c")).read()
    for needle in ("-behaviour(vmq_reg_view)", "fold(", "start_link()", "stats()", "subscribe_subscriber_changes",
                   "drain_events", "vmqg_nif:apply_many"):
        assert needle in erl, needle
    for needle in ("ERL_NIF_INIT", "vmqgb_view_match", "vmqgb_view_release", "vmqgb_fold", "vmqgb_view_apply_ops",
                   "vmqgb_batch_add_many", "nif_apply_many", "ERL_NIF_DIRTY_JOB_CPU_BOUND"):
        assert needle in nif, needle


def _nif_script(seed=11, n_subs=3000, n_pubs=2500):
    """A subscription set (wildcards, $share groups on several nodes, remote
    nodes incl. one >= 64, $-topics), publishes, and the script that drives
    tools/bin/batch_gpu_check through it; plus the same changes as
    subscriber-store events for the oracle."""
    import random
    r = random.Random(seed)
    nodes = ["n0@h"] + ["n%d@h" % k for k in range(1, 6)] + ["n70@h"]
    node_ids = list(range(6)) + [70]
    words = [b"a", b"b", b"c", b"d"]

    def rand_filter():
        pre = (b"$share", r.choice([b"g1", b"g2", b"g3"])) if r.random() < 0.2 else ()
        L = r.randint(1, 4)
        t = [b"+" if r.random() < 0.25 else (b"#" if (i == L - 1 and r.random() < 0.15) else r.choice(words))
             for i in range(L)]
        if r.random() < 0.05:
            t[0] = b"$SYS"
        return pre + tuple(t)

    subs = []
    for k in range(n_subs):
        ni = r.choice(range(len(nodes))) if r.random() < 0.3 else 0
        subs.append((ni, k, r.randint(0, 2), rand_filter()))
    pubs = []
    for _ in range(n_pubs):
        L = r.randint(1, 5)
        t = [r.choice(words) for _ in range(L)]
        if r.random() < 0.05:
            t[0] = b"$SYS"
        pubs.append(tuple(t))
    lines = []
    line = lambda c, s: "%s %d %d %d 0 %s" % (c, node_ids[s[0]], s[1], s[2], b"/".join(s[3]).decode())
    lines += [line("S", s) for s in subs] + ["A"]
    lines += ["P 0 %s" % b"/".join(t).decode() for t in pubs]
    lines += ["M records 8 64", "M ranges 4 100"]
    gone = subs[::3]
    lines += [line("U", s) for s in gone] + ["A"]
    lines += ["M records 16 37", "C ranges 8 50 300"]
    sid = lambda k: ("", b"c%d" % k)
    ev_add = [("updated", sid(k), None, [(nodes[ni], True, [(f, q)])]) for ni, k, q, f in subs]
    ev_del = [("deleted", sid(k), [(nodes[ni], True, [(f, q)])]) for ni, k, q, f in gone]
    return "\n".join(lines) + "\n", nodes, node_ids, pubs, ev_add, ev_del


def _parse_blocks(text, nodes, node_ids):
    from oracle import oracle as O
    name = {nid: nodes[i] for i, nid in enumerate(node_ids)}
    blocks, cur = [], None
    for ln in text.splitlines():
        if ln.startswith("M "):
            cur = []
            blocks.append(cur)
            continue
        f = ln.split(" ")
        rc = int(f[1])
        ents = []
        for e in f[2:]:
            kind, node, group, sub, info = e.split(",")
            kind, node, sub, info = int(kind), int(node), int(sub), int(info)
            if kind == 1:
                ents.append(("A", ("", b"c%d" % sub), O.subinfo_repr(info)))
            elif kind == 2:
                ents.append(("B", name[node], group.encode(), ("", b"c%d" % sub), O.subinfo_repr(info)))
            else:
                ents.append(("C", name[node]))
        cur.append((rc, sorted(ents)))
    return blocks


@pytest.mark.gpu
def test_batch_layer_on_the_gpu_with_concurrent_batchers(tmp_path):
    """vmqg_batch.c on the device, driven as vmqg_nif.c drives it: 4-16
    batcher threads with their own batches under the view's locks (records
    and ranges, overflow retries, the fold), then after deletes, and once
    more while a writer applies changes between batches — every publish's
    entries equal the oracle's."""
    import subprocess
    from oracle import oracle as O
    exe = os.path.join(ROOT, "tools", "bin", "batch_gpu_check")
    assert os.path.exists(exe), "tools/bin/batch_gpu_check not built (__graft_entry__.build())"
    script, nodes, node_ids, pubs, ev_add, ev_del = _nif_script()
    (tmp_path / "s.txt").write_text(script)
    r = subprocess.run([exe, str(tmp_path / "s.txt"), str(tmp_path / "o.txt")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    blocks = _parse_blocks((tmp_path / "o.txt").read_text(), nodes, node_ids)
    assert len(blocks) == 4 and all(len(b) == len(pubs) for b in blocks)
    orc = O.TrieOracle(nodes[0])
    orc.apply(ev_add)
    want1 = [sorted(x) for x in orc.fold_batch([("", b"pub", t) for t in pubs])]
    orc.apply(ev_del)
    want2 = [sorted(x) for x in orc.fold_batch([("", b"pub", t) for t in pubs])]
    assert sum(len(x) for x in want1) > len(pubs)
    for bi, want in ((0, want1), (1, want1), (2, want2), (3, want2)):
        bad = [i for i in range(len(pubs)) if blocks[bi][i] != (0, want[i])]
        assert not bad, (bi, len(bad), pubs[bad[0]], blocks[bi][bad[0]][1][:5], want[bad[0]][:5])


def _churn_script(seed=23, n_subs=2000, n_pubs=2000, n_groups=30):
    """An initial subscription set, publishes (some holding words no filter
    has yet), and two rounds of churn groups that DO change the answers:
    subscribes of new filters (some bringing those words), unsubscribes of
    live ones, $share groups, remote nodes.  Returns the script for
    tools/bin/batch_gpu_check and, per W run, the groups as oracle events."""
    import random
    r = random.Random(seed)
    nodes = ["n0@h", "n1@h", "n2@h", "n70@h"]
    node_ids = [0, 1, 2, 70]
    words = [b"a", b"b", b"c", b"d"]
    fresh = [b"zz%d" % k for k in range(12)]   # unknown to every filter at first, held by publishes

    def rand_filter(ws):
        pre = (b"$share", r.choice([b"g1", b"g2"])) if r.random() < 0.15 else ()
        L = r.randint(1, 4)
        t = [b"+" if r.random() < 0.25 else (b"#" if (i == L - 1 and r.random() < 0.2) else r.choice(ws))
             for i in range(L)]
        return pre + tuple(t)

    live = {}
    lines = []
    sid = lambda k: ("", b"c%d" % k)
    line = lambda c, k, f: "%s %d %d %d 0 %s" % (c, node_ids[live[k][0]] if k in live else 0, k, live[k][1] if k in live else 0,
                                                 b"/".join(f).decode())
    for k in range(n_subs):
        live[k] = (r.choice(range(len(nodes))) if r.random() < 0.3 else 0, r.randint(0, 2), rand_filter(words))
        lines.append(line("S", k, live[k][2]))
    lines.append("A")
    init_events = [("updated", sid(k), None, [(nodes[ni], True, [(f, q)])]) for k, (ni, q, f) in live.items()]
    pubs = []
    for _ in range(n_pubs):
        L = r.randint(1, 4)
        t = [r.choice(words + fresh[:6]) if r.random() < 0.8 else r.choice(fresh) for _ in range(L)]
        pubs.append(tuple(t))
    lines += ["P 0 %s" % b"/".join(t).decode() for t in pubs]
    runs = []
    next_k = n_subs
    for mode in ("records", "ranges"):
        groups = []
        for g in range(n_groups):
            evs = []
            for _ in range(r.randint(1, 8)):
                if r.random() < 0.45 and live:
                    k = r.choice(sorted(live))
                    ni, q, f = live[k]
                    lines.append("X " + line("U", k, f))
                    evs.append(("deleted", sid(k), [(nodes[ni], True, [(f, q)])]))
                    del live[k]
                else:
                    k = next_k
                    next_k += 1
                    f = rand_filter(words + fresh)
                    live[k] = (r.choice(range(len(nodes))) if r.random() < 0.3 else 0, r.randint(0, 2), f)
                    lines.append("X " + line("S", k, f))
                    evs.append(("updated", sid(k), None, [(nodes[live[k][0]], True, [(f, live[k][1])])]))
            lines.append("G")
            groups.append(evs)
        lines.append("W %s 8 600 3" % mode)
        runs.append(groups)
    return "\n".join(lines) + "\n", nodes, node_ids, pubs, init_events, runs


@pytest.mark.gpu
def test_batchers_while_a_writer_changes_the_answers(tmp_path):
    """Verdict r3 next-round item 1: batchers of 600 publishes (a yield
    after 512, as the NIF prepares) match over and over while a writer
    applies 30 groups of subscribes / unsubscribes that change what the
    publishes match — some bringing words that publishes already hold, so
    batches prepared before such a group hold a stale unknown word.  Every
    matched publish's entries must equal the oracle's at the epoch its batch
    reports (the combined round's epoch); both device-side modes."""
    from oracle import oracle as O
    exe = os.path.join(ROOT, "tools", "bin", "batch_gpu_check")
    assert os.path.exists(exe), "tools/bin/batch_gpu_check not built (__graft_entry__.build())"
    script, nodes, node_ids, pubs, init_events, runs = _churn_script()
    (tmp_path / "s.txt").write_text(script)
    r = subprocess.run([exe, str(tmp_path / "s.txt"), str(tmp_path / "o.txt")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr
    name = {nid: nodes[i] for i, nid in enumerate(node_ids)}
    text = (tmp_path / "o.txt").read_text().splitlines()
    orc = O.TrieOracle(nodes[0])
    orc.apply(init_events)
    pos = 0
    for groups in runs:
        head = text[pos].split()
        assert head[0] == "W", head
        e0, ng, nl = int(head[1]), int(head[2]), int(head[3])
        assert ng == len(groups)
        gep = [int(text[pos + 1 + k].split()[2]) for k in range(ng)]
        assert gep == [e0 + k + 1 for k in range(ng)], (e0, gep[:5])
        body = text[pos + 1 + ng: pos + 1 + ng + nl]
        stats = text[pos + 1 + ng + nl].split()
        assert stats[0] == "v" and int(stats[1]) > 0
        pos += 2 + ng + nl
        by_state = {}
        for ln in body:
            f = ln.split(" ")
            i, ep, rc = int(f[0]), int(f[1]), int(f[2])
            assert rc == 0, ln[:200]
            j = ep - e0
            assert 0 <= j <= ng, (ep, e0)
            ents = []
            for e in f[3:]:
                kind, node, group, sub, info = e.split(",")
                kind, node, sub, info = int(kind), int(node), int(sub), int(info)
                if kind == 1:
                    ents.append(("A", ("", b"c%d" % sub), O.subinfo_repr(info)))
                elif kind == 2:
                    ents.append(("B", name[node], group.encode(), ("", b"c%d" % sub), O.subinfo_repr(info)))
                else:
                    ents.append(("C", name[node]))
            by_state.setdefault(j, []).append((i, sorted(ents)))
        assert len(by_state) >= 3, sorted(by_state)   # the matches interleaved with the writer
        changed = 0
        prev = None
        for j in range(ng + 1):
            if j:
                orc.apply(groups[j - 1])
            want = [sorted(x) for x in orc.fold_batch([("", b"pub", t) for t in pubs])]
            if prev is not None:
                changed += sum(a != b for a, b in zip(prev, want))
            prev = want
            for i, got in by_state.get(j, []):
                assert got == want[i], (j, i, pubs[i], got[:4], want[i][:4])
        assert changed > 0   # the writer's groups did change answers
