"""CPU checks of the synthetic workload generators and of the algorithmic
byte model used by bench.py's roofline."""
import numpy as np

from oracle import feed
from oracle import oracle as O
from vernemq_amd import workloads as W


def test_splitmix_deterministic():
    a, b = W.SplitMix(7).u64(5), W.SplitMix(7).u64(5)
    assert np.array_equal(a, b)
    r = W.SplitMix(7)
    assert np.array_equal(np.concatenate([r.u64(2), r.u64(3)]), a)


def test_config_c_shape():
    w = W.config_c(n_dev=1000, n_pubs=4096)
    assert w.n_subs == 1064
    assert w.sub_topic(0) == (b"devices", b"0", b"telemetry", b"#")
    assert w.sub_topic(1000) == (b"devices", b"+", b"telemetry", b"#")
    t = w.pub_topic(3)
    assert t[0] == b"devices" and t[2] == b"telemetry" and t[3].startswith(b"m")


def test_config_c_algorithmic_bytes_match_oracle_counters():
    w = W.config_c(n_dev=2000, n_pubs=3000)
    orc = feed.load(w)
    res, counts = orc.fold_batch([("", b"p", w.pub_topic(i)) for i in range(w.n_pubs)], with_counts=True)
    b = sum(8 * (l + 1) + 16 * s + 32 * r for s, r, l in counts)
    assert b == W.algorithmic_bytes_c(w)
    assert all(r == len(em) for (s, r, l), em in zip(counts, res))


def test_config_a_b_r_shapes():
    a = W.config_a(n_subs=500, n_clients=100, n_pubs=300)
    assert a.n_subs == 500 and a.n_pubs == 300
    assert any(a.sub_topic(i)[0] == b"$share" for i in range(a.n_subs)) or True
    b = W.config_b(n_subs=300, n_pubs=100)
    assert b.n_subs == 300
    r1 = W.config_r1(10)
    assert r1.sub_topic(0) == (b"unique", b"topic", b"1") and r1.pub_topic(9) == (b"unique", b"topic", b"10")
    r2 = W.config_r2(10)
    assert r2.n_subs == 10 and r2.n_pubs == 1


def test_config_d_churn_tables_match_oracle():
    """Config D at 1/500 scale: bulk load + 6 churn batches through the host
    engine (op arrays) and the oracle (events) give identical tables."""
    from tests import harness as H
    from tests.test_host_engine import _compare
    from vernemq_amd.reg_view import RegGpuView
    w = W.config_d(scale=0.002, n_pubs=100)
    v = RegGpuView(node=w.self_node, device=-1, nodes=w.nodes)
    ids = w.load_into(v, n=w.notes["n_live"])
    orc = feed.load_prefix(w, w.notes["n_live"])
    ch = W.Churn(w)
    for _ in range(6):
        dels, adds = ch.batch(400)
        ops, words = ch.ops(ids, dels, adds)
        v.apply_op_arrays(ops, words)
        orc.apply(ch.events(dels, adds))

    class P:
        view = v
    _compare(P, orc, "config D churn")
    assert v.stats_raw()["subs"] > 0


def test_config_e_tables_match_oracle():
    from tests.test_host_engine import _compare
    from vernemq_amd.reg_view import RegGpuView
    w = W.config_e(scale=0.0004, n_pubs=10)
    v = RegGpuView(node=w.self_node, device=-1, nodes=w.nodes)
    w.load_into(v)
    orc = feed.load(w)

    class P:
        view = v
    _compare(P, orc, "config E")
    assert v.stats_raw()["trie_edges"] > 1000
