"""Diagnosis aid: the shape of a config's match output on the GPU — per
publish, range entries (non-empty keys + remote nodes) and records — and
the engine's counters of one call (wide / retried / deduped publishes).
usage: python tools/diag_shape.py <config> [scale]   (E at 0.2 by default)"""
import sys

import numpy as np

sys.path.insert(0, ".")
from vernemq_amd import workloads as W            # noqa: E402
from vernemq_amd.reg_view import RegGpuView        # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "E"
    kw = {}
    if cfg == "E":
        kw["scale"] = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
    w = W.CONFIGS[cfg](**kw)
    v = RegGpuView(node=w.self_node, device=0, nodes=getattr(w, "nodes", None))
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    rng, roffs = v.match_ranges(pubs, words)
    recs, offs = v.match_arrays(pubs, words)
    st = v.stats_raw()
    ne = np.diff(np.asarray(roffs).astype(np.int64))
    nr = np.diff(np.asarray(offs).astype(np.int64))
    rg = np.asarray(rng).view(np.uint32).reshape(-1, 2)
    nkeys = np.zeros(len(ne), np.int64)
    starts = np.asarray(roffs).astype(np.int64)[:-1]
    iskey = (rg[:, 1] > 0).astype(np.int64)
    cs = np.concatenate([[0], np.cumsum(iskey)])
    nkeys = cs[starts + ne] - cs[starts]
    print(cfg, kw, "publishes", len(ne), "records", int(nr.sum()), "mean", float(nr.mean()))
    print("keys per publish hist (0..9, 10+):", np.bincount(np.minimum(nkeys, 10), minlength=11).tolist())
    print("remote entries per publish mean", float((ne - nkeys).mean()))
    q = np.percentile(nr, [50, 90, 99, 99.9])
    print("records per publish p50/p90/p99/p99.9", q.tolist(), "max", int(nr.max()))
    big = nkeys > 2
    print("publishes with > 2 keys:", int(big.sum()), "their records", int(nr[big].sum()))
    if st is not None:
        print("stats", {k: st[k] for k in ("many_key", "retried", "deferred_tier1", "deferred_tier2", "dedup",
                                            "dedup_walked") if k in st})


if __name__ == "__main__":
    main()
