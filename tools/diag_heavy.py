"""Diagnosis aid: where heavy-publish routing (vmqg_set_option "heavy_min")
writes different records than the fast EMIT (config A / B, records mode)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from vernemq_amd import workloads as W            # noqa: E402
from vernemq_amd.reg_view import RegGpuView        # noqa: E402


def run(cfg, settings):
    w = W.CONFIGS[cfg]()
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    outs = {}
    for hm, dd in settings:
        v.set_option("heavy_min", hm)
        v.set_option("dedupe", dd)
        recs, offs = v.match_arrays(pubs, words)
        outs[(hm, dd)] = (np.asarray(offs).astype(np.int64).copy(), np.asarray(recs).view(np.uint32).reshape(-1, 4).copy())
    o0, r0 = outs[settings[0]]
    cnt = np.diff(o0)
    print(cfg, "publishes", len(cnt), "records", int(o0[-1]), flush=True)
    for k in settings[1:]:
        o, r = outs[k]
        same_o = np.array_equal(o, o0)
        bad = np.nonzero((r != r0).any(axis=1))[0] if same_o else np.array([], np.int64)
        print(k, "offsets equal", same_o, "differing records", len(bad), flush=True)
        if len(bad):
            ps = np.unique(np.searchsorted(o0, bad, side="right") - 1)
            print("  publishes", len(ps), "counts", np.bincount(np.minimum(cnt[ps], 20)).tolist(), flush=True)
            for p in ps[:6]:
                a, b = o0[p], o0[p + 1]
                print("  p", int(p), "count", int(b - a), "pub", pubs[p].tolist() if hasattr(pubs[p], "tolist") else pubs[p])
                print("    want", r0[a:min(b, a + 4)].tolist())
                print("    got ", r[a:min(b, a + 4)].tolist(), flush=True)


if __name__ == "__main__":
    run("A", [(0, 0), (2, 0), (40, 0), (2, 1), (40, 1)])
    run("B", [(0, 0), (2, 0), (16, 0)])
