"""Records-mode output check on config E (scale given): the output buffer is
filled with a sentinel before each match, so a record position the kernels
never write shows up as the sentinel; run once per option setting (dedupe,
output groups) and compare the outputs of the settings byte for byte.
Prints one JSON line per setting.  GPU tool, not a test.

    python tools/diag_holes.py [scale]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vernemq_amd import workloads as W            # noqa: E402
from vernemq_amd.reg_view import RegGpuView       # noqa: E402


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.2
    w = W.config_e(scale=scale)
    n = w.n_subs
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes, max_mountpoints=max(1024, len(w.mps) + 1),
                   hints={"edges": 2 * n, "paths": 2 * n, "keys": n * 5 // 4, "records": n * 5 // 4,
                          "exact": n * 5 // 4})
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    npub = len(pubs)
    rng, roffs = v.match_ranges(pubs, words)
    per = np.where(rng["count"] > 0, rng["count"], 1).astype(np.int64)
    want = np.zeros(npub, dtype=np.int64)
    np.add.at(want, np.repeat(np.arange(npub), np.diff(roffs.astype(np.int64))), per)
    total = int(want.sum())
    dev = torch.device("cuda", 0)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = total + 1024
    sp = torch.cuda.current_stream().cuda_stream
    # how often each topic repeats in the batch (dedupe's duplicates)
    keys = [(int(pubs[i]["mountpoint"]), w.pub_topic(i)) for i in range(npub)]
    first_of = {}
    rep = np.zeros(npub, dtype=np.int64)
    for i, k in enumerate(keys):
        rep[i] = first_of.setdefault(k, i)
    ref = None
    for dd, gr in [(None, None), (0, 0), (0, 1), (1, 0), (1, 1), (2, 1)]:
        if dd is not None:   # the first pass: library defaults, right after the range match (the test's order)
            v.set_option("dedupe", dd)
            v.set_option("groups", gr)
        d_out = torch.full((cap * 4,), -1, dtype=torch.int32, device=dev)
        d_offs = torch.zeros(npub + 1, dtype=torch.int64, device=dev)
        for _ in range(1 if dd is None else 2):   # the second call runs with the mode the first chose (dedupe 2)
            d_out.fill_(-1)
            v.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(), sp)
            torch.cuda.synchronize()
            status = v.match_status(sp)
        offs = d_offs.cpu().numpy().astype(np.int64)
        recs = d_out.view(-1, 4)[:total]
        hole = (recs == -1).all(dim=1).cpu().numpy()
        hole_at = np.flatnonzero(hole)
        pub_of = np.searchsorted(offs, hole_at, side="right") - 1
        bad_pubs, per_pub = np.unique(pub_of, return_counts=True)
        st = v.stats_raw()
        line = {"dedupe": dd, "groups": gr, "status": status, "counts_ok": bool(np.array_equal(np.diff(offs), want)),
                "holes": int(hole.sum()), "publishes_with_holes": int(len(bad_pubs)),
                "stats": {k: st[k] for k in st if k.startswith(("dedup", "deferred", "many", "huge", "group"))}}
        if len(bad_pubs):
            ex = []
            for p, c in list(zip(bad_pubs, per_pub))[:12]:
                p = int(p)
                ex.append({"pub": p, "count": int(want[p]), "holes": int(c), "rep": int(rep[p]),
                           "rep_holes": bool(hole[offs[rep[p]]:offs[rep[p] + 1]].any()) if rep[p] != p else None,
                           "first_hole_rel": int(hole_at[pub_of == p][0] - offs[p]), "topic": keys[p][1].decode()})
            line["examples"] = ex
            whole = sum(1 for p, c in zip(bad_pubs, per_pub) if c == want[p])
            line["whole_publishes_unwritten"] = int(whole)
            line["bad_are_duplicates"] = int(sum(1 for p in bad_pubs if rep[p] != p))
            line["hole_pub_count_hist"] = np.histogram(np.log2(want[bad_pubs] + 1), bins=range(0, 24))[0].tolist()
        out = d_out[:total * 4].cpu().numpy()
        if ref is None:
            ref = out
        else:
            line["equal_to_first"] = bool(np.array_equal(out, ref))
            if not line["equal_to_first"]:
                diff = np.flatnonzero((out.reshape(-1, 4) != ref.reshape(-1, 4)).any(axis=1))
                line["differing_records"] = int(len(diff))
                dp = np.unique(np.searchsorted(offs, diff, side="right") - 1)
                line["differing_publishes"] = int(len(dp))
                line["differing_examples"] = [{"pub": int(p), "count": int(want[p]), "rep": int(rep[p])} for p in dp[:8]]
        print(json.dumps(line), flush=True)
        del d_out


if __name__ == "__main__":
    main()
