#!/usr/bin/env python3
"""Fixed cost of one vmqg_match_device call on config C: step time with the
library's kernel timing events on and off, and over batch sizes 2^17..2^21
(the intercept of a least-squares line through them is the per-call cost
that does not scale with the batch: launches, their gaps, empty wave-tier
launches, the scan), and the host time per call to enqueue it.  Interleaved rounds, one process, one JSON line."""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    dev = torch.device("cuda", 0)
    w = W.config_c(n_pubs=1 << 21)
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = 66 * len(pubs)
    d_out = torch.empty(cap * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(len(pubs) + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    sizes = [1 << 17, 1 << 18, 1 << 19, 1 << 20, 1 << 21]
    variants = [(n, t) for n in sizes for t in (0, 1)]
    res = {str(x): [] for x in variants}
    enq = {str(x): [] for x in variants}   # host time per call to enqueue (no sync)
    steps = 20
    for _ in range(5):
        for n, t in variants:
            v.set_timing(bool(t))
            for _ in range(2):
                v.match_device(d_pubs.data_ptr(), n, d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(), sp)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                v.match_device(d_pubs.data_ptr(), n, d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(), sp)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            res[str((n, t))].append((time.perf_counter() - t0) / steps * 1e6)
            enq[str((n, t))].append((t1 - t0) / steps * 1e6)
            v.set_timing(False)
    assert v.match_status(sp) == 0
    med = {k: statistics.median(x) for k, x in res.items()}
    out = {"config": "C", "step_us": med, "host_enqueue_us": {k: statistics.median(x) for k, x in enq.items()}}
    for t in (0, 1):
        xs = np.array(sizes, dtype=float)
        ys = np.array([med[str((n, t))] for n in sizes])
        b, a = np.polyfit(xs, ys, 1)
        out["fit_timing%d" % t] = {"per_call_us": a, "ns_per_publish": b * 1e3}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
