#!/usr/bin/env python3
"""Cost of each half of the pipelined (mixed) launch on config C: a big batch
followed by a 1-publish batch makes the mixed launch EMIT-only (big EMIT +
1 COUNT); the next big batch makes it COUNT-only; a third big one mixes both.
Prints the median HIP-event duration of each kind, and of the unpipelined
COUNT / EMIT launches, as one JSON line."""
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    dev = torch.device("cuda", 0)
    w = W.config_c()
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    n = len(pubs)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = 66 * n
    outs = [torch.empty(cap * 4, dtype=torch.int32, device=dev) for _ in range(3)]
    offs = [torch.zeros(n + 1, dtype=torch.int64, device=dev) for _ in range(3)]
    sp = torch.cuda.current_stream().cuda_stream
    k = [0]

    def sub(npub):
        i = k[0] % 3
        k[0] += 1
        v.match_submit(d_pubs.data_ptr(), npub, d_words.data_ptr(), outs[i].data_ptr(), cap, offs[i].data_ptr(), sp)

    def timed_submit(npub):
        v.set_timing(True)
        sub(npub)
        torch.cuda.synchronize()
        m, nm, _, _ = v.pipeline_times()
        v.set_timing(False)
        assert nm == 1
        return m / 1e3

    res = {"emit_only": [], "count_only": [], "both": [], "count": [], "emit": []}
    for rep in range(6):
        sub(n)
        res["emit_only"].append(timed_submit(1))
        res["count_only"].append(timed_submit(n))
        res["both"].append(timed_submit(n))
        v.match_flush()
        assert v.match_status(sp) == 0
        v.set_timing(True)
        v.match_device(d_pubs.data_ptr(), n, d_words.data_ptr(), outs[0].data_ptr(), cap, offs[0].data_ptr(), sp)
        torch.cuda.synchronize()
        c, e, _ = v.kernel_times()
        v.set_timing(False)
        res["count"].append(c / 1e3)
        res["emit"].append(e / 1e3)
    print(json.dumps({k2: statistics.median(x) for k2, x in res.items()}))


if __name__ == "__main__":
    main()
