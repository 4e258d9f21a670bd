#!/usr/bin/env python3
"""Probe: does COUNT of batch k+1 overlap EMIT of batch k?  Two matcher
contexts (two arenas) on two streams, batches alternating, vs one context
on one stream.  Prints us per batch for both.  (Feasibility probe for
double-buffered match scratch; not a bench line.)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vernemq_amd import workloads as W  # noqa: E402
from vernemq_amd.reg_view import RegGpuView  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
w = W.config_c(n_dev=1_000_000, n_pubs=1 << 20, seed=0xC)
views = []
for _ in range(2):
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes,
                   hints={"edges": 3_001_024, "paths": 3_001_024, "keys": 1_001_024, "records": 1_001_024})
    w.load_into(v)
    views.append(v)
pwid = views[0].intern_words(w.pub_words, create=False).astype(np.int64)
pubs, words = w.publish_arrays_ids(pwid, np.array([0], dtype=np.uint32))
n = len(pubs)
d_p = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
d_w = torch.from_numpy(words.astype(np.int32)).to(dev)
cap = 65 * n
outs = [torch.empty(cap * 4, dtype=torch.int32, device=dev) for _ in range(2)]
offs = [torch.zeros(n + 1, dtype=torch.int64, device=dev) for _ in range(2)]
streams = [torch.cuda.Stream() for _ in range(2)]


def run(k_steps, two):
    for i in range(k_steps):
        j = i % 2 if two else 0
        views[j].match_device(d_p.data_ptr(), n, d_w.data_ptr(), outs[j].data_ptr(), cap, offs[j].data_ptr(),
                              streams[j].cuda_stream)


for two in (False, True, False, True):
    run(4, two)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(40, two)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print("two contexts/streams" if two else "one context/stream", "%.1f us per batch" % (el / 40 * 1e6), flush=True)
for v in views:
    assert v.match_status(0) == 0
