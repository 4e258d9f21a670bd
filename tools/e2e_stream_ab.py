#!/usr/bin/env python3
"""Range-mode end-to-end pass of config C (H2D publishes + words, match,
D2H offsets + entries, pinned host buffers) on torch's default stream (NULL:
the library runs on the legacy stream) vs an explicit torch stream,
interleaved; prints the median ms per batch of each as one JSON line."""
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
    w = W.config_c()
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    n = len(pubs)
    h_pubs = torch.from_numpy(pubs.view(np.uint32).view(np.int32).reshape(-1).copy()).pin_memory()
    h_words = torch.from_numpy(words.astype(np.int32)).pin_memory()
    d_pubs = torch.empty_like(h_pubs, device=dev)
    d_words = torch.empty_like(h_words, device=dev)
    cap = 4 * n
    d_rng = torch.empty(cap * 2, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    h_offs = torch.empty(n + 1, dtype=torch.int64).pin_memory()
    d_pubs.copy_(h_pubs)
    d_words.copy_(h_words)
    v.match_ranges_device(d_pubs.data_ptr(), n, d_words.data_ptr(), d_rng.data_ptr(), cap, d_offs.data_ptr(), 0)
    assert v.match_status(0) == 0
    ne = int(d_offs[-1].item())
    h_rng = torch.empty(ne * 2, dtype=torch.int32).pin_memory()
    side = torch.cuda.Stream()

    def step(sp):
        d_pubs.copy_(h_pubs, non_blocking=True)
        d_words.copy_(h_words, non_blocking=True)
        v.match_ranges_device(d_pubs.data_ptr(), n, d_words.data_ptr(), d_rng.data_ptr(), cap, d_offs.data_ptr(), sp)
        h_offs.copy_(d_offs, non_blocking=True)
        h_rng.copy_(d_rng[: ne * 2], non_blocking=True)

    res = {"default": [], "explicit": []}
    for rnd in range(6):
        for kind in ("default", "explicit"):
            ctx = torch.cuda.stream(side) if kind == "explicit" else torch.cuda.stream(torch.cuda.default_stream())
            with ctx:
                s = torch.cuda.current_stream()
                sp = s.cuda_stream
                step(sp)
                s.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    step(sp)
                s.synchronize()
                res[kind].append((time.perf_counter() - t0) / 10 * 1e3)
            assert v.match_status(sp) == 0
            assert int(h_offs[-1]) == ne
    print(json.dumps({k: statistics.median(x) for k, x in res.items()} | {"entries": ne, "publishes": n}))


if __name__ == "__main__":
    main()
