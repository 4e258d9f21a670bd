#!/usr/bin/env python3
"""Where does the GPU idle between two vmqg_match_device calls?  Config C,
2^20 publishes; mode 0: calls back to back; mode 1: a one-element torch fill
kernel queued between calls.  Run under rocprofv3 --kernel-trace and read the
gaps between kernels from the trace (see tools/gap_report.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    dev = torch.device("cuda", 0)
    w = W.config_c()
    v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
    w.load_into(v)
    pubs, words = w.publish_arrays(v)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = 66 * len(pubs)
    d_out = torch.empty(cap * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(len(pubs) + 1, dtype=torch.int64, device=dev)
    x = torch.zeros(1, dtype=torch.int32, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(12):
        v.match_device(d_pubs.data_ptr(), len(pubs), d_words.data_ptr(), d_out.data_ptr(), cap, d_offs.data_ptr(), sp)
        if mode == 1:
            x.fill_(1)
    torch.cuda.synchronize()
    assert v.match_status(sp) == 0


if __name__ == "__main__":
    main()
