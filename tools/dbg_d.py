#!/usr/bin/env python3
"""Config D at reduced scale, step by step with timings (debug of the
test_config_d_churn_parity run that went silent): load, oracle load, match
per mode, status after every call.  A Python stack dump after 100 s."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(100, exit=False)
t0 = time.time()


def log(*a):
    print("[%6.1fs]" % (time.time() - t0), *a, flush=True)


import numpy as np  # noqa: E402
from vernemq_amd import workloads as W  # noqa: E402
from vernemq_amd.reg_view import RegGpuView  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.05
fast_g = int(sys.argv[2]) if len(sys.argv) > 2 else 1
w = W.config_d(scale=scale, n_pubs=20_000)
log("generated", w.notes["n_live"])
v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
v.set_option("fast_g", fast_g)
ids = w.load_into(v, n=w.notes["n_live"])
log("loaded")
pubs, words = w.publish_arrays(v)
for mode in ("records", "ranges"):
    for rep in range(2):
        t = time.time()
        if mode == "records":
            recs, offs = v.match_arrays(pubs, words)
        else:
            rng, offs = v.match_ranges(pubs, words)
        log(mode, rep, "%.1f ms" % ((time.time() - t) * 1e3), "total", int(offs[-1]), v.stats_raw()["deferred_tier1"])
log("done")
