"""Tier-2 (global-stack) walks in numbers: n publishes of x^16 against the
2^16 filters of 16 levels of {x, +}; prints rc, the error bits (VMQG_DEBUG)
and the stats per n.  GPU tool, not a test."""
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import harness as H          # noqa: E402
from vernemq_amd import _lib            # noqa: E402

node = "n@h"
prod = H.ProductDriver(node, device=0)
v = prod.view
v.set_option("dedupe", 0)
subs = [("updated", ("", b"s%d" % i), None, [(node, True, [(combo, i % 3)])])
        for i, combo in enumerate(itertools.product([b"x", b"+"], repeat=16))]
for lo in range(0, len(subs), 8192):
    prod.apply(subs[lo:lo + 8192])
arr, words = v.prepare([("", (b"x",) * 16)])
for n in [int(x) for x in (sys.argv[1:] or ["512", "1024", "2048", "3072", "4096"])]:
    for mode in ("records", "ranges"):
        try:
            if mode == "records":
                recs, offs = v.match_arrays(arr[np.zeros(n, dtype=np.int64)], words)
            else:
                rng, offs = v.match_ranges(arr[np.zeros(n, dtype=np.int64)], words)
            counts = np.diff(offs.astype(np.int64))
            res = "ok counts %s" % np.unique(counts)[:4]
        except _lib.VmqgError as e:
            res = "error %s" % e
        st = v.stats_raw()
        print(n, mode, res, {k: st[k] for k in ("deferred_tier1", "deferred_tier2", "wave_entries", "error_bits")},
              flush=True)
