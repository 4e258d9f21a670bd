#!/usr/bin/env python3
"""The deferral-heavy scenario of test_output_offsets_of_a_large_deferral_heavy_batch
under every fast_g and store policy: which combination fails, and
how (debug of a VMQG_E_DEVICE)."""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import harness as H  # noqa: E402

node = "n@h"
orc = O.TrieOracle(node)
evs = []
hot = (b"h", b"x", b"y", b"z")
filters = set()
for combo in itertools.product([0, 1], repeat=4):
    t = tuple(b"+" if c else hot[i] for i, c in enumerate(combo))
    filters.add(t)
    for k in range(4):
        filters.add(t[:k] + (b"#",))
for i, t in enumerate(sorted(filters)):
    evs.append(("updated", ("", b"f%d" % i), None, [(node, True, [(t, i % 3)])]))
for j in range(0, 1000, 2):
    evs.append(("updated", ("", b"n%d" % j), None, [(node, True, [((b"n", b"%d" % j), 1)])]))
orc.apply(evs)
topics = [("", (b"n", b"%d" % j)) for j in range(1000)] + [("", hot)]
want = np.array([len(x) for x in orc.fold_batch([(mp, b"pub", t) for mp, t in topics])], dtype=np.int64)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
for fg, nt in itertools.product([1, 2, 4], [0, 1]):
    prod = H.ProductDriver(node, device=0)
    prod.apply(evs)
    v = prod.view
    for k, x in (("fast_g", fg), ("nt_stores", nt)):
        v.set_option(k, x)
    arr, words = v.prepare(topics)
    idx = np.arange(n) % 1000
    idx[::23] = 1000
    try:
        recs, offs = v.match_arrays(arr[idx], words)
        counts = np.diff(offs.astype(np.int64))
        bad = np.flatnonzero(counts != want[idx])
        print("fast_g %d nt_stores %d: ok, %d counts differ%s, stats %s" % (
            fg, nt, len(bad), (" first %d got %d want %d" % (bad[0], counts[bad[0]], want[idx][bad[0]])) if len(bad) else "",
            {k: v.stats_raw()[k] for k in ("deferred_tier1", "deferred_tier2", "retried", "many_key")}), flush=True)
    except Exception as e:
        print("fast_g %d nt_stores %d: %s" % (fg, nt, e), flush=True)
    del prod
