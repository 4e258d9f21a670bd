#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/.

usage: summarize_prof.py <stats_dir> <fetch_dir> <write_dir> <out_json> [tag] [l2_dir] [lds_dir]

* kernel-trace stats: copied verbatim (…_kernel_stats.csv) — the average
  duration per kernel that bench.py's HIP-event timing must agree with;
* PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run): per-kernel
  mean per dispatch, in bytes = KB x 1024.  gfx950 correction (MI355X_MICROARCH.md
  §HBM): FETCH_SIZE reads half of a wide coalesced read stream, so the
  corrected read bytes are 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B/lane
  streaming stores.  Both raw and corrected numbers are kept;
* the build id of the profiled libvmqgpu.so (vmqg_build_id), which bench.py
  requires to equal the loaded library's before it reports `traffic`;
* optional passes: L2 hit rate TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum),
  LDS bank conflicts SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (cycles).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def find(d, pat):
    return sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))


def col(row, *names):
    for n in names:
        for k in row:
            if k.lower().replace("-", "_") == n.lower():
                return row[k]
    raise KeyError(names)


def pmc(d, counter):
    per = defaultdict(lambda: defaultdict(float))
    for f in find(d, "*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if col(row, "counter_name") != counter:
                continue
            k = col(row, "kernel_name")
            disp = col(row, "dispatch_id")
            per[k][disp] += float(col(row, "counter_value"))
    return {k: sum(v.values()) / len(v) for k, v in per.items()}


def main():
    sdir, fdir, wdir, out = sys.argv[1:5]
    tag = sys.argv[5] if len(sys.argv) > 5 else "latest"
    pdir = os.path.dirname(os.path.abspath(out))
    stats = {}
    for f in find(sdir, "*kernel_stats.csv"):
        shutil.copy(f, os.path.join(pdir, "kernel_stats_%s.csv" % tag))
        for row in csv.DictReader(open(f)):
            stats[col(row, "name")] = {"calls": int(col(row, "calls")),
                                       "avg_ns": float(col(row, "averagens")),
                                       "total_ns": float(col(row, "totaldurationns"))}
    fetch = pmc(fdir, "FETCH_SIZE")
    write = pmc(wdir, "WRITE_SIZE")
    l2dir = sys.argv[6] if len(sys.argv) > 6 else None
    ldsdir = sys.argv[7] if len(sys.argv) > 7 else None
    hit = pmc(l2dir, "TCC_HIT_sum") if l2dir else {}
    miss = pmc(l2dir, "TCC_MISS_sum") if l2dir else {}
    bank = pmc(ldsdir, "SQ_LDS_BANK_CONFLICT") if ldsdir else {}
    ldsact = pmc(ldsdir, "SQ_LDS_IDX_ACTIVE") if ldsdir else {}
    kernels = {}
    for name in set(fetch) | set(write) | set(stats):
        short = name.split("(")[0].replace("void ", "").replace("vmqg::", "")
        fk, wk = fetch.get(name), write.get(name)
        ent = {"full_name": name}
        if name in stats:
            ent.update(stats[name])
        if fk is not None:
            ent["fetch_kb_raw"] = fk
            ent["read_bytes_corrected"] = 2 * fk * 1024
        if wk is not None:
            ent["write_kb_raw"] = wk
            ent["write_bytes"] = wk * 1024
        if fk is not None and wk is not None:
            ent["hbm_bytes_per_launch"] = 2 * fk * 1024 + wk * 1024
        if name in hit and name in miss and hit[name] + miss[name] > 0:
            ent["l2_hit_rate"] = hit[name] / (hit[name] + miss[name])
        if name in bank and ldsact.get(name):
            ent["lds_bank_conflict_frac"] = bank[name] / ldsact[name]
            ent["lds_bank_conflict_cycles"] = bank[name]
        kernels[short] = ent
    build_id = os.environ.get("BUILD_ID")
    if not build_id:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from vernemq_amd import _lib
        build_id = _lib.build_id()
    json.dump({"tag": tag, "build_id": build_id, "kernels": kernels,
               "notes": "rocprofv3 --kernel-trace --stats, then separate --pmc FETCH_SIZE, --pmc WRITE_SIZE, "
                        "--pmc TCC_HIT_sum TCC_MISS_sum and --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE runs "
                        "of the same bench command; read bytes = 2 x FETCH_SIZE (gfx950 correction)"},
              open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(kernels, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
