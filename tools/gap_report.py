#!/usr/bin/env python3
"""Per-step GPU timeline of bench.py config C from a rocprofv3 kernel trace:
for the last `--steps` match calls (five launches each: COUNT fast tier,
scan (+ wave tiers), EMIT fast tier; older builds had separate wave-tier
launches), the median duration
of every launch and of the idle gap before it (end of the previous kernel to
start of this one).  usage: gap_report.py <kernel_trace.csv> [--steps N]"""
import argparse
import csv
import json
import statistics


def short(name):
    for k in ("k_match_fast<0", "k_match_fast<1", "k_match_wave<0", "k_match_wave<1", "k_scan_offsets"):
        if k in name:
            return k
    return name.split("(")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    match = [r for r in rows if r[2].startswith("k_match") or r[2] == "k_scan_offsets"]
    # a step: the launches from one COUNT fast tier to the next
    starts = [i for i, r in enumerate(match) if r[2] == "k_match_fast<0"]
    steps = [match[a:b] for a, b in zip(starts, starts[1:])][-args.steps:]
    seq = [k for (_, _, k) in steps[-1]]
    steps = [st for st in steps if [k for (_, _, k) in st] == seq]
    dur = {k: [] for k in seq}
    gap = {k: [] for k in seq}
    step_ns = []
    for s_idx, st in enumerate(steps):
        prev_end = None
        if s_idx > 0:
            prev_end = steps[s_idx - 1][-1][1]
        for (t0, t1, k) in st:
            dur[k].append(t1 - t0)
            if prev_end is not None:
                gap[k].append(t0 - prev_end)
            prev_end = t1
        if s_idx > 0:
            step_ns.append(st[-1][1] - steps[s_idx - 1][-1][1])
    med = lambda x: statistics.median(x) / 1e3 if x else None
    out = {"steps": len(steps), "kernel_us": {k: med(v) for k, v in dur.items()},
           "gap_before_us": {k: med(v) for k, v in gap.items()},
           "step_us": med(step_ns),
           "kernels_sum_us": sum(med(v) for v in dur.values()),
           "gaps_sum_us": sum(med(v) for v in gap.values() if v)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
