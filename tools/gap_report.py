#!/usr/bin/env python3
"""Print the last kernels of a rocprofv3 kernel trace with their durations
and the idle gap before each.  usage: gap_report.py run_kernel_trace.csv [n]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
prev = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-44s dur %8.1f us  gap %7.1f us" % (r["Kernel_Name"][:44], (e - s) / 1e3, (s - prev) / 1e3 if prev else 0))
    prev = e
