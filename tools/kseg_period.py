#!/usr/bin/env python3
"""Median start-to-start period and median duration of the KSEG kernel in a
rocprofv3 kernel trace (run_kernel_trace.csv / *_kernel_trace.csv): period -
duration is what each step spends outside the kernel (other kernels, gaps)."""
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "kseg_entry" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    du = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    per = [b - a for a, b in zip(st, st[1:])]
    tail = per[-99:]                      # the timed steps
    print("%s: kseg launches %d, median period %.2f us, median duration %.2f us, outside %.2f us" % (
        d, len(rows), statistics.median(tail) / 1e3, statistics.median(du[-100:]) / 1e3,
        (statistics.median(tail) - statistics.median(du[-100:])) / 1e3))
