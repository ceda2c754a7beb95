#!/usr/bin/env python3
"""Table of tools/placement_pmc.sh: per pass, the last reps x launches
kseg_entry dispatches grouped by state (median duration and mean counters).
usage: placement_pmc_table.py [dir=gpurun_out] [reps=6] [launches=5]"""
import collections
import csv
import os
import statistics as stt
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
launches = int(sys.argv[3]) if len(sys.argv) > 3 else 5
for name in sorted(x for x in os.listdir(d) if x.startswith("ppmc_") and os.path.isdir(os.path.join(d, x))):
    rows = [r for r in csv.DictReader(open(os.path.join(d, name, "p_counter_collection.csv")))
            if "kseg_entry" in r["Kernel_Name"]]
    per = collections.OrderedDict()
    for r in rows:
        e = per.setdefault(int(r["Dispatch_Id"]), {"ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    disp = list(per.values())[-reps * launches:]
    names = [k for k in disp[0] if k != "ms"]
    print("%s  state   ms      %s" % (name, "  ".join("%14s" % n.replace("_sum", "")[-14:] for n in names)))
    for s in range(reps):
        g = disp[s * launches:(s + 1) * launches]
        print("%s  %5d  %.4f  %s" % (name, s, stt.median(x["ms"] for x in g),
                                     "  ".join("%14.4g" % stt.mean(x[n] for x in g) for n in names)))
