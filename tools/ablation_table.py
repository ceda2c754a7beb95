#!/usr/bin/env python3
"""Table of tools/ablation_gpu.sh results: interleaved kernel time (times.txt)
and the per-build counters (rocprofv3 --pmc, the last 3 of 5 KSEG dispatches):
VALU wave-instructions per launch, fp64 classes, and the effective clock
GRBM_GUI_ACTIVE / 8 XCDs / dispatch time.   usage: ablation_table.py [dir]"""
import collections
import csv
import glob
import os
import re
import sys

d0 = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abl"
P = "F32" if len(sys.argv) > 2 and sys.argv[2] == "fp32" else "F64"
times = {}
for line in open(os.path.join(d0, "times.txt")):
    m = re.match(r"(\S+)\.so\s+median ([\d.]+) ms.*ratio-to-first ([\d.]+)", line)
    if m:
        times[m.group(1)] = (float(m.group(2)), float(m.group(3)))
rows = {}
for d in sorted(glob.glob(os.path.join(d0, "pmc_*/"))):
    n = os.path.basename(d.rstrip("/"))[4:]
    cc = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    kt = glob.glob(d + "**/*kernel_trace.csv", recursive=True)
    if not cc or not kt:
        continue
    dur = {r["Dispatch_Id"]: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
           for r in csv.DictReader(open(kt[0])) if "kseg_entry" in r["Kernel_Name"]}
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(cc[0])):
        if r["Dispatch_Id"] in dur:
            acc[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    disp = sorted(dur, key=int)[-3:]
    cnt = collections.defaultdict(float)
    for dd in disp:
        for (x, cn), v in acc.items():
            if x == dd:
                cnt[cn] += v / len(disp)
    ms = 1e3 * sum(dur[x] for x in disp) / len(disp)
    rows[n] = (cnt, ms)
base = rows["full"][0]["SQ_INSTS_VALU"]
order = sorted(rows, key=lambda n: times.get(n, (0, 9))[1])
print("%-9s %10s %8s %8s %9s %9s %9s %9s %8s %7s" % ("build", "time ms", "t/full", "VALU", "dVALU %", "FMA",
                                                    "MUL", "ADD", "pmc ms", "GHz"))
for n in order:
    c, ms = rows[n]
    t = times.get(n, (float("nan"), float("nan")))
    ghz = c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9
    print("%-9s %10.4f %8.4f %8.3e %9.1f %9.3e %9.3e %9.3e %8.3f %7.2f" % (
        n, t[0], t[1], c["SQ_INSTS_VALU"], 100 * (c["SQ_INSTS_VALU"] / base - 1), c["SQ_INSTS_VALU_FMA_" + P],
        c["SQ_INSTS_VALU_MUL_" + P], c["SQ_INSTS_VALU_ADD_" + P], ms, ghz))
