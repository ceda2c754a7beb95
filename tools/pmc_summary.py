#!/usr/bin/env python3
"""Summarise rocprofv3 counter passes (tools/pmc_session.sh output): per-dispatch
average of every counter for the main kernel, plus derived quantities."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirname, kernel_regex="kcache_entry|scc_entry|kseg_entry"):
    import re
    vals = defaultdict(list)
    dur = []
    for f in sorted(glob.glob(os.path.join(dirname, "p*", "run_counter_collection.csv"))):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if not re.search(kernel_regex, row["Kernel_Name"]):
                continue
            key = (row["Dispatch_Id"], row["Counter_Name"])
            per[key] += float(row["Counter_Value"])
        for (d, name), v in per.items():
            vals[name].append(v)
    for f in sorted(glob.glob(os.path.join(dirname, "p*", "run_kernel_trace.csv"))):
        for row in csv.DictReader(open(f)):
            if re.search(kernel_regex, row["Kernel_Name"]):
                dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    avg["_kernel_ms_avg_profiled"] = sum(dur) / len(dur) if dur else None
    return avg


if __name__ == "__main__":
    for d in sys.argv[1:]:
        a = load(d)
        print("==", d)
        for k in sorted(a):
            print("  %-32s %.6g" % (k, a[k]) if a[k] is not None else "  %s None" % k)
        w = a.get("SQ_WAVES", 0)
        if w:
            print("  per-wave: VALU %.0f SALU %.0f SMEM %.0f VMEM_RD %.0f VMEM_WR %.0f BRANCH %.0f" % tuple(
                a.get(n, 0) / w for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                                          "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH")))
        if "SQ_WAVE_CYCLES" in a:
            wc = a["SQ_WAVE_CYCLES"]
            print("  wave-cycle shares: wait_any %.3f wait_inst_any %.3f active_any %.3f active_valu %.3f" % (
                a["SQ_WAIT_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc, a["SQ_ACTIVE_INST_ANY"] / wc,
                a["SQ_ACTIVE_INST_VALU"] / wc))
        if "SQC_ICACHE_HITS" in a:
            h, m = a["SQC_ICACHE_HITS"], a["SQC_ICACHE_MISSES"]
            print("  icache hit rate %.4f" % (h / (h + m)))
        if "FETCH_SIZE" in a:
            print("  FETCH_SIZE KB %.0f (x2 gfx950 correction -> %.3f GB)  WRITE_SIZE KB %.0f (%.3f GB)" % (
                a["FETCH_SIZE"], 2 * a["FETCH_SIZE"] * 1024 / 1e9, a.get("WRITE_SIZE", 0),
                a.get("WRITE_SIZE", 0) * 1024 / 1e9))
