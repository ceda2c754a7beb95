#!/usr/bin/env python3
"""Per-launch HBM traffic of the main kernel from rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md §HBM):
traffic = 2 x FETCH_SIZE (gfx950 reports half the bytes of coalesced reads)
        + WRITE_SIZE, both in KiB per dispatch.  Writes/updates the JSON that
bench.py reads for roofline.traffic.

usage: pmc_traffic.py <key> <fetch_dir> <write_dir> <out_json> [kernel_regex]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def per_dispatch(dirname, counter, regex):
    per = defaultdict(float)
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter and re.search(regex, row["Kernel_Name"]):
                per[row["Dispatch_Id"]] += float(row["Counter_Value"])
    return list(per.values())


def effective_clock_ghz(dirname, regex, nxcd=8):
    """Mean GRBM_GUI_ACTIVE cycles per XCD over the dispatch's duration (kernel
    trace of the same pass): the shader clock the kernel actually ran at."""
    grbm = per_dispatch_by_id(dirname, "GRBM_GUI_ACTIVE", regex)
    dur = {}
    for f in glob.glob(os.path.join(dirname, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if re.search(regex, row["Kernel_Name"]):
                dur[row["Dispatch_Id"]] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    ghz = [grbm[d] / nxcd / dur[d] for d in grbm if dur.get(d)]
    return round(sum(ghz) / len(ghz), 3) if ghz else None


def per_dispatch_by_id(dirname, counter, regex):
    per = defaultdict(float)
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter and re.search(regex, row["Kernel_Name"]):
                per[row["Dispatch_Id"]] += float(row["Counter_Value"])
    return per


def main():
    key, fdir, wdir, out = sys.argv[1:5]
    regex = sys.argv[5] if len(sys.argv) > 5 else "kseg_entry|kcache_entry|scc_entry"
    fe = per_dispatch(fdir, "FETCH_SIZE", regex)
    wr = per_dispatch(wdir, "WRITE_SIZE", regex)
    if not fe or not wr:
        sys.exit("no dispatches matched %r" % regex)
    fetch = sum(fe) / len(fe) * 1024.0
    write = sum(wr) / len(wr) * 1024.0
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dwarf-p-cloudsc_amd"))
    import cloudsc_amd as ca
    clock = effective_clock_ghz(fdir, regex)
    entry = {"fetch_size_bytes_raw": fetch, "write_size_bytes": write,
             "hbm_bytes_per_launch": 2.0 * fetch + write, "dispatches": [len(fe), len(wr)],
             "correction": "FETCH_SIZE x2 (gfx950 coalesced-read under-count), WRITE_SIZE as reported",
             "kernel_source_hash": ca.kernel_source_hash()}
    if clock:
        entry["effective_sclk_ghz"] = clock
        entry["effective_sclk_note"] = "GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration (FETCH pass)"
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[key] = entry
    json.dump(data, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(entry))


if __name__ == "__main__":
    main()
