#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration at the kernels' own access widths
(VERDICT r04 weak 5).  MI355X_MICROARCH.md calibrates FETCH_SIZE (reports 1/2
of the bytes) and WRITE_SIZE (exact) only for 16-B-per-lane streaming
accesses; the CLOUDSC kernels move 8 B (fp64) / 4 B (fp32) per lane.

Two modes:
  run       (under rocprofv3 --pmc, one counter per run): stream a known byte
            count through cloudsc_debug_stream_probe, read and write, at 4, 8
            and 16 B per lane, `reps` launches each (the dispatch order is fixed:
            width 4, 8, 16 for reads, then for writes).
  analyse   <fetch_dir> <write_dir> [out_json]: per (mode, width) the counter's
            bytes per launch over the known bytes -> the factor that turns the
            counter into bytes; printed, and merged into the traffic JSON under
            "calibration".
usage: python tools/calib_counters.py run [--gib 4] [--reps 3]
       python tools/calib_counters.py analyse <fetch_dir> <write_dir> [profiles/traffic_latest.json]
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
WIDTHS = (4, 8, 16)


def run(gib, reps):
    import ctypes as C
    import cloudsc_amd as ca
    lib = ca.gpu_lib()
    lib.cloudsc_debug_stream_probe.argtypes = [C.c_int, C.c_int, C.c_int, C.c_longlong, C.c_int,
                                               C.POINTER(C.c_double)]
    nbytes = int(gib * (1 << 30))
    for mode in (0, 1):
        for w in WIDTHS:
            ms = C.c_double()
            ca.check(lib.cloudsc_debug_stream_probe(0, mode, w, nbytes, reps, C.byref(ms)))
            print(json.dumps({"mode": "write" if mode else "read", "width": w, "bytes": nbytes, "reps": reps,
                              "ms": round(ms.value, 4), "GBs": round(nbytes / ms.value / 1e6, 1)}), flush=True)


def dispatch_values(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "stream_probe" in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    per = {}
    for did, name, v in rows:
        per.setdefault(did, [name, 0.0])[1] += v
    return [per[k] for k in sorted(per)]


def analyse(fdir, wdir, out=None, gib=4.0, reps=3):
    nbytes = gib * (1 << 30)
    res = {}
    for d, counter in ((fdir, "FETCH_SIZE"), (wdir, "WRITE_SIZE")):
        disp = dispatch_values(d, counter)
        # 6 configurations x reps launches, in run() order
        for k, (mode, w) in enumerate((m, w) for m in ("read", "write") for w in WIDTHS):
            vals = [v for _, v in disp[k * reps:(k + 1) * reps]]
            names = {n for n, _ in disp[k * reps:(k + 1) * reps]}
            kb = sum(vals) / len(vals)
            key = "%s_%dB_per_lane" % (mode, w)
            res.setdefault(key, {})[counter] = {"counter_bytes": kb * 1024.0, "known_bytes": nbytes,
                                                "bytes_per_counter_byte": round(nbytes / (kb * 1024.0), 4)
                                                if kb else None, "kernels": sorted(names)}
    print(json.dumps(res, indent=1))
    if out:
        data = json.load(open(out)) if os.path.exists(out) else {}
        data["calibration"] = {"what": "rocprofv3 FETCH_SIZE / WRITE_SIZE over a known byte count streamed with "
                                       "each access width (cloudsc_debug_stream_probe, non-temporal, consecutive "
                                       "lanes on consecutive elements); bytes_per_counter_byte is the factor",
                               "results": res}
        json.dump(data, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        gib = float(sys.argv[sys.argv.index("--gib") + 1]) if "--gib" in sys.argv else 4.0
        reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
        run(gib, reps)
    else:
        analyse(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
