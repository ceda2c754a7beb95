#!/usr/bin/env python3
"""Diagnostic: schedule of the persistent segmented kernel (KSEG) from the trace
build (build/libkseg_trace.so: make -C dwarf-p-cloudsc_amd variant
VFLAGS=-DCLOUDSC_KSEG_TRACE OUT=../build/libkseg_trace.so): per-item start/end on the
100 MHz realtime clock, workgroup and XCC.  Prints per-segment item durations,
the makespan, the workgroups' busy fraction and the tail."""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
os.environ.setdefault("CLOUDSC_AMD_LIB", os.path.join(REPO, "build", "libkseg_trace.so"))
import cloudsc_amd as ca  # noqa: E402

lib = ca.gpu_lib()
lib.cloudsc_kseg_trace.argtypes = [C.c_void_p, C.c_int]
ds = ca.load_dataset()
prec = ca.FP64 if (len(sys.argv) < 2 or sys.argv[1] == "fp64") else ca.FP32
ngptot, nproma = 163840, int(os.environ.get("TRACE_NPROMA", "64"))
nb = (ngptot // nproma) * ((nproma + 63) // 64)   # one-wave items: 64-column sub-blocks
g = ca.GpuState(ds, ngptot, nproma, prec)
for nseg in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,1,3").split(",")]:
    ca.kseg_schedule(nseg, 0)      # segments per column (0 = the default)
    g.run(ca.VARIANT_KSEG, 2)
    ms = g.run(ca.VARIANT_KSEG, 1)
    n = nseg * nb
    buf = np.zeros(4 * n, dtype=np.uint64)
    ca.check(lib.cloudsc_kseg_trace(buf.ctypes.data, n))
    t = buf.reshape(n, 4).astype(np.int64)
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0   # microseconds
    dur = en - st
    wg = t[:, 2]
    wait = (t[:, 3] - t[:, 0]) / 100.0                       # microseconds spent polling for the predecessor
    makespan = en.max()
    busy = {}
    last_end = {}
    for i in range(n):
        busy[wg[i]] = busy.get(wg[i], 0.0) + dur[i]
        last_end[wg[i]] = max(last_end.get(wg[i], 0.0), en[i])
    nwg = len(busy)
    segd = [dur[s * nb:(s + 1) * nb] for s in range(nseg)]
    le = np.array(sorted(last_end.values()))
    out = {"nseg": nseg, "kernel_ms": float(ms[0]), "makespan_us": round(float(makespan), 1),
           "workgroups": nwg, "busy_frac": round(float(sum(busy.values()) / (nwg * makespan)), 4),
           "wg_last_end_us_p10_p50_p90": [round(float(np.percentile(le, q)), 1) for q in (10, 50, 90)],
           "first_start_spread_us": round(float(np.sort(st)[min(nwg, n) - 1]), 1),
           "seg_dur_us_mean": [round(float(d.mean()), 1) for d in segd],
           "seg_dur_us_p10_p90": [[round(float(np.percentile(d, 10)), 1), round(float(np.percentile(d, 90)), 1)]
                                  for d in segd],
           "wait_frac_of_busy": round(float(wait.sum() / dur.sum()), 4),
           "seg_wait_us_mean": [round(float(wait[s * nb:(s + 1) * nb].mean()), 1) for s in range(nseg)]}
    # concurrency timeline: mean number of running items in 20 equal time bins,
    # and the mean duration of the items that START in each bin (per segment)
    edges = np.linspace(0.0, makespan, 21)
    active = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(en, b) - np.maximum(st, a), 0.0, None)
        active.append(round(float(ov.sum() / (b - a)), 1))
    out["active_items_per_bin"] = active
    out["first_drop_below_full_us"] = round(float(le[0]), 1)
    sbin = np.clip(np.digitize(st, edges) - 1, 0, 19)
    out["dur_us_by_start_bin"] = [round(float(dur[sbin == i].mean()), 1) if np.any(sbin == i) else None
                                  for i in range(20)]
    print(json.dumps(out), flush=True)
ca.kseg_schedule(0, 0)
g.close()
