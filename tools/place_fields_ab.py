#!/usr/bin/env python3
"""Placement of caller-owned field sets (done-when:
"8 interleaved caller-owned-buffer states allocated through it spread <= 3 %").

N field sets allocated through cloudsc_fields_alloc WITH the write-pattern
search and N without it (CLOUDSC_PLACE_NONE), created alternately; each set's
inputs are copied from one state (search off) device-to-device, then the KSEG
kernel runs on every set round-robin through cloudsc_gpu_run on one shared
workspace, plude restored before each launch.  Kernel time = HIP events on the
null stream around each cloudsc_gpu_run.  One JSON line per set, then the
spread (slowest / fastest - 1) and median per group, and the search's cost.

Round 6 ("caller-owned sets from cloudsc_fields_alloc are never
more than 3 % above the state path"): --searched-only drops the unsearched
group, and --with-state adds a state created with its own (kernel-timed)
placement search, launched the same way on its own fields in the same rotation;
the summary then gives every searched set's time over the state's.

usage (GPU box): python tools/place_fields_ab.py [--sets 8] [--rounds 12] [--fp32] [--searched-only] [--with-state]
"""
import argparse
import ctypes as C
import json
import os
import statistics as stt
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--ngptot", type=int, default=163840)
    ap.add_argument("--nproma", type=int, default=64)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--searched-only", action="store_true")
    ap.add_argument("--with-state", action="store_true")
    a = ap.parse_args()
    prec = ca.FP32 if a.fp32 else ca.FP64
    lib = ca.gpu_lib()
    hip = C.CDLL("libamdhip64.so")
    for fn, args in (("hipMalloc", [C.POINTER(C.c_void_p), C.c_size_t]), ("hipMemset", [C.c_void_p, C.c_int, C.c_size_t]),
                     ("hipMemcpy", [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
                     ("hipEventCreate", [C.POINTER(C.c_void_p)]), ("hipEventRecord", [C.c_void_p, C.c_void_p]),
                     ("hipEventSynchronize", [C.c_void_p]),
                     ("hipEventElapsedTime", [C.POINTER(C.c_float), C.c_void_p, C.c_void_p])):
        getattr(hip, fn).argtypes = args
    ds = ca.load_dataset()
    ca.check(lib.cloudsc_debug_set_placement_search(0))
    src = ca.GpuState(ds, a.ngptot, a.nproma, prec)
    sf = ca.Fields()
    ca.check(lib.cloudsc_state_fields(src.h, C.byref(sf)))
    p = ca.Params.from_dict(ds.params)
    ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))
    sets = []
    for i in range(a.sets if a.searched_only else 2 * a.sets):
        place = a.searched_only or i % 2 == 0
        df = ca.DeviceFields(a.ngptot, a.nproma, ds.klev, prec, place=place)
        df.copy_from(sf, list(ca.INPUT_FIELDS))
        sets.append((place, df))
    ref_state = None
    if a.with_state:   # the state path: its own search (the KSEG kernel on its inputs), launched like the sets

        class StateFields:
            def __init__(self, g):
                self.g, self.f = g, ca.Fields()
                ca.check(lib.cloudsc_state_fields(g.h, C.byref(self.f)))

            def copy_from(self, src_fields, names):   # plude: the state's own pristine input
                ca.check(lib.cloudsc_state_reset(self.g.h))
                ca.check(lib.cloudsc_state_sync(self.g.h))

        ca.check(lib.cloudsc_debug_set_placement_search(-1))
        ref_state = ca.GpuState(ds, a.ngptot, a.nproma, prec)
        ca.check(lib.cloudsc_debug_set_placement_search(0))
        sets.append(("state", StateFields(ref_state)))
    ws = C.c_void_p()
    nb = lib.cloudsc_gpu_scratch_bytes(prec, ca.VARIANT_KSEG, a.ngptot, a.nproma, ds.klev)
    assert hip.hipMalloc(C.byref(ws), nb) == 0 and hip.hipMemset(ws, 0, 256) == 0
    e0, e1 = C.c_void_p(), C.c_void_p()
    hip.hipEventCreate(C.byref(e0))
    hip.hipEventCreate(C.byref(e1))

    def launch(df):
        df.copy_from(sf, ["plude"])
        hip.hipEventRecord(e0, None)
        ca.check(lib.cloudsc_gpu_run(0, None, prec, ca.VARIANT_KSEG, a.ngptot, a.nproma, ds.klev, C.byref(df.f), ws))
        hip.hipEventRecord(e1, None)
        hip.hipEventSynchronize(e1)
        t = C.c_float()
        hip.hipEventElapsedTime(C.byref(t), e0, e1)
        return t.value

    for _ in range(3):                      # warm the clock
        for _, df in sets:
            launch(df)
    times = [[] for _ in sets]
    for r in range(a.rounds):
        order = range(len(sets)) if r % 2 == 0 else reversed(range(len(sets)))
        for i in order:
            times[i].append(launch(sets[i][1]))
    ca.check(lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ws))
    med = [stt.median(t) for t in times]
    for i, (place, df) in enumerate(sets):
        rep = df.report.to_dict() if place != "state" else ref_state.placement_report()
        print(json.dumps({"set": i, "searched": place, "kernel_ms_median": round(med[i], 4),
                          "kernel_ms_min": round(min(times[i]), 4), "placement": rep}), flush=True)
    summary = {"precision": "fp32" if a.fp32 else "fp64", "sets_per_group": a.sets, "rounds": a.rounds}
    for place in ((True,) if a.searched_only else (False, True)):
        m = [med[i] for i, (pl, _) in enumerate(sets) if pl is place]
        key = "searched" if place else "unsearched"
        summary[key] = {"median_ms": round(stt.median(m), 4), "fastest_ms": round(min(m), 4),
                        "slowest_ms": round(max(m), 4), "spread": round(max(m) / min(m) - 1, 4)}
    if ref_state is not None:
        st_ms = [med[i] for i, (pl, _) in enumerate(sets) if pl == "state"][0]
        m = [med[i] for i, (pl, _) in enumerate(sets) if pl is True]
        summary["state_path_ms"] = round(st_ms, 4)
        summary["searched_over_state"] = {"median": round(stt.median(m) / st_ms, 4), "worst": round(max(m) / st_ms, 4),
                                          "best": round(min(m) / st_ms, 4)}
    cost = [df.report for pl, df in sets if pl is True]
    summary["search_cost"] = {"search_ms_median": round(stt.median(c.search_ms for c in cost), 1),
                              "launches_median": stt.median(c.launches for c in cost),
                              "peak_transient_gb_max": round(max(c.peak_transient_bytes for c in cost) / 1e9, 2)}
    print(json.dumps(summary), flush=True)
    hip.hipFree(ws)
    for pl, df in sets:
        if pl != "state":
            df.close()
    if ref_state is not None:
        ref_state.close()
    src.close()


if __name__ == "__main__":
    main()
