#!/usr/bin/env python3
"""Per-call cost of cloudsc_host_run (the GPU drop-in's engine) by part, call
by call (round 6).

For each (ncols, nproma) block shape: a host state in block layout whose output
arrays are fresh np.empty allocations (their pages not yet touched, like the
reference driver's freshly allocated outputs) and calls 1..N of
cloudsc_host_run on it with cloudsc_host_run_profile on, one profile per call:
the first call carries the context and buffer allocations (and, in a fresh
process, the HIP runtime's start-up), the second the first touch of the output
pages, the later ones are the steady state.  One JSON line per call.

usage (GPU box): python tools/host_run_cost.py [--shapes 32:32,512:512] [--calls 4]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


class Profile(C.Structure):
    _fields_ = [("calls", C.c_longlong)] + [(n, C.c_double) for n in (
        "setup_ms", "pack_ms", "h2d_ms", "kernel_ms", "d2h_ms", "wait_ms", "unpack_ms", "total_ms", "alloc_ms",
        "enqueue_ms", "max_call_ms")] + [("first_calls", C.c_longlong), ("first_calls_ms", C.c_double)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="32:32,512:512")
    ap.add_argument("--calls", type=int, default=4)
    a = ap.parse_args()
    lib = ca.gpu_lib()
    lib.cloudsc_host_run_profile.argtypes = [C.c_int, C.POINTER(Profile)]
    ds = ca.load_dataset()
    p = ca.Params.from_dict(ds.params)
    for shape in a.shapes.split(","):
        ncols, nproma = (int(x) for x in shape.split(":"))
        st = ca.make_host_state(ds, ncols, nproma, ca.FP64)
        plude0 = st.arrays["plude"].copy()
        # outputs on fresh, untouched pages
        for k in ca.OUTPUT_FIELDS:
            if k in st.arrays:
                st.arrays[k] = np.empty_like(st.arrays[k])
        f = st.fields()
        variant = ca.VARIANT_KCACHE if nproma <= 256 else ca.VARIANT_KSEG
        for i in range(a.calls):
            np.copyto(st.arrays["plude"], plude0)
            ca.check(lib.cloudsc_host_run_profile(1, None))
            ca.check(lib.cloudsc_host_run(0, ca.FP64, variant, ncols, nproma, ds.klev, C.byref(p), C.byref(f)))
            pr = Profile()
            ca.check(lib.cloudsc_host_run_profile(-1, C.byref(pr)))
            row = {"ncols": ncols, "nproma": nproma, "call": i + 1}
            row.update({n: round(getattr(pr, n), 4) for n, _ in Profile._fields_[1:] if n != "max_call_ms"})
            if pr.first_calls:   # the context's first call is counted apart
                row["total_ms"] = round(pr.first_calls_ms, 4)
            print(json.dumps(row), flush=True)
        worst = ca.validate_host_state(ds, st)
        print(json.dumps({"ncols": ncols, "nproma": nproma, "worst_rel_l1_vs_reference": worst}), flush=True)
        del st


if __name__ == "__main__":
    main()
