#!/usr/bin/env python3
"""Kernel-boundary cost of the timed physics launches (diagnostic).

The bench's per-step time exceeds the kernel's own duration by ~9 us
(profiles/r02/experiment_kseg_epoch.txt).  This times `--reps` back-to-back
launches on one state in three forms, interleaved over `--rounds` rounds
(cloudsc_debug_launch_forms, debug builds only):
  0 events  -- the product form: each dispatch records its own event pair
  1 plain   -- the same dispatches without events
  2 graph   -- one hipGraph of the workspace reset and the `--reps` launches
and prints the median per-launch time of each form; the kernel's own median
duration (state_run's events) is printed beside them.

  python tools/exp_variant.py lf64 - -DCLOUDSC_DEBUG_LAUNCH_FORMS -DCLOUDSC_ONLY_KSEG=8
  CLOUDSC_AMD_LIB=build/liblf64.so python tools/launch_forms.py --precision fp64"""
import argparse
import ctypes as C
import os
import statistics as stt
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="fp64")
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--reps", type=int, default=100)
    p.add_argument("--rounds", type=int, default=8)
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    lib = ca.gpu_lib()
    lib.cloudsc_debug_launch_forms.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
    ds = ca.load_dataset()
    g = ca.GpuState(ds, a.ngptot, a.nproma, prec)
    try:
        res = {0: [], 1: [], 2: [], "kernel": []}
        for _ in range(a.rounds):
            for mode in (0, 1, 2):
                ms = C.c_double()
                ca.check(lib.cloudsc_debug_launch_forms(g.h, ca.VARIANT_KSEG, a.reps, mode, C.byref(ms)))
                res[mode].append(ms.value)
            res["kernel"].append(float(stt.median(g.run(ca.VARIANT_KSEG, a.reps))))
            print("round", {k: round(v[-1] * 1e3, 2) for k, v in res.items()}, "us", flush=True)
        k = stt.median(res["kernel"])
        for mode, name in ((0, "events"), (1, "plain"), (2, "graph")):
            m = stt.median(res[mode])
            print("%-7s %s  median %.4f ms per launch, %.2f us above the kernel's median duration %.4f ms"
                  % (name, a.precision, m, (m - k) * 1e3, k), flush=True)
    finally:
        g.close()


if __name__ == "__main__":
    main()
