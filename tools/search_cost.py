#!/usr/bin/env python3
"""Wall time of a state's placement search, alternating library builds
(CLOUDSC_AMD_LIB-style paths on the command line): create a state with the
search on, report cloudsc_state_placement_report, destroy it; N rounds.
usage: search_cost.py [--rounds 3] lib0.so lib1.so ..."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    ds = ca.load_dataset()
    libs = []
    for p in a.libs:
        ca._lib = None
        libs.append(ca.gpu_lib(os.path.realpath(p)))
    for r in range(a.rounds):
        for p, lib in zip(a.libs, libs):
            ca._lib = lib
            t0 = time.perf_counter()
            g = ca.GpuState(ds, 163840, 64, ca.FP64)
            t1 = time.perf_counter()
            rep = g.placement_report()
            ms = g.run(ca.VARIANT_KSEG, 20)
            g.close()
            print(json.dumps({"round": r, "lib": os.path.basename(p), "create_s": round(t1 - t0, 3),
                              "kernel_ms_median": round(sorted(ms)[10], 4), **rep}), flush=True)


if __name__ == "__main__":
    main()
