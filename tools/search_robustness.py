#!/usr/bin/env python3
"""How often does a state stay slow after its placement search?  (diagnostic)

Creates `--states` fp64 KSEG states (NPROMA cycling 64/128/256 by default, as
in the run where one stayed at 1.95 ms), all kept alive, and times each with
20 plain launches (best of 3).  Prints each state's time, its search report,
and the count of states slower than 1.07x the fastest.  Run it with different
builds (CLOUDSC_AMD_LIB) to compare search strategies."""
import argparse
import os
import statistics as stt
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--states", type=int, default=16)
    p.add_argument("--nproma", type=int, nargs="+", default=[64, 128, 256])
    p.add_argument("--passes", type=int, default=-1, help="field passes of the search (-1: the library's default)")
    a = p.parse_args()
    ca.check(ca.gpu_lib().cloudsc_set_placement_search(a.passes))
    ds = ca.load_dataset()
    states, times = [], []
    try:
        for i in range(a.states):
            npr = a.nproma[i % len(a.nproma)]
            g = ca.GpuState(ds, 163840, npr, ca.FP64)
            states.append(g)
            g.run_span(ca.VARIANT_KSEG, 5)
            t = min(g.run_span(ca.VARIANT_KSEG, 20) / 20 for _ in range(3))
            times.append(t)
            r = g.placement_report()
            print("state %2d nproma %3d: %.4f ms  (first %.4f kept %.4f tries %d moves %d launches %d search %.0f ms "
                  "peak %.1f GB)" % (i, npr, t, r["probe_first_ms"], r["probe_final_ms"], r["tries"], r["moves"],
                                     r["launches"], r["search_ms"], r["peak_transient_bytes"] / 1e9), flush=True)
        lo = min(times)
        slow = [i for i, t in enumerate(times) if t > 1.07 * lo]
        print("lib %s passes %d: %d states, fastest %.4f, median %.4f, slowest %.4f, > 1.07x fastest: %d %s"
              % (os.path.basename(os.environ.get("CLOUDSC_AMD_LIB", ca.LIB_PATH)), a.passes, len(times), lo,
                 stt.median(times), max(times), len(slow), slow), flush=True)
    finally:
        for g in states:
            g.close()


if __name__ == "__main__":
    main()
