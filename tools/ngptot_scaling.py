#!/usr/bin/env python3
"""Time per column against the number of columns (diagnostic): how much of a
KSEG step is the schedule's last, partly filled round.  163,840 columns are
2,560 one-wave units on 2,048 resident waves (1.25 per wave); at 131,072 and
262,144 columns the ratio is a whole number.  One placement-searched state per
size, interleaved rounds of plain launches (cloudsc_state_run_span).

  python tools/ngptot_scaling.py --precision fp64"""
import argparse
import os
import statistics as stt
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="fp64")
    p.add_argument("--ngptot", type=int, nargs="+", default=[131072, 163840, 196608, 229376, 262144, 327680])
    p.add_argument("--nseg", type=int, nargs="+", default=[0])
    p.add_argument("--rounds", type=int, default=20)
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    ds = ca.load_dataset()
    states = [(n, ca.GpuState(ds, n, 64, prec)) for n in a.ngptot]
    try:
        res = {(n, s): [] for n, _ in states for s in a.nseg}
        for _ in range(a.rounds):
            for s in a.nseg:
                ca.kseg_schedule(s, 0)
                for n, g in states:
                    res[(n, s)].append(g.run_span(ca.VARIANT_KSEG, 10) / 10)
        ca.kseg_schedule(0, 0)
        for (n, s), v in sorted(res.items()):
            m = stt.median(v)
            print("%s ngptot %7d (%.3f units per wave) nseg %s: %.4f ms, %.3f ns per column" % (
                a.precision, n, n / 64 / 2048, s or "default", m, m * 1e6 / n), flush=True)
    finally:
        for _, g in states:
            g.close()


if __name__ == "__main__":
    main()
