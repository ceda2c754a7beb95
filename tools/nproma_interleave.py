#!/usr/bin/env python3
"""KSEG at several NPROMA on one box, interleaved (diagnostic): one placement-
searched state per (NPROMA, replica), then rounds of `--reps` timed launches
per state round-robin (cloudsc_state_run_span).  Median ms per launch per state.

  python tools/nproma_interleave.py --precision fp64 --nproma 64 128 256"""
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
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--nproma", type=int, nargs="+", default=[64, 128, 256])
    p.add_argument("--replicas", type=int, default=2)
    p.add_argument("--rounds", type=int, default=30)
    p.add_argument("--reps", type=int, default=10)
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    ds = ca.load_dataset()
    states = []
    for rep in range(a.replicas):
        for npr in a.nproma:
            g = ca.GpuState(ds, a.ngptot, npr, prec)
            states.append(((npr, rep), g, g.placement_report()))
            print("created nproma %d replica %d placement %s" % (npr, rep, states[-1][2]), flush=True)
    try:
        for _, g, _ in states:
            g.run_span(ca.VARIANT_KSEG, 40)
        res = {key: [] for key, _, _ in states}
        for r in range(a.rounds):
            for key, g, _ in states:
                res[key].append(g.run_span(ca.VARIANT_KSEG, a.reps) / a.reps)
            if r % 10 == 9:
                print("round", r + 1, flush=True)
        base = stt.median(res[states[0][0]])
        for key, _, rep in states:
            m = stt.median(res[key])
            print("%s nproma %4d replica %d  median %.4f ms  ratio %.4f  (placement first %.4f kept %.4f)"
                  % (a.precision, key[0], key[1], m, m / base, rep["probe_first_ms"], rep["probe_final_ms"]),
                  flush=True)
    finally:
        for _, g, _ in states:
            g.close()


if __name__ == "__main__":
    main()
