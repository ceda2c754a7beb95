#!/usr/bin/env python3
"""A/B of the output placement search (cloudsc_state_placement): `--reps`
states created with the search off and `--reps` with it on (alternating), all
launched round-robin (order reversed every other round); per state the median
KSEG time and the search's record, then the spread of each group.
usage: placement_search_ab.py [--precision fp64] [--reps 6] [--rounds 30]"""
import argparse
import json
import os
import statistics as stt
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="fp64")
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--reps", type=int, default=6)
    p.add_argument("--rounds", type=int, default=30)
    p.add_argument("--warmup", type=int, default=15)
    p.add_argument("--passes", type=int, default=-1, help="search passes of the 'on' group (-1: default)")
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    lib = ca.gpu_lib()
    ds = ca.load_dataset()
    states = []
    try:
        for r in range(a.reps):
            for on in (False, True):
                ca.check(lib.cloudsc_debug_set_placement_search(a.passes if on else 0))
                states.append((on, ca.GpuState(ds, a.ngptot, a.nproma, prec)))
        ca.check(lib.cloudsc_debug_set_placement_search(-1))
        ms = [[] for _ in states]
        for rnd in range(a.warmup + a.rounds):
            order = range(len(states)) if rnd % 2 == 0 else reversed(range(len(states)))
            for i in order:
                t = float(states[i][1].run(ca.VARIANT_KSEG, 1)[0])
                if rnd >= a.warmup:
                    ms[i].append(t)
        med = [stt.median(m) for m in ms]
        for (on, st), m in zip(states, med):
            print(json.dumps({"precision": a.precision, "search": on, "kernel_ms": round(m, 4), **st.placement()}),
                  flush=True)
        for on in (False, True):
            g = [m for (o, _), m in zip(states, med) if o == on]
            print(json.dumps({"precision": a.precision, "search": on, "states": len(g),
                              "median_ms": round(stt.median(g), 4), "min_ms": round(min(g), 4),
                              "max_ms": round(max(g), 4), "spread": round(max(g) / min(g) - 1, 4)}), flush=True)
    finally:
        for _, st in states:
            st.close()


if __name__ == "__main__":
    main()
