#!/usr/bin/env python3
"""Kernel time against the HBM placement of a state's fields (diagnostic).

For each layout (cloudsc_debug_set_state_layout: -1 = one hipMalloc per field,
s >= 0 = one arena, field i at a 2 MiB boundary + (i*s) mod 2 MiB) it creates
`--reps` states, then launches all states round-robin, one step each per
round (so clock drift hits every state alike), and reports per layout the
median kernel time of each replica and over all of them.

A layout is stagger[:alloc_flags]; the library now refuses alloc_flags != 0
(profiles/r03/contiguous_alloc_hazard.txt), the form stays for the records of
experiment_field_placement.txt.

usage: ab_layout.py [--precision fp64] [--reps 2] [--rounds 40] layout [layout ...]"""
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
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--rounds", type=int, default=40)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("staggers", nargs="+", help="stagger[:alloc_flags]")
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    lib = ca.gpu_lib()
    lib.cloudsc_debug_set_state_layout.argtypes = [C.c_longlong, C.c_uint]
    ds = ca.load_dataset()
    states = []
    for r in range(a.reps):
        for s in a.staggers:
            st, _, fl = s.partition(":")
            ca.check(lib.cloudsc_debug_set_state_layout(int(st), int(fl or 0)))
            try:
                states.append((s, r, ca.GpuState(ds, a.ngptot, a.nproma, prec)))
            except ca.CloudscError as e:
                print("layout %s replica %d: state creation failed (%s)" % (s, r, e), flush=True)
    ca.check(lib.cloudsc_debug_set_state_layout(-1, 0))
    ms = [[] for _ in states]
    try:
        for rnd in range(a.warmup + a.rounds):
            order = range(len(states)) if rnd % 2 == 0 else reversed(range(len(states)))
            for i in order:
                t = float(states[i][2].run(ca.VARIANT_KSEG, 1)[0])
                if rnd >= a.warmup:
                    ms[i].append(t)
    finally:
        for _, _, st in states:
            st.close()
    ref = stt.median(ms[0])
    for s in a.staggers:
        per = [stt.median(m) for (sx, _, _), m in zip(states, ms) if sx == s]
        if not per:
            continue
        print("layout %-12s replicas %s  mean %.4f ms  (x%.4f of the first replica of the first layout)" % (
            s, " ".join("%.4f" % x for x in per), sum(per) / len(per), sum(per) / len(per) / ref), flush=True)


if __name__ == "__main__":
    main()
