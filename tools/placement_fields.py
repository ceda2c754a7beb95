#!/usr/bin/env python3
"""Which fields' HBM placement decides the KSEG kernel time.

1. `--reps` states of the same configuration and the default placement (one
   hipMalloc per field) are launched round-robin (one step each per round, the
   order reversed every other round, so clock drift hits all alike); the median
   of each replica gives the placement spread.
2. The slowest replica is then walked field by field: each field in turn is
   moved to a fresh allocation (cloudsc_debug_state_relocate_field -- a device
   copy onto other physical pages; earlier moves are kept), and after every move
   the slow state is timed against the fastest replica (the control), again
   interleaved.  A field whose move changes the slow/fast ratio by more than the
   noise names itself; `--reroll` further passes move EVERY field at once and
   show whether a fresh placement of all fields lands anywhere in the spread.

One JSON line per measurement.
usage: placement_fields.py [--precision fp64] [--reps 6] [--rounds 20] [--reroll 3]"""
import argparse
import ctypes as C
import json
import os
import statistics as stt
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def interleaved(states, rounds, variant=ca.VARIANT_KSEG):
    ms = [[] for _ in states]
    for rnd in range(rounds):
        order = range(len(states)) if rnd % 2 == 0 else reversed(range(len(states)))
        for i in order:
            ms[i].append(float(states[i].run(variant, 1)[0]))
    return [stt.median(m) for m in ms]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="fp64")
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--reps", type=int, default=6)
    p.add_argument("--rounds", type=int, default=20)
    p.add_argument("--warmup", type=int, default=15)
    p.add_argument("--reroll", type=int, default=3)
    p.add_argument("--search", type=int, default=0, help="placement search passes at creation (0: off)")
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    lib = ca.gpu_lib()
    lib.cloudsc_debug_state_relocate_field.argtypes = [C.c_void_p, C.c_int]
    ds = ca.load_dataset()
    ca.check(lib.cloudsc_debug_set_placement_search(a.search))
    states = [ca.GpuState(ds, a.ngptot, a.nproma, prec) for _ in range(a.reps)]
    ca.check(lib.cloudsc_debug_set_placement_search(-1))
    names = [n for n, _ in ca.Fields._fields_]
    try:
        interleaved(states, a.warmup)
        med = interleaved(states, 2 * a.rounds)
        print(json.dumps({"precision": a.precision, "phase": "replicas", "ms": [round(x, 4) for x in med],
                          "spread": round(max(med) / min(med) - 1, 4)}), flush=True)
        slow, fast = med.index(max(med)), med.index(min(med))
        pair = [states[slow], states[fast]]

        def ratio():
            m = interleaved(pair, a.rounds)
            return m[0], m[1], m[0] / m[1]

        s0, f0, r0 = ratio()
        print(json.dumps({"phase": "start", "slow_ms": round(s0, 4), "fast_ms": round(f0, 4),
                          "ratio": round(r0, 4)}), flush=True)
        prev = r0
        for i, n in enumerate(names):
            if lib.cloudsc_debug_state_relocate_field(states[slow].h, i) != 0:
                continue                     # a field this state does not hold
            s, f, r = ratio()
            print(json.dumps({"phase": "move", "field": n, "slow_ms": round(s, 4), "fast_ms": round(f, 4),
                              "ratio": round(r, 4), "step": round(r / prev - 1, 4)}), flush=True)
            prev = r
        for k in range(a.reroll):
            for i in range(len(names)):
                lib.cloudsc_debug_state_relocate_field(states[slow].h, i)
            s, f, r = ratio()
            print(json.dumps({"phase": "reroll", "pass": k, "slow_ms": round(s, 4), "fast_ms": round(f, 4),
                              "ratio": round(r, 4)}), flush=True)
        # the moved state still computes the same bits as the control
        a_out, b_out = states[slow].outputs(), states[fast].outputs()
        same = all(np.array_equal(a_out[k].view(np.uint64), b_out[k].view(np.uint64)) for k in a_out)
        print(json.dumps({"phase": "check", "outputs_bitwise_equal": bool(same)}), flush=True)
    finally:
        for st in states:
            st.close()


if __name__ == "__main__":
    main()
