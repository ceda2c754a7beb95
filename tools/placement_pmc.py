#!/usr/bin/env python3
"""Counters of fast- and slow-placed states (companion of placement_fields.py).

Creates `--reps` states of one configuration (default placement), then runs
`--launches` KSEG steps of each state in turn, state 0 first.  Run it under
`rocprofv3 --pmc ... --kernel-trace`: the last reps x launches kseg_entry
dispatches belong to the states in that order, and their durations say which
replica is slow.  Prints one JSON line per state with the device addresses of
its fields (cloudsc_state_fields), for relating speed to address.
usage: placement_pmc.py [--precision fp64] [--reps 6] [--launches 5]"""
import argparse
import json
import os
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
    p.add_argument("--launches", type=int, default=5)
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    lib = ca.gpu_lib()
    ds = ca.load_dataset()
    states = [ca.GpuState(ds, a.ngptot, a.nproma, prec) for _ in range(a.reps)]
    try:
        for st in states:                       # warm every state, then the measured launches in order
            st.run(ca.VARIANT_KSEG, 3)
        for i, st in enumerate(states):
            ms = st.run(ca.VARIANT_KSEG, a.launches)
            f = ca.Fields()
            ca.check(lib.cloudsc_state_fields(st.h, ca.C.byref(f)))
            addr = {n: hex(getattr(f, n)) for n, _ in ca.Fields._fields_ if getattr(f, n)}
            print(json.dumps({"state": i, "ms": [round(float(x), 4) for x in ms], "addr": addr}), flush=True)
    finally:
        for st in states:
            st.close()


if __name__ == "__main__":
    main()
