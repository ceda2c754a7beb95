#!/usr/bin/env python3
"""Why is a state slow in every placement?  (diagnostic, round 5)

In tools/nproma_interleave.py's run one state of six (fp64, NPROMA 256, the last
created) probed 1.95 ms at creation and none of the search's 293 candidates
(8 output sets, 21 single fields, 4 input sets) was 1 % faster, while its
siblings ran 1.65-1.71 ms (profiles/r05/kseg_nproma_interleaved.txt); the
driver's round-4 box had one such state too.  This creates
states in the same order (NPROMA 64, 128, 256, twice, then more), all kept
alive, times each (20 plain launches), and for a state slower than 1.07x the
fastest so far moves, one at a time, the buffers the search never moves (the
KSEG workspace, the pristine plude copy), then every input field, then every
output field (cloudsc_debug_state_relocate_aux / _field), timing after each
move.  Free device memory is printed at each creation."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

NAMES = [f[0] for f in ca.Fields._fields_]


def free_gib():
    hip = C.CDLL("libamdhip64.so")
    fr, tot = C.c_size_t(), C.c_size_t()
    hip.hipMemGetInfo(C.byref(fr), C.byref(tot))
    return fr.value / 2**30


def t_of(g, n=20):
    g.run_span(ca.VARIANT_KSEG, 5)
    return min(g.run_span(ca.VARIANT_KSEG, n) / n for _ in range(3))


def main():
    prec = ca.FP64
    lib = ca.gpu_lib()
    lib.cloudsc_debug_state_relocate_aux.argtypes = [C.c_void_p, C.c_int]
    lib.cloudsc_debug_state_relocate_field.argtypes = [C.c_void_p, C.c_int]
    ds = ca.load_dataset()
    order = [64, 128, 256, 64, 128, 256, 64, 128, 256, 64]
    states, best, diagnosed = [], None, 0
    try:
        for i, npr in enumerate(order):
            g = ca.GpuState(ds, 163840, npr, prec)
            states.append(g)
            rep = g.placement_report()
            t = t_of(g)
            best = t if best is None else min(best, t)
            print("state %d nproma %d: %.4f ms (placement first %.4f kept %.4f tries %d moves %d launches %d "
                  "search %.0f ms); free %.1f GiB" % (i, npr, t, rep["probe_first_ms"], rep["probe_final_ms"],
                                                     rep["tries"], rep["moves"], rep["launches"], rep["search_ms"],
                                                     free_gib()), flush=True)
            if t < 1.07 * best or diagnosed >= 2:
                continue
            diagnosed += 1
            print("  slow state %d: moving buffers one at a time" % i, flush=True)
            for which, name in ((1, "KSEG workspace"), (0, "pristine plude")):
                ca.check(lib.cloudsc_debug_state_relocate_aux(g.h, which))
                print("    after moving %-16s %.4f ms" % (name, t_of(g)), flush=True)
            f = ca.Fields()
            ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
            for group, names in (("input", list(ca.INPUT_FIELDS) + ["plude"]), ("output", list(ca.OUTPUT_FIELDS))):
                for name in names:
                    if name not in NAMES or not getattr(f, name):
                        continue
                    ca.check(lib.cloudsc_debug_state_relocate_field(g.h, NAMES.index(name)))
                    print("    after moving %s %-18s %.4f ms" % (group, name, t_of(g)), flush=True)
            # all the others destroyed: does a new state come out fast?
        for g in states[:-1]:
            g.close()
        states = states[-1:]
        print("free after closing all but the last: %.1f GiB" % free_gib(), flush=True)
        g = ca.GpuState(ds, 163840, 64, prec)
        states.append(g)
        rep = g.placement_report()
        print("new nproma-64 state alone: %.4f ms (placement first %.4f kept %.4f)"
              % (t_of(g), rep["probe_first_ms"], rep["probe_final_ms"]), flush=True)
    finally:
        for g in states:
            g.close()


if __name__ == "__main__":
    main()
