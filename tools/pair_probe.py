#!/usr/bin/env python3
"""Does writing (and reading) two levels of a plane back to back move the
kernel's traffic faster than one level at a time?  (diagnostic, experiment
build with the paired probe: modes 2 / 3 of cloudsc_debug_memory_probe)

One state's own field buffers; modes 0 (write, one level per step), 1 (read +
write, one level), 2 (write, two levels per step), 3 (read + write, two
levels), interleaved over rounds; the state's KSEG kernel beside them."""
import ctypes as C
import os
import statistics as stt
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def main():
    lib = ca.gpu_lib()
    lib.cloudsc_debug_memory_probe.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                               C.c_int, C.POINTER(C.c_float)]
    ds = ca.load_dataset()
    res = {}
    for rep in range(2):
        g = ca.GpuState(ds, 163840, 64, ca.FP64)
        try:
            f = ca.Fields()
            ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
            for _ in range(15):
                for mode in (0, 1, 2, 3):
                    ms = C.c_float()
                    ca.check(lib.cloudsc_debug_memory_probe(0, ca.FP64, 163840, 64, ds.klev, C.byref(f), mode, 2,
                                                            C.byref(ms)))
                    res.setdefault((rep, mode), []).append(ms.value)
                res.setdefault((rep, "kernel"), []).append(g.run_span(ca.VARIANT_KSEG, 5) / 5)
        finally:
            g.close()
    for (rep, mode), v in sorted(res.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
        print("state %d %-7s median %.4f ms" % (rep, mode, stt.median(v)), flush=True)


if __name__ == "__main__":
    main()
