#!/usr/bin/env python3
"""A few launches of the write-pattern probe (mode 1: the kernel's reads and
writes without the physics) on one state's buffers, for counter passes beside
the KSEG kernel's (tools/pmc_tlb.sh).  The state's placement search is off."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

lib = ca.gpu_lib()
lib.cloudsc_debug_memory_probe.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                           C.POINTER(C.c_float)]
ca.check(lib.cloudsc_set_placement_search(0))
ds = ca.load_dataset()
g = ca.GpuState(ds, 163840, 64, ca.FP64)
try:
    f = ca.Fields()
    ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
    ms = C.c_float()
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ca.check(lib.cloudsc_debug_memory_probe(0, ca.FP64, 163840, 64, ds.klev, C.byref(f), mode, 3, C.byref(ms)))
    print("probe mode %d: %.4f ms" % (mode, ms.value))
finally:
    g.close()
