#!/usr/bin/env python3
"""Diagnostic: fraction of physics level-waves that execute each branch body
(build/libbranch_stats.so, built from tools/branch_stats.hip)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
os.environ["CLOUDSC_AMD_LIB"] = os.path.join(REPO, "build", "libbranch_stats.so")
import cloudsc_amd as ca  # noqa: E402
import make_fixtures as mf  # noqa: E402

NAMES = {0: "3.1 supersat", 1: "3.1 psupsat", 2: "3.4 erosion", 3: "3.4a evap cloud", 4: "3.4b1 cond existing",
         5: "3.4b2 new cloud (outer)", 6: "3.4b2 new cloud (inner)", 7: "3.7 deposition (exp+3 pow)",
         8: "4.2 precip cover", 9: "4.3a snow autoconv (2 exp)", 10: "4.3b warm rain (outer)",
         11: "4.3b KK (2 pow)", 12: "riming (2 pow)", 13: "4.4a melting", 14: "4.4b rain present",
         15: "4.4c freezing liquid", 16: "4.5 rain evap (6 pow)", 17: "4.5 snow evap (1 pow)"}

lib = ca.gpu_lib()
lib.cloudsc_branch_stats.argtypes = [C.c_void_p]
base = ca.load_dataset()
prev = [0] * 32
for name, ds in (("reference data", base), ("scenario W", mf.load_scenario("W", base)),
                 ("scenario M", mf.load_scenario("M", base))):
    g = ca.GpuState(ds, 163840, 128, ca.FP64)
    g.run(ca.VARIANT_KCACHE, 1)
    g.close()
    buf = (C.c_ulonglong * 32)()
    lib.cloudsc_branch_stats(buf)
    cur = list(buf)
    d = [a - b for a, b in zip(cur, prev)]
    prev = cur
    tot = d[31]
    print("== %s: %d physics level-waves" % (name, tot))
    for i in sorted(NAMES):
        print("  %-32s %6.3f" % (NAMES[i], d[i] / tot))
