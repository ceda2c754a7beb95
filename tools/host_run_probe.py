#!/usr/bin/env python3
"""Diagnostic: cloudsc_host_run (the per-call host-array entry point under the
GPU drop-in cloudsc_c) over a few (ngptot, nproma, variant) cases, each checked
against cloudsc_cpu_run on the same arrays; a native backtrace is printed if
the process faults (tools/segv_bt.c, loaded first).
usage: host_run_probe.py [ngptot:nproma:variant ...]"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
bt = os.path.join(REPO, "build", "libsegv_bt.so")
if os.path.exists(bt):
    C.CDLL(bt)
import cloudsc_amd as ca  # noqa: E402

cases = sys.argv[1:] or ["32:32:2", "32:32:3", "294:300:3", "300:300:3", "1000:64:3", "1000:300:3"]
lib = ca.gpu_lib()
ds = ca.load_dataset()
p = ca.Params.from_dict(ds.params)
for case in cases:
    ng, npr, var = (int(x) for x in case.split(":"))
    print("case ngptot=%d nproma=%d variant=%d" % (ng, npr, var), flush=True)
    a = ca.make_host_state(ds, ng, npr, ca.FP64)
    b = ca.make_host_state(ds, ng, npr, ca.FP64)
    ca.check(lib.cloudsc_cpu_run(1, ng, npr, ds.klev, C.byref(p), C.byref(b.fields()), None))
    rc = lib.cloudsc_host_run(0, ca.FP64, var, ng, npr, ds.klev, C.byref(p), C.byref(a.fields()))
    print("  rc", rc, ca.gpu_lib().cloudsc_last_hip_error(), flush=True)
    bad = [k for _, k in ca.VALIDATED
           if not np.array_equal(ca.blocks_to_columns(a.arrays[k], ng).view(np.uint64),
                                 ca.blocks_to_columns(b.arrays[k], ng).view(np.uint64))]
    print("  differs from cloudsc_cpu_run in", bad, flush=True)
