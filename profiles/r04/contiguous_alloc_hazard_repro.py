"""Round-4 re-run of the round-3 contiguous-allocation reproducer (VERDICT r03,
next #1), on the current sources (parameter and reference uploads ordered with
the launches), against the ORACLE rather than against "run 0".

Needs the diagnostic library, which re-admits allocation flags:
    make -C dwarf-p-cloudsc_amd variant VFLAGS=-DCLOUDSC_DEBUG_KNOBS OUT=../build/libcloudsc_dbg.so
    CLOUDSC_AMD_LIB=build/libcloudsc_dbg.so python profiles/r04/contiguous_alloc_hazard_repro.py

Layout (stagger, flags): stagger -1 = one hipMalloc per field, >= 0 = one arena;
flags 4 = hipDeviceMallocContiguous.  Every layout step runs KSEG and KCACHE on
the same state.  fp64 is compared bit for bit with the oracle; fp32 (fast libm
default, tolerance-gated) bit for bit with the first fp32 run of its variant,
and by relL1 with the fp32 oracle.  For a differing field the columns and the
level range that differ are printed (the KSEG hand-off splits the levels at
NCLDTOP + 55 % / 50 % of the physics levels)."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cloudsc_amd as ca  # noqa: E402
import oracle  # noqa: E402

NG, NP = 3000, 64
lib = ca.gpu_lib()
lib.cloudsc_debug_set_state_layout.argtypes = [C.c_longlong, C.c_uint]
print("library:", os.environ.get("CLOUDSC_AMD_LIB", ca.LIB_PATH), " ".join(sys.argv[1:]), flush=True)
ds = ca.load_dataset()
VARS = (("KSEG", ca.VARIANT_KSEG), ("KCACHE", ca.VARIANT_KCACHE))


def run(prec, stagger, flags):
    ca.check(lib.cloudsc_debug_set_state_layout(stagger, flags))
    g = ca.GpuState(ds, NG, NP, prec)
    try:
        out = {}
        for name, v in VARS:
            g.run(v, 1)
            out[name] = g.outputs()
        return out
    finally:
        g.close()
        ca.check(lib.cloudsc_debug_set_state_layout(-1, 0))


def bits_differ(a, b):
    return [k for k in b if not np.array_equal(np.asarray(a[k]).view(np.uint8), np.asarray(b[k]).view(np.uint8))]


def where(a, b):
    d = np.asarray(a) != np.asarray(b)
    if d.ndim == 1:
        return "cols %d" % d.sum()
    lev = np.nonzero(d.reshape(-1, d.shape[-1]).any(axis=1))[0] % d.shape[-2]
    cols = np.nonzero(d.reshape(-1, d.shape[-1]).any(axis=0))[0]
    return "cols %d (%d..%d) levels %d..%d" % (len(cols), cols.min(), cols.max(), lev.min(), lev.max())


def rel(a, r):
    den = np.abs(r).sum()
    return float(np.abs(a - r).sum() / den) if den > 0 else float(np.abs(a - r).sum())


seq = [(-1, 0), (0, 0), (-1, 0), (4608, 0), (-1, 0), (-1, 4), (-1, 0), (-1, 0), (-1, 4), (0, 0), (-1, 0)]
bad = 0
ORDER = [ca.FP64, ca.FP32] if "--fp64-first" in sys.argv else [ca.FP32, ca.FP64]
for prec in ORDER:
    st, _ = oracle.run_oracle(ds, NG, NP, prec)
    ref = ca.state_outputs_to_template(st.arrays, NG)
    first = {}
    for lay in seq:
        out = run(prec, *lay)
        for name, _ in VARS:
            o = out[name]
            if prec == ca.FP64:
                diff = bits_differ(o, ref)
                extra = ""
            else:
                first.setdefault(name, o)
                diff = bits_differ(o, first[name])
                extra = " worst relL1 vs fp32 oracle %.2e" % max(rel(o[k], ref[k]) for k in ref)
            bad += bool(diff)
            base = "oracle" if prec == ca.FP64 else "first run"
            print("fp%d %-6s layout %-10s differs from %s in %s%s" % (8 * prec, name, lay, base, diff[:8], extra),
                  flush=True)
            for k in diff[:3]:
                print("    %-16s %s" % (k, where(o[k], ref[k] if prec == ca.FP64 else first[name][k])), flush=True)
print("RESULT: %d of %d runs differ" % (bad, 2 * 2 * len(seq)))
