#!/usr/bin/env python3
"""Same-process A/B timing of several builds of libcloudsc_amd.so (diagnostic).

All builds run on the SAME device buffers: one state (built with the first
library) holds the fields, one hipMalloc'ed KSEG workspace is shared, and each
library's cloudsc_gpu_run is launched on them round-robin, one step per
library per round, with plude restored from a pristine copy before every
launch (cloudsc_gpu_run updates it in place).  Two states of the same build
differ by up to 4 % in kernel time through their memory placement alone
(profiles/r03/experiment_ab_method.txt), and a box's clock drifts by several
per cent within a call: sharing the buffers removes the first, interleaving
the second.  Kernel time = HIP events around each cloudsc_gpu_run on the null
stream (includes the ~5 us KSEG prepare kernel, the same for every build).

usage: ab_interleave.py [--precision fp64] [--variant kseg] [--nproma 64]
                        [--rounds 60] lib0.so lib1.so ..."""
import argparse
import ctypes as C
import os
import statistics as stt
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipFree.argtypes = [C.c_void_p]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    h.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    h.hipEventSynchronize.argtypes = [C.c_void_p]
    h.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    return h


def ok(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: %d" % (what, rc))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="fp64")
    p.add_argument("--variant", default="kseg")
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--rounds", type=int, default=60)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--schedule", action="append", default=[],
                   help="IDX:NSEG:GRID -- cloudsc_debug_set_kseg_schedule(NSEG, GRID) on library IDX (0-based; "
                        "0 = the library's default); repeatable")
    p.add_argument("libs", nargs="+")
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    variant = {"kseg": ca.VARIANT_KSEG, "kcache": ca.VARIANT_KCACHE}[a.variant]
    ds = ca.load_dataset()
    H = hip()
    libs = []
    for path in a.libs:
        ca._lib = None
        libs.append(ca.gpu_lib(os.path.realpath(path)))
    ca._lib = libs[0]
    st = ca.GpuState(ds, a.ngptot, a.nproma, prec)
    f = ca.Fields()
    ca.check(libs[0].cloudsc_state_fields(st.h, C.byref(f)))
    params = ca.Params.from_dict(ds.params)
    for lib in libs:
        ca.check(lib.cloudsc_gpu_init(0, C.byref(params)))
    for spec in a.schedule:
        idx, nseg, grid = (int(x) for x in spec.split(":"))
        ca.check(libs[idx].cloudsc_debug_set_kseg_schedule(nseg, grid))
    nbytes = max(lib.cloudsc_gpu_scratch_bytes(prec, variant, a.ngptot, a.nproma, ds.klev) for lib in libs)
    ws, pristine = C.c_void_p(), C.c_void_p()
    plude_bytes = a.ngptot // a.nproma * a.nproma + (a.nproma if a.ngptot % a.nproma else 0)
    plude_bytes *= ds.klev * (8 if prec == ca.FP64 else 4)
    ok(H.hipMalloc(C.byref(ws), max(nbytes, 256)), "hipMalloc(ws)")
    ok(H.hipMalloc(C.byref(pristine), plude_bytes), "hipMalloc(plude)")
    ok(H.hipMemcpy(pristine, f.plude, plude_bytes, 3), "hipMemcpy")
    e0, e1 = C.c_void_p(), C.c_void_p()
    H.hipEventCreate(C.byref(e0))
    H.hipEventCreate(C.byref(e1))
    ms = [[] for _ in libs]
    try:
        for r in range(a.warmup + a.rounds):
            order = list(range(len(libs))) if r % 2 == 0 else list(reversed(range(len(libs))))
            for i in order:
                ok(H.hipMemcpy(f.plude, pristine, plude_bytes, 3), "hipMemcpy")
                H.hipEventRecord(e0, None)
                ca.check(libs[i].cloudsc_gpu_run(0, None, prec, variant, a.ngptot, a.nproma, ds.klev,
                                                 C.byref(f), ws))
                H.hipEventRecord(e1, None)
                H.hipEventSynchronize(e1)
                ca.check(libs[i].cloudsc_gpu_check(0, None, variant, ws))
                t = C.c_float()
                H.hipEventElapsedTime(C.byref(t), e0, e1)
                if r >= a.warmup:
                    ms[i].append(t.value)
    finally:
        H.hipFree(ws)
        H.hipFree(pristine)
        st.close()
    base = ms[0]
    for path, m in zip(a.libs, ms):
        ratio = stt.median(x / y for x, y in zip(m, base))
        q = stt.quantiles(m, n=10)
        print("%-34s median %.4f ms  min %.4f ms  p10 %.4f  p90 %.4f  ratio-to-first %.4f" % (
            os.path.basename(path), stt.median(m), min(m), q[0], q[-1], ratio), flush=True)


if __name__ == "__main__":
    main()
