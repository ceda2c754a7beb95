#!/usr/bin/env python3
"""Same-process A/B of kernel CONFIGURATIONS of the diagnostic build (round 6).

One diagnostic library (-DCLOUDSC_DEBUG_KNOBS), one state's fields, one shared
KSEG workspace; each combination `cfg:grid:nseg` (CLOUDSC_KCACHE_CFG,
CLOUDSC_KSEG_GRID, CLOUDSC_KSEG_NSEG; grid 0 = the library's choice) is set in
the environment before its launch -- the diagnostic build reads it at every
launch -- and the combinations run round-robin, plude restored before each
launch.  After the timing, every combination's 21 outputs are compared bit for
bit with the first one's (SHA-256 of each field).

usage: cfg_interleave.py [--precision fp64] [--rounds 30] cfg:grid:nseg ...
  (CLOUDSC_AMD_LIB must name the diagnostic build)"""
import argparse
import ctypes as C
import hashlib
import json
import os
import statistics as stt
import sys


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import cloudsc_amd as ca  # noqa: E402
from ab_interleave import hip, ok  # noqa: E402


def set_combo(c):
    cfg, grid, nseg = c.split(":")
    os.environ["CLOUDSC_KCACHE_CFG"] = cfg
    os.environ["CLOUDSC_KSEG_GRID"] = grid
    os.environ["CLOUDSC_KSEG_NSEG"] = nseg


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="fp64")
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--rounds", type=int, default=30)
    p.add_argument("--warmup", type=int, default=6)
    p.add_argument("combos", nargs="+")
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    variant = ca.VARIANT_KSEG
    ds = ca.load_dataset()
    H = hip()
    lib = ca.gpu_lib()
    st = ca.GpuState(ds, a.ngptot, a.nproma, prec)
    f = ca.Fields()
    ca.check(lib.cloudsc_state_fields(st.h, C.byref(f)))
    params = ca.Params.from_dict(ds.params)
    ca.check(lib.cloudsc_gpu_init(0, C.byref(params)))
    nbytes = lib.cloudsc_gpu_scratch_bytes(prec, variant, a.ngptot, a.nproma, ds.klev)
    es = 8 if prec == ca.FP64 else 4
    nblocks = (a.ngptot + a.nproma - 1) // a.nproma
    plude_bytes = nblocks * a.nproma * ds.klev * es
    ws, pristine = C.c_void_p(), C.c_void_p()
    ok(H.hipMalloc(C.byref(ws), max(nbytes, 256)), "hipMalloc(ws)")
    ok(H.hipMalloc(C.byref(pristine), plude_bytes), "hipMalloc(plude)")
    ok(H.hipMemcpy(pristine, f.plude, plude_bytes, 3), "hipMemcpy")
    e0, e1 = C.c_void_p(), C.c_void_p()
    H.hipEventCreate(C.byref(e0))
    H.hipEventCreate(C.byref(e1))

    def launch(c):
        set_combo(c)
        ok(H.hipMemcpy(f.plude, pristine, plude_bytes, 3), "hipMemcpy")
        H.hipEventRecord(e0, None)
        ca.check(lib.cloudsc_gpu_run(0, None, prec, variant, a.ngptot, a.nproma, ds.klev, C.byref(f), ws))
        H.hipEventRecord(e1, None)
        H.hipEventSynchronize(e1)
        ca.check(lib.cloudsc_gpu_check(0, None, variant, ws))
        t = C.c_float()
        H.hipEventElapsedTime(C.byref(t), e0, e1)
        return t.value

    def digest():
        return {k: hashlib.sha256(st.download(k).tobytes()).hexdigest()[:16] for _, k in ca.VALIDATED}

    ms = {c: [] for c in a.combos}
    try:
        for r in range(a.warmup + a.rounds):
            order = a.combos if r % 2 == 0 else list(reversed(a.combos))
            for c in order:
                t = launch(c)
                if r >= a.warmup:
                    ms[c].append(t)
        hashes = {}
        for c in a.combos:
            launch(c)
            hashes[c] = digest()
    finally:
        H.hipFree(ws)
        H.hipFree(pristine)
        st.close()
    base = ms[a.combos[0]]
    for c in a.combos:
        m = ms[c]
        diff = [k for k in hashes[c] if hashes[c][k] != hashes[a.combos[0]][k]]
        print(json.dumps({"combo": c, "precision": a.precision, "median_ms": round(stt.median(m), 4),
                          "min_ms": round(min(m), 4), "ratio_to_first": round(stt.median(x / y for x, y in zip(m, base)), 4),
                          "fields_differing_from_first": diff}), flush=True)


if __name__ == "__main__":
    main()
