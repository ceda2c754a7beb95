#!/usr/bin/env python3
"""Stress of the KSEG carried-state hand-off across launches (diagnostic).

Two states hold DIFFERENT inputs (B = A with its columns rotated by half the
template, so every block carries other values between its segments).  Both
run through cloudsc_gpu_run on ONE shared KSEG workspace, alternately, so the
carried-state slots always hold the other state's values from the previous
launch: a consumer that reads its block's slot before the producer's values
are visible to it reads the other state's numbers, and the outputs of its
segment differ.  Every launch's pcovptot and pfplsl are compared bit for bit
with that state's reference (two launches on fresh workspaces, which must
agree); the count of launches and blocks that differ is printed.

usage: handoff_stress.py [--lib path] [--precision fp32] [--ngptot 3000] [--iters 400]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import cloudsc_amd as ca  # noqa: E402
from ab_interleave import hip, ok  # noqa: E402

FIELDS = ("pcovptot", "pfplsl")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None)
    p.add_argument("--precision", default="fp32")
    p.add_argument("--ngptot", type=int, default=3000)
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--iters", type=int, default=400)
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    esz = 8 if prec == ca.FP64 else 4
    lib = ca.gpu_lib(os.path.realpath(a.lib) if a.lib else None)
    H = hip()
    ds_a = ca.load_dataset()
    ds_b = ds_a.copy()
    for k, v in ds_b.inputs.items():
        if v.ndim >= 1 and v.shape[-1] == ds_a.klon:
            ds_b.inputs[k] = np.ascontiguousarray(np.roll(v, ds_a.klon // 2, axis=-1))
    states = [ca.GpuState(d, a.ngptot, a.nproma, prec) for d in (ds_a, ds_b)]
    fl = []
    for st in states:
        f = ca.Fields()
        ca.check(lib.cloudsc_state_fields(st.h, C.byref(f)))
        fl.append(f)
    params = ca.Params.from_dict(ds_a.params)
    ca.check(lib.cloudsc_gpu_init(0, C.byref(params)))
    nb = ca.nblocks_of(a.ngptot, a.nproma)
    klev = ds_a.klev
    fbytes = {n: nb * int(np.prod(ca.field_shape(ca.ALL_FIELDS[n], klev, a.nproma))) * esz for n in FIELDS}
    plude_bytes = nb * a.nproma * klev * esz
    nbytes = lib.cloudsc_gpu_scratch_bytes(prec, ca.VARIANT_KSEG, a.ngptot, a.nproma, klev)
    bufs = []

    def dmalloc(n):
        d = C.c_void_p()
        ok(H.hipMalloc(C.byref(d), n), "hipMalloc")
        bufs.append(d)
        return d

    pristine = []
    for f in fl:
        d = dmalloc(plude_bytes)
        ok(H.hipMemcpy(d, f.plude, plude_bytes, 3), "hipMemcpy")
        pristine.append(d)

    def launch(i, ws):
        ok(H.hipMemcpy(fl[i].plude, pristine[i], plude_bytes, 3), "hipMemcpy")
        ca.check(lib.cloudsc_gpu_run(0, None, prec, ca.VARIANT_KSEG, a.ngptot, a.nproma, klev,
                                     C.byref(fl[i]), ws))
        ca.check(lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ws))
        out = []
        for name in FIELDS:
            h = np.empty(fbytes[name], dtype=np.uint8)
            ok(H.hipMemcpy(h.ctypes.data, getattr(fl[i], name), fbytes[name], 2), "hipMemcpy D2H")
            out.append(h.view(np.uint32 if esz == 4 else np.uint64).reshape(nb, -1))
        return out

    try:
        refs = []
        for i in range(2):
            r = [launch(i, dmalloc(max(nbytes, 256))) for _ in range(2)]
            assert all((x == y).all() for x, y in zip(r[0], r[1])), "reference launches disagree"
            refs.append(r[0])
        assert not (refs[0][0] == refs[1][0]).all(), "the two states compute the same values"
        ws = dmalloc(max(nbytes, 256))
        bad_launches, bad_blocks = 0, 0
        for it in range(a.iters):
            i = it & 1
            out = launch(i, ws)
            blocks = set()
            for o, r in zip(out, refs[i]):
                blocks |= set(np.nonzero((o != r).any(axis=1))[0].tolist())
            if blocks:
                bad_launches += 1
                bad_blocks += len(blocks)
                print("launch %d (state %d): %d block(s) differ: %s" % (it, i, len(blocks), sorted(blocks)[:8]),
                      flush=True)
            if it % 200 == 199:
                print("... %d launches, %d differing" % (it + 1, bad_launches), flush=True)
        print('{"lib": "%s", "precision": "%s", "ngptot": %d, "iters": %d, "bad_launches": %d, "bad_blocks": %d}'
              % (os.path.basename(a.lib or ca.LIB_PATH), a.precision, a.ngptot, a.iters, bad_launches, bad_blocks),
              flush=True)
    finally:
        for d in bufs:
            H.hipFree(d)
        for st in states:
            st.close()


if __name__ == "__main__":
    main()
