#!/usr/bin/env python3
"""Kernel time against the field layout in HBM (diagnostic, cloudsc_gpu_run_layout).

Builds the same workload (reference state expanded to --ngptot columns) in
three layouts, each in its own device memory:
  ref    the reference block layout, one allocation per field
  joint  the level inputs AND outputs of one (block, level) interleaved in one
         arena: [block][level][37 planes][nproma] (27 input planes: 17 fields +
         5 pclv + 5 tendency_tmp_cld; 10 output planes: plude, tendency_loc_t/q/a,
         pcovptot, 5 tendency_loc_cld); the 14 fluxes in a second arena
         [block][level+1][14][nproma]
  split  inputs and outputs in two arenas of 27 planes per level each (the
         output arena padded to the input stride so plude can be read and
         written in place)
paph and the surface fields stay in the reference layout.  The layouts are
launched round-robin (plude restored before every launch); reports the median
kernel time per layout and checks every output field of every layout against
the reference layout's, bit for bit.

usage: layout_experiment.py [--precision fp64] [--rounds 30] [--reps 2]"""
import argparse
import ctypes as C
import os
import statistics as stt
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

IN2 = ["pt", "pq", "tendency_tmp_t", "tendency_tmp_q", "tendency_tmp_a", "pvfl", "pvfi", "phrsw", "phrlw",
       "pvervel", "pap", "plu", "psnde", "pmfu", "pmfd", "pa", "psupsat"]
IN3 = ["pclv", "tendency_tmp_cld"]
OUT2 = ["plude", "tendency_loc_t", "tendency_loc_q", "tendency_loc_a", "pcovptot"]
OUT3 = ["tendency_loc_cld"]
FLUX = ["pfsqlf", "pfsqif", "pfcqnng", "pfcqlng", "pfsqrf", "pfsqsf", "pfcqrng", "pfcqsng", "pfsqltur", "pfsqitur",
        "pfplsl", "pfplsn", "pfhpsl", "pfhpsn"]


class Layout(C.Structure):
    _fields_ = [(n, C.c_longlong) for n in (
        "in_block in_level in_species in_species_block out_block out_level out_species out_species_block "
        "paph_block paph_level flux_block flux_level").split()]


def hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipFree.argtypes = [C.c_void_p]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipMemcpy2D.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int]
    h.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    h.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    h.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    h.hipEventSynchronize.argtypes = [C.c_void_p]
    h.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    return h


H2D, D2H, D2D = 1, 2, 3


class Dev:
    def __init__(self, H):
        self.H, self.ptrs = H, []

    def alloc(self, nbytes):
        p = C.c_void_p()
        if self.H.hipMalloc(C.byref(p), nbytes) != 0:
            raise RuntimeError("hipMalloc(%d)" % nbytes)
        self.ptrs.append(p.value)
        return p.value

    def upload(self, arr):
        a = np.ascontiguousarray(arr)
        p = self.alloc(a.nbytes)
        assert self.H.hipMemcpy(p, a.ctypes.data, a.nbytes, H2D) == 0
        return p

    def free(self):
        for p in self.ptrs:
            self.H.hipFree(p)
        self.ptrs = []


def build(kind, hs, dev, es):
    """device fields + layout (None = reference) + plude (pointer, pitch bytes)"""
    A = hs.arrays
    nb, kl, np_ = A["pt"].shape
    f = ca.Fields()
    for name in ("paph", "plsm", "ktype", "prainfrac_toprfz"):
        setattr(f, name, dev.upload(A[name]))
    if kind == "ref":
        for name, _ in ca.Fields._fields_:
            if getattr(f, name) is None and A.get(name) is not None:
                setattr(f, name, dev.upload(A[name]))
        return f, None, (f.plude, np_ * es)
    nin = len(IN2) + 5 * len(IN3)
    nout = len(OUT2) + 5 * len(OUT3)
    nf_in = nin + nout if kind == "joint" else nin
    real = A["pt"].dtype
    arena_in = np.zeros((nb, kl, nf_in, np_), dtype=real)
    slot = {}
    q = 0
    for name in IN2:
        arena_in[:, :, q, :] = A[name]; slot[name] = (0, q); q += 1
    for name in IN3:
        for m in range(5):
            arena_in[:, :, q + m, :] = A[name][:, m]
        slot[name] = (0, q); q += 5
    if kind == "joint":
        arena_out, oq, oidx = arena_in, q, 0
    else:
        arena_out, oq, oidx = np.zeros((nb, kl, nf_in, np_), dtype=real), 0, 1
    arena_out[:, :, oq, :] = A["plude"]
    slot["plude"] = (oidx, oq)
    oq += 1
    for name in OUT2[1:]:
        slot[name] = (oidx, oq); oq += 1
    slot["tendency_loc_cld"] = (oidx, oq); oq += 5
    bases = [dev.upload(arena_in)]
    if kind == "split":
        bases.append(dev.upload(arena_out))
    for name, (which, s) in slot.items():
        setattr(f, name, bases[which] + s * np_ * es)
    fx = dev.alloc(nb * (kl + 1) * len(FLUX) * np_ * es)
    for i, name in enumerate(FLUX):
        setattr(f, name, fx + i * np_ * es)
    L = Layout()
    L.in_block = L.out_block = L.in_species_block = L.out_species_block = kl * nf_in * np_
    L.in_level = L.out_level = nf_in * np_
    L.in_species = L.out_species = np_
    L.paph_block, L.paph_level = (kl + 1) * np_, np_
    L.flux_block, L.flux_level = (kl + 1) * len(FLUX) * np_, len(FLUX) * np_
    return f, L, (f.plude, nf_in * np_ * es)


def fetch(H, f, L, name, shape, es, real):
    """download one output field into the reference layout"""
    out = np.empty(shape, dtype=real)
    nb, np_ = shape[0], shape[-1]
    if L is None:
        assert H.hipMemcpy(out.ctypes.data, getattr(f, name), out.nbytes, D2H) == 0
        return out
    if name in FLUX:
        pitch, rows = L.flux_level * es, nb * shape[1]
        assert H.hipMemcpy2D(out.ctypes.data, np_ * es, getattr(f, name), pitch, np_ * es, rows, D2H) == 0
        return out
    pitch = L.out_level * es
    if name == "tendency_loc_cld":
        tmp = np.empty((nb, shape[2], 5, np_), dtype=real)
        # species planes are adjacent: one 2-D copy of 5*np_ wide rows
        assert H.hipMemcpy2D(tmp.ctypes.data, 5 * np_ * es, getattr(f, name), pitch, 5 * np_ * es,
                             nb * shape[2], D2H) == 0
        return np.ascontiguousarray(tmp.transpose(0, 2, 1, 3))
    assert H.hipMemcpy2D(out.ctypes.data, np_ * es, getattr(f, name), pitch, np_ * es, nb * shape[1], D2H) == 0
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--precision", default="fp64")
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--nproma", type=int, default=64)
    p.add_argument("--rounds", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--layouts", default="ref,joint,split")
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    es = 8 if prec == ca.FP64 else 4
    lib = ca.gpu_lib()
    lib.cloudsc_gpu_run_layout.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.POINTER(ca.Fields), C.POINTER(Layout), C.c_void_p]
    H = hip()
    ds = ca.load_dataset()
    params = ca.Params.from_dict(ds.params)
    ca.check(lib.cloudsc_gpu_init(0, C.byref(params)))
    hs = ca.make_host_state(ds, a.ngptot, a.nproma, prec)
    nb, kl, np_ = hs.arrays["pt"].shape
    dev = Dev(H)
    pristine = dev.upload(hs.arrays["plude"])
    ws = dev.alloc(max(lib.cloudsc_gpu_scratch_bytes(prec, ca.VARIANT_KSEG, a.ngptot, a.nproma, kl), 256))
    runs = []
    for r in range(a.reps):
        for kind in a.layouts.split(","):
            f, L, plude = build(kind, hs, dev, es)
            runs.append((kind, r, f, L, plude))
            print("built", kind, r, flush=True)
    e0, e1 = C.c_void_p(), C.c_void_p()
    H.hipEventCreate(C.byref(e0))
    H.hipEventCreate(C.byref(e1))
    ms = [[] for _ in runs]
    try:
        for rnd in range(a.warmup + a.rounds):
            order = range(len(runs)) if rnd % 2 == 0 else reversed(range(len(runs)))
            for i in order:
                kind, r, f, L, (pl, pitch) = runs[i]
                assert H.hipMemcpy2D(pl, pitch, pristine, np_ * es, np_ * es, nb * kl, D2D) == 0
                H.hipEventRecord(e0, None)
                ca.check(lib.cloudsc_gpu_run_layout(0, None, prec, ca.VARIANT_KSEG, a.ngptot, a.nproma, kl,
                                                    C.byref(f), C.byref(L) if L is not None else None, ws))
                H.hipEventRecord(e1, None)
                H.hipEventSynchronize(e1)
                ca.check(lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ws))
                t = C.c_float()
                H.hipEventElapsedTime(C.byref(t), e0, e1)
                if rnd >= a.warmup:
                    ms[i].append(t.value)
        # bit identity of every output against the reference layout (after a
        # final launch of each from the pristine plude)
        real = np.float64 if prec == ca.FP64 else np.float32
        outs = {}
        for i, (kind, r, f, L, (pl, pitch)) in enumerate(runs):
            assert H.hipMemcpy2D(pl, pitch, pristine, np_ * es, np_ * es, nb * kl, D2D) == 0
            ca.check(lib.cloudsc_gpu_run_layout(0, None, prec, ca.VARIANT_KSEG, a.ngptot, a.nproma, kl,
                                                C.byref(f), C.byref(L) if L is not None else None, ws))
            ca.check(lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ws))
            outs[i] = {name: fetch(H, f, L, name, hs.arrays[name].shape, es, real) for name in FLUX + OUT2 + OUT3}
        ref = next(i for i, x in enumerate(runs) if x[0] == "ref")
        for i, (kind, r, *_rest) in enumerate(runs):
            bad = [n for n in outs[i] if not np.array_equal(outs[i][n].view(np.uint8), outs[ref][n].view(np.uint8))]
            print("%-6s replica %d: median %.4f ms  min %.4f ms  outputs bit-identical to ref: %s" % (
                kind, r, stt.median(ms[i]), min(ms[i]), "yes" if not bad else "NO " + ",".join(bad)), flush=True)
    finally:
        dev.free()


if __name__ == "__main__":
    main()
