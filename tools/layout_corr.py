#!/usr/bin/env python3
"""Round-6 layout study: does an interleaved HBM layout take
the fields out of the placement lottery?

Instrument: the memory-pattern probe of cloudsc_place.hip (the KSEG kernel's
loads and stores, no physics) in its read+write form, which ranks placements
like the kernel (Pearson 0.986 / Spearman 0.988 over 10 states with the
write-through store policy, profiles/r06/place_corr_sc1_fp64.jsonl), run over
field sets in three layouts through cloudsc_debug_memory_probe_layout:

  P  the reference layout: one buffer per field (cloudsc_fields_alloc, no search)
  B  per-block interleave: one input arena and one output arena, each block's
     chunks of every field side by side ([block][field][rows][nproma])
  I  per-row interleave: one input arena [block][row][planes][nproma] (a
     wave-level's input loads are one contiguous run) and one output arena the
     same way, the half-level fluxes shifted one row down so that a level's
     24 output stores are ONE contiguous 12 KiB run

NSETS fresh sets per layout, allocated alternately, timed round-robin over
ROUNDS (median per set); per layout the median set, fastest, slowest, spread.
A layout is placement-free if its spread stays within the probe's noise (~1-2 %)
and it is only worth adopting if its median is no slower than the fastest sets
of P (what the placement search finds).

usage (GPU box): python tools/layout_corr.py [--sets 6] [--rounds 8] [--layouts P,B,I]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

# the probe's fields (cloudsc_place.hip probe_args)
IN_LEVEL = ["pt", "pq", "tendency_tmp_t", "tendency_tmp_q", "tendency_tmp_a", "pvfl", "pvfi", "phrsw", "phrlw",
            "pvervel", "pap", "plu", "psnde", "pmfu", "pmfd", "pa", "psupsat"]
IN_SPECIES = ["tendency_tmp_cld", "pclv"]
IN_HALF = ["paph"]
OUT_LEVEL = ["plude", "tendency_loc_t", "tendency_loc_q", "tendency_loc_a", "pcovptot"]
OUT_SPECIES = ["tendency_loc_cld"]
OUT_HALF = ["pfsqlf", "pfsqif", "pfcqnng", "pfcqlng", "pfsqrf", "pfsqsf", "pfcqrng", "pfcqsng", "pfsqltur",
            "pfsqitur", "pfplsl", "pfplsn", "pfhpsl", "pfhpsn"]


class Hip:
    def __init__(self):
        h = C.CDLL("libamdhip64.so")
        h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        h.hipFree.argtypes = [C.c_void_p]
        h.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        self.h = h

    def alloc(self, nbytes):
        p = C.c_void_p()
        rc = self.h.hipMalloc(C.byref(p), nbytes)
        if rc != 0:
            raise RuntimeError("hipMalloc(%d) failed: %d" % (nbytes, rc))
        assert self.h.hipMemset(p, 0, nbytes) == 0
        return p.value


def arena_set(hip, layout, nblocks, nproma, klev, es):
    """Field pointers and strides of one B or I set; returns (Fields, strides, owned pointers)."""
    f = ca.Fields()
    owned = []
    if layout == "B":
        def arena(groups):
            per = sum(n * rows for n, rows in groups)          # elements per block
            base = hip.alloc(nblocks * per * nproma * es)
            owned.append(base)
            return base, per * nproma
        # inputs: level planes (klev rows), species fields (5 klev rows), paph (klev + 1 rows)
        ib, ibs = arena([(len(IN_LEVEL), klev), (len(IN_SPECIES), 5 * klev), (len(IN_HALF), klev + 1)])
        off = 0
        for n in IN_LEVEL:
            setattr(f, n, ib + off * es); off += klev * nproma
        for n in IN_SPECIES:
            setattr(f, n, ib + off * es); off += 5 * klev * nproma
        for n in IN_HALF:
            setattr(f, n, ib + off * es); off += (klev + 1) * nproma
        ob, obs = arena([(len(OUT_LEVEL), klev), (len(OUT_SPECIES), 5 * klev), (len(OUT_HALF), klev + 1)])
        off = 0
        for n in OUT_LEVEL:
            setattr(f, n, ob + off * es); off += klev * nproma
        for n in OUT_SPECIES:
            setattr(f, n, ob + off * es); off += 5 * klev * nproma
        for n in OUT_HALF:
            setattr(f, n, ob + off * es); off += (klev + 1) * nproma
        strides = [ibs, nproma, klev * nproma, obs, nproma, klev * nproma]
    else:   # "I"
        rows = klev + 1
        # inputs: row r = the level planes of level r, the 5 species planes of each species field, paph(r)
        w_in = len(IN_LEVEL) + 5 * len(IN_SPECIES) + len(IN_HALF)
        rs_in = w_in * nproma
        ib = hip.alloc(nblocks * rows * rs_in * es)
        owned.append(ib)
        slot = 0
        for n in IN_LEVEL:
            setattr(f, n, ib + slot * nproma * es); slot += 1
        for n in IN_SPECIES:
            setattr(f, n, ib + slot * nproma * es); slot += 5
        for n in IN_HALF:
            setattr(f, n, ib + slot * nproma * es); slot += 1
        # outputs: row r = level r's planes, then half level r+1's fluxes (stored one row down), plus one
        # leading row so that half level 0 of block 0 stays inside the allocation
        w_out = len(OUT_LEVEL) + 5 * len(OUT_SPECIES) + len(OUT_HALF)
        rs_out = w_out * nproma
        ob0 = hip.alloc((nblocks * rows + 1) * rs_out * es)
        owned.append(ob0)
        ob = ob0 + rs_out * es
        slot = 0
        for n in OUT_LEVEL:
            setattr(f, n, ob + slot * nproma * es); slot += 1
        for n in OUT_SPECIES:
            setattr(f, n, ob + slot * nproma * es); slot += 5
        for n in OUT_HALF:
            setattr(f, n, ob + (slot * nproma - rs_out) * es); slot += 1
        strides = [rows * rs_in, rs_in, nproma, rows * rs_out, rs_out, nproma]
    pr = hip.alloc(nblocks * nproma * es)            # prainfrac (surface) stays a buffer of its own
    owned.append(pr)
    f.prainfrac_toprfz = pr
    return f, strides, owned


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--layouts", default="P,B,I")
    ap.add_argument("--ngptot", type=int, default=163840)
    ap.add_argument("--nproma", type=int, default=64)
    a = ap.parse_args()
    lib = ca.gpu_lib()
    lib.cloudsc_debug_memory_probe_layout.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                      C.POINTER(ca.Fields), C.c_int, C.c_int,
                                                      C.POINTER(C.c_longlong), C.POINTER(C.c_float)]
    ds = ca.load_dataset()
    klev, prec, es = ds.klev, ca.FP64, 8
    nblocks = (a.ngptot + a.nproma - 1) // a.nproma
    hip = Hip()
    layouts = a.layouts.split(",")
    sets = []                      # (layout, Fields, strides, keepalive)
    for i in range(a.sets):
        for L in layouts:
            if L == "P":
                df = ca.DeviceFields(a.ngptot, a.nproma, klev, prec, place=False)
                sets.append((L, df.f, [0] * 6, df))
            else:
                f, st, owned = arena_set(hip, L, nblocks, a.nproma, klev, es)
                sets.append((L, f, st, owned))

    def probe(f, st, mode):
        ms = C.c_float()
        s6 = (C.c_longlong * 6)(*st)
        ca.check(lib.cloudsc_debug_memory_probe_layout(0, prec, a.ngptot, a.nproma, klev, C.byref(f), mode, 2, s6,
                                                       C.byref(ms)))
        return ms.value

    for _ in range(3):                           # clock warm-up
        for L, f, st, _k in sets:
            probe(f, st, 1)
    rw = [[] for _ in sets]
    wo = [[] for _ in sets]
    for r in range(a.rounds):
        order = range(len(sets)) if r % 2 == 0 else reversed(range(len(sets)))
        for i in order:
            L, f, st, _k = sets[i]
            rw[i].append(probe(f, st, 1))
            wo[i].append(probe(f, st, 0))
    for L in layouts:
        idx = [i for i, s in enumerate(sets) if s[0] == L]
        for name, data in (("rw", rw), ("write", wo)):
            med = sorted(float(np.median(data[i])) for i in idx)
            print(json.dumps({"layout": L, "probe": name, "sets": len(idx), "rounds": a.rounds,
                              "set_medians_ms": [round(float(np.median(data[i])), 4) for i in idx],
                              "median_ms": round(med[len(med) // 2], 4), "fastest_ms": round(med[0], 4),
                              "slowest_ms": round(med[-1], 4), "spread": round(med[-1] / med[0] - 1, 4)}),
                  flush=True)
    for L, f, st, keep in sets:
        if L == "P":
            keep.close()
        else:
            for p in keep:
                hip.h.hipFree(p)


if __name__ == "__main__":
    main()
