#!/usr/bin/env python3
"""Round-5 record of the contiguous-allocation failure.

Round 4 left this open: in the diagnostic build that admits allocation flags,
fp32 states created after hipDeviceMallocContiguous states had been destroyed
(profiles/r04/contiguous_alloc_hazard_repro.py --fp64-first) hold wrong INPUT
words right after cloudsc_state_create.  Two hypotheses were not tested:
  (a) an out-of-bounds store -- state creation runs ~250 KSEG launches (the
      placement search), so "right after create" is not "before any kernel";
  (b) stale cache lines written back late (the wrong-byte counts FELL after
      later launches in round 4, which an out-of-bounds store cannot do).
This script runs the failing sequence ONCE against a build with 64 KiB guard
bands around every device buffer of the states and searches
(-DCLOUDSC_DEBUG_CANARY) and records, per state:
  - the guard bands after creation and after each launch (hypothesis a);
  - every wrong input word, read by a copy engine (hipMemcpy) AND by a kernel
    (cloudsc_debug_kernel_copy, 4-byte loads through the caches on all XCDs):
    where the two readers disagree the memory and a cache disagree;
  - the wrong words' layout: runs of consecutive wrong 4-byte words, their
    start offsets modulo 64 / 128 / 4096 and their lengths;
  - their provenance: whether each wrong value is a word of a previously
    destroyed state (any field, and the same field at the same offset).
Pass 1 with the placement search on (the default), pass 2 with it off.

  make -C dwarf-p-cloudsc_amd variant VFLAGS="-DCLOUDSC_DEBUG_KNOBS -DCLOUDSC_DEBUG_CANARY" \\
       OUT=../diag/libcloudsc_canary.so
  CLOUDSC_AMD_LIB=diag/libcloudsc_canary.so python tools/contig_diag_r05.py > profiles/r05/contig_diag.txt
"""
import collections
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cloudsc_amd as ca  # noqa: E402
import oracle  # noqa: E402

NG, NP = 3000, 64
lib = ca.gpu_lib()
lib.cloudsc_debug_set_state_layout.argtypes = [C.c_longlong, C.c_uint]
lib.cloudsc_debug_canary_check.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_longlong)]
lib.cloudsc_debug_kernel_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong]
hip = C.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipFree.argtypes = [C.c_void_p]
ds = ca.load_dataset()
NAMES = [f[0] for f in ca.Fields._fields_]


def canaries():
    live, bad, nbytes = C.c_int(), C.c_int(), C.c_longlong()
    ca.check(lib.cloudsc_debug_canary_check(C.byref(live), C.byref(bad), C.byref(nbytes)))
    return "%d live, %d with changed guard bytes, %d bytes changed" % (live.value, bad.value, nbytes.value)


def nbytes_of(name, prec):
    es = 4 if (name == "ktype" or prec == ca.FP32) else 8
    return ca.nblocks_of(NG, NP) * int(np.prod(ca.field_shape(ca.ALL_FIELDS[name], ds.klev, NP))) * es


def read_sdma(ptr, n):
    out = np.empty(n // 4, dtype=np.uint32)
    assert hip.hipMemcpy(out.ctypes.data, ptr, n, 2) == 0
    return out


def read_kernel(ptr, n):
    tmp = C.c_void_p()
    assert hip.hipMalloc(C.byref(tmp), n) == 0
    try:
        ca.check(lib.cloudsc_debug_kernel_copy(tmp, ptr, n))
        return read_sdma(tmp, n)
    finally:
        hip.hipFree(tmp)


def fields_of(g):
    f = ca.Fields()
    ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
    return f


def snapshot(g, prec):
    """every buffer of the state as 4-byte words (copy-engine reads)"""
    f = fields_of(g)
    return {n: read_sdma(getattr(f, n), nbytes_of(n, prec)) for n in NAMES
            if getattr(f, n) and n in ca.ALL_FIELDS}


def runs_of(mask):
    """(start word, length) of the runs of True in mask"""
    d = np.diff(np.concatenate(([0], mask.astype(np.int8), [0])))
    starts = np.nonzero(d == 1)[0]
    ends = np.nonzero(d == -1)[0]
    return list(zip(starts.tolist(), (ends - starts).tolist()))


def analyse(name, got, want, kread, history):
    bad = got != want
    nbad = int(bad.sum())
    kbad = int((kread != want).sum())
    disagree = int((kread != got).sum())
    runs = runs_of(bad)
    lens = collections.Counter(min(l * 4, 4096) for _, l in runs)
    al64 = collections.Counter((s * 4) % 64 for s, _ in runs)
    al128 = sum(1 for s, _ in runs if (s * 4) % 128 == 0)
    al4k = sum(1 for s, _ in runs if (s * 4) % 4096 == 0)
    # provenance: each wrong value among the words of previously destroyed states
    vals = got[bad]
    prov_any, prov_same = collections.Counter(), 0
    for age, snap in enumerate(history):
        for fname, words in snap.items():
            hit = np.isin(vals, words)
            if hit.any():
                prov_any["state-%d:%s" % (age + 1, fname)] += int(hit.sum())
        if name in snap and snap[name].shape == got.shape:
            prov_same += int((snap[name][bad] == vals).sum())
    in_any = np.zeros(vals.shape, dtype=bool)
    for snap in history:
        for words in snap.values():
            in_any |= np.isin(vals, words)
    return ("%s: %d wrong words (copy engine), %d wrong by kernel read, %d words where the two readers differ; "
            "%d runs, lengths(B) %s; run starts mod 64 B %s, 128-B aligned %d, 4-KiB aligned %d; "
            "wrong values found in earlier states' buffers: %d of %d (same field, same offset: %d), top sources %s"
            % (name, nbad, kbad, disagree, len(runs), dict(sorted(lens.items())[:6]), dict(sorted(al64.items())),
               al128, al4k, int(in_any.sum()), nbad, prov_same, prov_any.most_common(4)))


def check_inputs(g, prec, history, detail):
    f = fields_of(g)
    host = ca.make_host_state(ds, NG, NP, prec)
    hip.hipDeviceSynchronize()
    out = []
    total = 0
    for name in ca.INPUT_FIELDS:
        ptr = getattr(f, name)
        if not ptr or name not in host.arrays:
            continue
        want = np.ascontiguousarray(host.arrays[name]).view(np.uint32).ravel()
        got = read_sdma(ptr, want.nbytes)
        if not (got != want).any():
            continue
        total += int((got != want).sum())
        if detail:
            out.append(analyse(name, got, want, read_kernel(ptr, want.nbytes), history))
    return total, out


def main():
    refs = {}
    for prec in (ca.FP64, ca.FP32):
        st, _ = oracle.run_oracle(ds, NG, NP, prec)
        refs[prec] = ca.state_outputs_to_template(st.arrays, NG)
    seq = [(-1, 0), (0, 0), (-1, 0), (4608, 0), (-1, 0), (-1, 4), (-1, 0), (-1, 0), (-1, 4), (0, 0), (-1, 0)]
    print("library:", os.environ.get("CLOUDSC_AMD_LIB", ca.LIB_PATH), flush=True)
    print("canaries at start:", canaries(), flush=True)
    for pass_no, search in ((1, -1), (2, 0)):
        ca.check(lib.cloudsc_set_placement_search(search))
        print("=== pass %d: placement search %s" % (pass_no, "on" if search else "off"), flush=True)
        history = []
        for prec in (ca.FP64, ca.FP32):
            for i, (stagger, flags) in enumerate(seq):
                ca.check(lib.cloudsc_debug_set_state_layout(stagger, flags))
                g = ca.GpuState(ds, NG, NP, prec)
                try:
                    rep = g.placement_report()
                    nbad, detail = check_inputs(g, prec, history, detail=True)
                    line = ["fp%d #%d layout %s search %s (%d launches): inputs wrong after create: %d words; "
                            "canaries %s" % (8 * prec, i, (stagger, flags), rep["method"], rep["launches"], nbad,
                                             canaries())]
                    line += ["    " + d for d in detail[:6]]
                    for vname, v in (("KSEG", ca.VARIANT_KSEG), ("KCACHE", ca.VARIANT_KCACHE)):
                        g.run(v, 1)
                        o = g.outputs()
                        ref = refs[prec]
                        if prec == ca.FP64:
                            diff = [k for k in ref if not np.array_equal(o[k].view(np.uint8), ref[k].view(np.uint8))]
                            res = "bit-equal to the oracle" if not diff else "differs in %s" % diff[:4]
                        else:
                            worst = max(float(np.abs(o[k] - ref[k]).sum() / max(np.abs(ref[k]).sum(), 1e-300))
                                        for k in ref)
                            res = "worst relL1 vs fp32 oracle %.2e" % worst
                        nb2, _ = check_inputs(g, prec, history, detail=False)
                        line.append("    %s: %s; inputs wrong after: %d words; canaries %s" % (vname, res, nb2,
                                                                                              canaries()))
                    print("\n".join(line), flush=True)
                    history.insert(0, snapshot(g, prec))
                    del history[3:]
                finally:
                    g.close()
                    ca.check(lib.cloudsc_debug_set_state_layout(-1, 0))
        print("canaries after pass %d: %s" % (pass_no, canaries()), flush=True)
    ca.check(lib.cloudsc_set_placement_search(-1))


if __name__ == "__main__":
    main()
