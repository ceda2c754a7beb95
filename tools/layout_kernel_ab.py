#!/usr/bin/env python3
"""Round-6 layout study in the REAL kernel: the KSEG fp64
kernel over field sets in the reference layout and in a per-block interleave,
through the experiment build of tools/exp_layout_edits.py (block strides in
the kernel arguments; every other line of the kernel unchanged).

Sets, allocated alternately, NSETS of each:
  P   reference layout, one buffer per field, no placement search
      (cloudsc_fields_alloc with CLOUDSC_PLACE_NONE)
  PS  reference layout placed by cloudsc_fields_alloc's search
  B   per-block interleave: one input arena and one output arena, each block's
      chunks of every field side by side ([block][field][rows][nproma]); the
      surface fields (plsm, ktype, prainfrac_toprfz) stay buffers of their own
Every set holds the same inputs (copied from one state, hipMemcpy2D into the
arenas); plude is out of place (read from plude_in, written to f.plude), so
repeated launches are the same step.  Timed round-robin, one shared KSEG
workspace, HIP events on the null stream; then every B set's outputs are copied
back to the reference layout and compared bit for bit with a P set's.

usage (GPU box): CLOUDSC_AMD_LIB=ab/liblayoutB.so python tools/layout_kernel_ab.py [--sets 6] [--rounds 10]
"""
import argparse
import ctypes as C
import json
import os
import statistics as stt
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

ES = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--ngptot", type=int, default=163840)
    ap.add_argument("--nproma", type=int, default=64)
    a = ap.parse_args()
    lib = ca.gpu_lib()
    lib.cloudsc_exp_set_block_strides.argtypes = [C.c_longlong, C.c_longlong]
    lib.cloudsc_exp_run.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(ca.Fields),
                                    C.c_void_p, C.c_void_p]
    hip = C.CDLL("libamdhip64.so")
    for fn, args in (("hipMalloc", [C.POINTER(C.c_void_p), C.c_size_t]), ("hipFree", [C.c_void_p]),
                     ("hipMemset", [C.c_void_p, C.c_int, C.c_size_t]),
                     ("hipMemcpy", [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
                     ("hipMemcpy2D", [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int]),
                     ("hipEventCreate", [C.POINTER(C.c_void_p)]), ("hipEventRecord", [C.c_void_p, C.c_void_p]),
                     ("hipEventSynchronize", [C.c_void_p]), ("hipDeviceSynchronize", []),
                     ("hipEventElapsedTime", [C.POINTER(C.c_float), C.c_void_p, C.c_void_p])):
        getattr(hip, fn).argtypes = args

    def ok(rc, what):
        if rc != 0:
            raise RuntimeError("%s failed: %d" % (what, rc))

    def dmalloc(n):
        p = C.c_void_p()
        ok(hip.hipMalloc(C.byref(p), n), "hipMalloc(%d)" % n)
        return p.value

    ds = ca.load_dataset()
    klev, npr, ngp = ds.klev, a.nproma, a.ngptot
    nb = (ngp + npr - 1) // npr
    ca.check(lib.cloudsc_debug_set_placement_search(0))
    src = ca.GpuState(ds, ngp, npr, ca.FP64)
    sf = ca.Fields()
    ca.check(lib.cloudsc_state_fields(src.h, C.byref(sf)))
    p = ca.Params.from_dict(ds.params)
    ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))

    def rows(kind):
        return {"2d": klev, "2dh": klev + 1, "3d": 5 * klev}[kind]

    in_arena = [n for n, k in ca.INPUT_FIELDS.items() if k != "1d"]
    out_arena = ["plude"] + [n for n, k in ca.OUTPUT_FIELDS.items() if k != "1d"]
    surface = [n for n, k in {**ca.INPUT_FIELDS, **ca.OUTPUT_FIELDS}.items() if k == "1d"]

    def per_block(name):
        return rows(ca.ALL_FIELDS[name]) * npr

    def planar_bytes(name):
        return nb * (npr if ca.ALL_FIELDS[name] == "1d" else per_block(name)) * (4 if name == "ktype" else ES)

    sets = []
    owned = []
    for i in range(a.sets):
        for lay in ("P", "PS", "B"):
            if lay in ("P", "PS"):
                df = ca.DeviceFields(ngp, npr, klev, ca.FP64, place=(lay == "PS"))
                df.copy_from(sf, list(ca.INPUT_FIELDS))
                pl = dmalloc(planar_bytes("plude"))
                ok(hip.hipMemcpy(pl, sf.plude, planar_bytes("plude"), 3), "copy plude")
                owned.append(pl)
                sets.append({"layout": lay, "f": df.f, "keep": df, "plude_in": pl, "bsi": 0, "bso": 0,
                             "placement": df.report.to_dict()})
                continue
            f = ca.Fields()
            # input arena (plude_in among its planes), output arena
            bsi = sum(per_block(n) for n in in_arena) + per_block("plude")
            bso = sum(per_block(n) for n in out_arena)
            ia, oa = dmalloc(nb * bsi * ES), dmalloc(nb * bso * ES)
            owned += [ia, oa]
            off = 0
            for n in in_arena:
                setattr(f, n, ia + off * ES)
                ok(hip.hipMemcpy2D(getattr(f, n), bsi * ES, getattr(sf, n), per_block(n) * ES, per_block(n) * ES, nb, 3),
                   "copy2D " + n)
                off += per_block(n)
            plude_in = ia + off * ES
            ok(hip.hipMemcpy2D(plude_in, bsi * ES, sf.plude, per_block("plude") * ES, per_block("plude") * ES, nb, 3),
               "copy2D plude")
            off = 0
            for n in out_arena:
                setattr(f, n, oa + off * ES)
                off += per_block(n)
            for n in surface:
                q = dmalloc(planar_bytes(n))
                owned.append(q)
                setattr(f, n, q)
                if n in ca.INPUT_FIELDS:
                    ok(hip.hipMemcpy(q, getattr(sf, n), planar_bytes(n), 3), "copy " + n)
            sets.append({"layout": "B", "f": f, "keep": None, "plude_in": plude_in, "bsi": bsi, "bso": bso,
                         "placement": None})
    ok(hip.hipDeviceSynchronize(), "sync")
    nbytes = lib.cloudsc_gpu_scratch_bytes(ca.FP64, ca.VARIANT_KSEG, ngp, npr, klev)
    ws = dmalloc(nbytes)
    ok(hip.hipMemset(ws, 0, 256), "memset ws")
    e0, e1 = C.c_void_p(), C.c_void_p()
    hip.hipEventCreate(C.byref(e0))
    hip.hipEventCreate(C.byref(e1))

    def launch(s):
        ca.check(lib.cloudsc_exp_set_block_strides(s["bsi"], s["bso"]))
        hip.hipEventRecord(e0, None)
        ca.check(lib.cloudsc_exp_run(0, None, ca.FP64, ngp, npr, klev, C.byref(s["f"]), ws, s["plude_in"]))
        hip.hipEventRecord(e1, None)
        hip.hipEventSynchronize(e1)
        t = C.c_float()
        hip.hipEventElapsedTime(C.byref(t), e0, e1)
        return t.value

    for _ in range(3):
        for s in sets:
            launch(s)
    times = [[] for _ in sets]
    for r in range(a.rounds):
        order = range(len(sets)) if r % 2 == 0 else reversed(range(len(sets)))
        for i in order:
            times[i].append(launch(sets[i]))
    ca.check(lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ws))

    # bit-for-bit: every B set's outputs, back in the reference layout, against the first P set's
    def outputs(s):
        res = {}
        for n in out_arena + ["prainfrac_toprfz"]:
            host = np.empty(planar_bytes(n) // ES)
            if s["bso"] and n != "prainfrac_toprfz":
                tmp = dmalloc(planar_bytes(n))
                ok(hip.hipMemcpy2D(tmp, per_block(n) * ES, getattr(s["f"], n), s["bso"] * ES, per_block(n) * ES, nb,
                                   3), "copy2D back " + n)
                ok(hip.hipMemcpy(host.ctypes.data, tmp, planar_bytes(n), 2), "D2H")
                hip.hipFree(tmp)
            else:
                ok(hip.hipMemcpy(host.ctypes.data, getattr(s["f"], n), planar_bytes(n), 2), "D2H")
            res[n] = host
        return res

    ref = outputs([s for s in sets if s["layout"] == "P"][0])
    diffs = []
    for i, s in enumerate(sets):
        if s["layout"] != "B":
            continue
        o = outputs(s)
        bad = [n for n in ref if not np.array_equal(o[n].view(np.uint64), ref[n].view(np.uint64))]
        diffs.append(bad)
    for i, s in enumerate(sets):
        print(json.dumps({"set": i, "layout": s["layout"], "kernel_ms_median": round(stt.median(times[i]), 4),
                          "kernel_ms_min": round(min(times[i]), 4), "placement": s["placement"]}), flush=True)
    summary = {"what": "KSEG fp64 163840/64, experiment build with block strides (tools/exp_layout_edits.py)",
               "sets_per_layout": a.sets, "rounds": a.rounds,
               "b_sets_bitwise_equal_to_reference": all(not d for d in diffs),
               "b_fields_differing": diffs}
    for lay in ("P", "PS", "B"):
        m = sorted(stt.median(times[i]) for i, s in enumerate(sets) if s["layout"] == lay)
        summary[lay] = {"median_ms": round(m[len(m) // 2], 4), "fastest_ms": round(m[0], 4),
                        "slowest_ms": round(m[-1], 4), "spread": round(m[-1] / m[0] - 1, 4)}
    print(json.dumps(summary), flush=True)
    for s in sets:
        if s["keep"] is not None:
            s["keep"].close()
    for q in owned + [ws]:
        hip.hipFree(q)
    src.close()


if __name__ == "__main__":
    main()
