"""Round-4 diagnosis of the contiguous-allocation hazard, second part: the order
that still fails with the parameter upload ordered (contiguous_alloc_hazard_repro.py
--fp64-first: fp32 states created after fp64 and fp32 hipDeviceMallocContiguous
states were destroyed compute wrong values, KSEG and KCACHE alike).

For the state under suspicion this downloads every INPUT field straight from the
device (hipMemcpy on the pointers cloudsc_state_fields returns) and compares it
with the host expansion of the same template, runs KCACHE twice on it, and
compares with the fp32 oracle -- to tell wrong inputs (expansion / copies) from
wrong arithmetic or lost stores.  Sequence (3000 columns, NPROMA 64): the repro's layouts, fp64 first, then fp32;
every state checked after creation and after each of its KSEG and KCACHE runs."""
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
hip = C.CDLL("libamdhip64.so.7")
ds = ca.load_dataset()
FIELDS = [f[0] for f in ca.Fields._fields_]


def device_inputs(g, prec):
    """every non-NULL input field of the state, downloaded with hipMemcpy"""
    f = ca.Fields()
    ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
    host = ca.make_host_state(ds, NG, NP, prec)
    bad = {}
    for name in ca.INPUT_FIELDS:
        ptr = getattr(f, name)
        if not ptr or name not in host.arrays:
            continue
        want = host.arrays[name]
        got = np.empty_like(want)
        again = np.empty_like(want)
        assert hip.hipDeviceSynchronize() == 0          # nothing of ours runs from here on
        assert hip.hipMemcpy(got.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), C.c_size_t(got.nbytes), 2) == 0
        assert hip.hipMemcpy(again.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), C.c_size_t(got.nbytes), 2) == 0
        n = int(np.count_nonzero(got.view(np.uint8) != want.view(np.uint8)))
        m = int(np.count_nonzero(got.view(np.uint8) != again.view(np.uint8)))
        if n or m:
            nan = int(np.count_nonzero(np.isnan(got)))
            bad[name] = "%d bytes wrong (%d NaN values), %d bytes differ between two reads" % (n, nan, m)
    return bad


def overlaps(g, prec):
    """pairs of the state's device fields whose [ptr, ptr + bytes) ranges overlap
    (two live allocations handed the same memory)"""
    f = ca.Fields()
    ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
    es = 8 if prec == ca.FP64 else 4
    nb = ca.nblocks_of(NG, NP)
    spans = []
    for name in FIELDS:
        ptr = getattr(f, name)
        if not ptr:
            continue
        kind = ca.ALL_FIELDS[name if name in ca.ALL_FIELDS else {"tendency_loc_t": "tendency_loc_t"}.get(name, name)]
        n = nb * int(np.prod(ca.field_shape(kind, ds.klev, NP))) * (4 if name == "ktype" else es)
        spans.append((ptr, ptr + n, name))
    spans.sort()
    out = []
    for i in range(len(spans)):
        for j in range(i + 1, len(spans)):
            if spans[j][0] < spans[i][1]:
                out.append("%s/%s" % (spans[i][2], spans[j][2]))
    return out


def run_state(prec, stagger, flags, ref):
    ca.check(lib.cloudsc_debug_set_state_layout(stagger, flags))
    g = ca.GpuState(ds, NG, NP, prec)
    try:
        ca.check(lib.cloudsc_state_sync(g.h))
        msg = ["fp%d layout %-10s" % (8 * prec, (stagger, flags))]
        msg.append("overlapping fields: %s" % (overlaps(g, prec) or "none"))
        msg.append("inputs bad after create: %s" % (device_inputs(g, prec) or "none"))
        for name, v in (("KSEG", ca.VARIANT_KSEG), ("KCACHE", ca.VARIANT_KCACHE)):
            g.run(v, 1)
            o = g.outputs()
            worst = max(float(np.abs(o[k] - ref[k]).sum() / max(np.abs(ref[k]).sum(), 1e-300)) for k in ref)
            nan = [k for k in o if np.isnan(o[k]).any()]
            msg.append("%s relL1 %.2e NaN in %s; inputs bad after: %s" % (name, worst, nan[:4] or "none",
                                                                     device_inputs(g, prec) or "none"))
        print("; ".join(msg), flush=True)
    finally:
        g.close()
        ca.check(lib.cloudsc_debug_set_state_layout(-1, 0))


refs = {}
for prec in (ca.FP64, ca.FP32):
    st, _ = oracle.run_oracle(ds, NG, NP, prec)
    refs[prec] = ca.state_outputs_to_template(st.arrays, NG)
seq = [(-1, 0), (0, 0), (-1, 0), (4608, 0), (-1, 0), (-1, 4), (-1, 0), (-1, 0), (-1, 4), (0, 0), (-1, 0)]
for prec in (ca.FP64, ca.FP32):
    for lay in seq:
        run_state(prec, *lay, refs[prec])
