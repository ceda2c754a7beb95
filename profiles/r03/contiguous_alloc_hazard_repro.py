import ctypes as C, sys, os
sys.path.insert(0, "dwarf-p-cloudsc_amd"); sys.path.insert(0, "tests")
import numpy as np
import cloudsc_amd as ca
lib = ca.gpu_lib(); lib.cloudsc_debug_set_state_layout.argtypes = [C.c_longlong, C.c_uint]
ds = ca.load_dataset()
def run(prec, st, fl):
    ca.check(lib.cloudsc_debug_set_state_layout(st, fl))
    g = ca.GpuState(ds, 3000, 64, prec)
    try:
        g.run(ca.VARIANT_KSEG, 1); return g.outputs()
    finally:
        g.close(); ca.check(lib.cloudsc_debug_set_state_layout(-1, 0))
def same(a, b):
    return [k for k in a if not np.array_equal(np.asarray(a[k]).view(np.uint8), np.asarray(b[k]).view(np.uint8))]
for prec in (ca.FP32, ca.FP64):
    seq = [(-1, 0), (0, 0), (-1, 0), (4608, 0), (-1, 0), (-1, 4), (-1, 0), (-1, 0), (-1, 4), (0, 0), (-1, 0)]
    outs = [run(prec, *l) for l in seq]
    for l, o in zip(seq, outs):
        print(prec, l, "differs from run 0 in", same(o, outs[0])[:6], flush=True)
