"""TEST INFRASTRUCTURE ONLY -- ctypes access to the CPU checker libraries.

* ``liboracle.so``            C restatement of the reference kernel (oracle/cloudsc_oracle.c)
* ``_ref/libcloudsc_ref.so``  the unmodified reference kernel, src/cloudsc_c/cloudsc/cloudsc_c.c,
                              compiled from /root/reference by oracle/Makefile (present only
                              where the reference checkout was available at build time)

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  Parity is pinned by tests/test_oracle.py: restatement ==
reference kernel bit for bit, and both vs the reference goldens.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

ORACLE_LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libcloudsc_ref.so")

_oracle = None
_ref = None


def oracle_lib():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_LIB):
            raise RuntimeError("oracle not built: make -C oracle")
        lib = C.CDLL(ORACLE_LIB)
        lib.cloudsc_oracle_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.POINTER(ca.Params), C.POINTER(ca.Fields),
                                           C.POINTER(C.c_double)]
        _oracle = lib
    return _oracle


def ref_available() -> bool:
    return os.path.exists(REF_LIB)


def ref_lib():
    global _ref
    if _ref is None:
        lib = C.CDLL(REF_LIB)
        lib.cloudsc_ref_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.POINTER(ca.Params), C.POINTER(ca.Fields),
                                        C.POINTER(C.c_double)]
        _ref = lib
    return _ref


def run_oracle(ds: "ca.Dataset", ngptot: int, nproma: int, precision: int = ca.FP64,
               nthreads: int = 0, col_offset: int = 0, libm_nudge: int = 0):
    """Expand ds to ngptot columns, run the restatement. Returns (HostState, seconds).
    libm_nudge (fp32 only): a non-zero seed moves every expf/powf result by -1/0/+1 ulp
    (cloudsc_oracle_set_libm_nudge) -- the sensitivity probe of the fp32 gates."""
    st = ca.make_host_state(ds, ngptot, nproma, precision, col_offset)
    p = ca.Params.from_dict(ds.params)
    f = st.fields()
    secs = C.c_double()
    lib = oracle_lib()
    lib.cloudsc_oracle_set_libm_nudge(C.c_uint(libm_nudge))
    try:
        rc = lib.cloudsc_oracle_run(nthreads, precision, ngptot, nproma, ds.klev,
                                    C.byref(p), C.byref(f), C.byref(secs))
    finally:
        lib.cloudsc_oracle_set_libm_nudge(C.c_uint(0))
    if rc != 0:
        raise RuntimeError("cloudsc_oracle_run failed: %d" % rc)
    return st, secs.value


def run_ref(ds: "ca.Dataset", ngptot: int, nproma: int, nthreads: int = 0, col_offset: int = 0):
    """Same for the reference kernel itself (fp64 only)."""
    st = ca.make_host_state(ds, ngptot, nproma, ca.FP64, col_offset)
    return st, run_ref_state(ds, st, nthreads)


def run_ref_state(ds: "ca.Dataset", st: "ca.HostState", nthreads: int = 0) -> float:
    """The reference kernel on an already expanded host state (plude is INOUT:
    the caller restores it between runs).  Returns seconds of the block loop."""
    ngptot, nproma = st.ngptot, st.nproma
    p = ca.Params.from_dict(ds.params)
    f = st.fields()
    secs = C.c_double()
    rc = ref_lib().cloudsc_ref_run(nthreads, ngptot, nproma, ds.klev, C.byref(p), C.byref(f),
                                   C.byref(secs))
    if rc != 0:
        raise RuntimeError("cloudsc_ref_run failed: %d" % rc)
    return secs.value
