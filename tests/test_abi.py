"""The drop-in boundary without a GPU: libcloudsc_amd.so loads, exports every
function include/cloudsc_amd.h declares, and its struct layouts agree with the
ctypes mirror in cloudsc_amd.py (no compute calls)."""
import ctypes as C
import os
import re

import pytest

import cloudsc_amd as ca

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "cloudsc_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:int|long long|char|void)\s*\*?\s*(cloudsc_\w+)\s*\(",
                                 text, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(ca.LIB_PATH):
        pytest.skip("libcloudsc_amd.so not built (__graft_entry__.build())")
    return C.CDLL(ca.LIB_PATH)


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("cloudsc_gpu_init", "cloudsc_gpu_run", "cloudsc_gpu_scratch_bytes", "cloudsc_strerror",
              "cloudsc_state_create", "cloudsc_state_run", "cloudsc_state_validate", "cloudsc_state_destroy"):
        assert f in fns, f
    assert len(fns) >= 16


def test_library_exports_every_declared_symbol(lib):
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_struct_sizes_match_ctypes_mirror(lib):
    lib.cloudsc_abi_sizeof.restype = C.c_longlong
    expect = [C.sizeof(ca.Params), C.sizeof(ca.Fields), C.sizeof(ca.Template), C.sizeof(ca.Reference),
              C.sizeof(ca.Stats)]
    got = [lib.cloudsc_abi_sizeof(i) for i in range(5)]
    assert got == expect
    assert lib.cloudsc_abi_sizeof(5) == -1


def test_param_layout():
    # one run of doubles then one run of ints, in the header's order
    assert len(ca.PARAM_DOUBLES) == 133 and len(ca.PARAM_INTS) == 18
    assert ca.Params.ptsphy.offset == 0
    assert ca.Params.lcldextra.offset == 8 * len(ca.PARAM_DOUBLES)


def test_strerror_and_scratch_sizes(lib):
    lib.cloudsc_strerror.restype = C.c_char_p
    lib.cloudsc_gpu_scratch_bytes.restype = C.c_longlong
    assert lib.cloudsc_strerror(0) == b"success"
    assert lib.cloudsc_strerror(-1) == b"invalid argument"
    assert lib.cloudsc_strerror(-99) == b"unknown error"
    assert b"hand-off" in lib.cloudsc_strerror(-7)
    # KCACHE needs no workspace; SCC and KSEG do; bad sizes -> -1
    assert lib.cloudsc_gpu_scratch_bytes(ca.FP64, ca.VARIANT_KCACHE, 163840, 128, 137) == 0
    assert lib.cloudsc_gpu_scratch_bytes(ca.FP64, ca.VARIANT_SCC_PRIVATE, 163840, 128, 137) == 0
    kseg = lib.cloudsc_gpu_scratch_bytes(ca.FP64, ca.VARIANT_KSEG, 163840, 128, 137)
    assert kseg >= 1280 * 19 * 128 * 8
    assert lib.cloudsc_gpu_scratch_bytes(ca.FP32, ca.VARIANT_KSEG, 163840, 128, 137) < kseg
    scc = lib.cloudsc_gpu_scratch_bytes(ca.FP64, ca.VARIANT_SCC, 163840, 128, 137)
    assert scc > 1280 * 128 * 137 * 8
    assert lib.cloudsc_gpu_scratch_bytes(ca.FP64, ca.VARIANT_SCC, 0, 128, 137) == -1
    assert lib.cloudsc_gpu_scratch_bytes(3, ca.VARIANT_KSEG, 1000, 128, 137) == -1


def test_gpu_lib_fails_loudly_without_library(tmp_path, monkeypatch):
    """No CPU fallback: a missing library raises."""
    monkeypatch.setattr(ca, "_lib", None)
    with pytest.raises(ca.CloudscError):
        ca.gpu_lib(str(tmp_path / "missing.so"))


def test_state_layout_knob_arguments(lib):
    """The diagnostic placement knob accepts staggers that keep every field
    aligned (multiples of 256 bytes; -1 = the default) and refuses misaligned
    ones and hipExtMallocWithFlags flags: after destroyed states whose fields
    were hipDeviceMallocContiguous allocations, later states computed wrong
    values (profiles/r04/contiguous_alloc_hazard.txt).  No device call."""
    lib.cloudsc_debug_set_state_layout.argtypes = [C.c_longlong, C.c_uint]
    assert lib.cloudsc_debug_set_state_layout(100, 0) == ca.EINVAL
    assert lib.cloudsc_debug_set_state_layout(-1, 4) == ca.EINVAL
    assert lib.cloudsc_debug_set_state_layout(-1, 1) == ca.EINVAL
    assert lib.cloudsc_debug_set_state_layout(4608, 0) == 0
    assert lib.cloudsc_debug_set_state_layout((1 << 40) + 256, 0) == 0    # taken modulo 2 MiB
    assert lib.cloudsc_debug_set_state_layout(-1, 0) == 0
