"""Host-side mirror of the CLOUDSC dwarf plumbing, over the libcloudsc_amd.so C ABI.

This is the Python face of the same boundary the C host driver
(``dwarf-p-cloudsc_amd/csrc/dwarf_cloudsc_amd.c``) uses.  It mirrors the
reference driver's plumbing:

* dataset loading -- the Serialbox raw arrays + global scalars the reference
  reads (``src/cloudsc_c/cloudsc/load_state.c:279-690``; the ``data/*.dat`` files
  are C-order ``[lev][klon]`` / ``[nclv][lev][klon]`` arrays, exactly the HDF5
  dataset layout of ``config-files/reference.h5``);
* NPROMA-block expansion with the global ``g % klon`` column map
  (``load_state.c:69-184``, ``src/common/module/expand_mod.F90:173-200``);
* field-wise validation with the Fortran ERROR_PRINT semantics
  (``src/common/module/validate_mod.F90:118-296``) -- ``fabs``, not the C
  validator's integer ``abs`` (``cloudsc_validate.c:74,109,147``);
* the GPU state API (device-side expand / run / validate) of ``cloudsc_amd.h``.

The GPU path has no fallback: if ``libcloudsc_amd.so`` is missing or no HIP
device is visible, :func:`gpu_lib` raises.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libcloudsc_amd.so")
DATA_DIR = os.path.join(REPO, "data", "cloudsc100")   # the reference's data/ arrays (tools/make_fixtures.py)

NCLV = 5
FP64, FP32 = 8, 4
VARIANT_SCC, VARIANT_KCACHE, VARIANT_KSEG, VARIANT_SCC_PRIVATE = 1, 2, 3, 4

# ---------------------------------------------------------------------------
# cloudsc_params_t  (order == include/cloudsc_amd.h)
# ---------------------------------------------------------------------------
PARAM_DOUBLES = (
    "ptsphy rg rd rcpd retv rlvtt rlstt rlmlt rtt rv "
    "r2es r3les r3ies r4les r4ies r5les r5ies r5alvcp r5alscp "
    "ralvdcp ralsdcp ralfdcp rtwat rtice rticecu rtwat_rtice_r rtwat_rticecu_r rkoop1 rkoop2 "
    "ramid rcldiff rcldiff_convi rclcrit rclcrit_sea rclcrit_land rkconv rprc1 rprc2 "
    "rcldmax rpecons rvrfactor rprecrhmax rtaumel ramin rlmin rkooptau rcldtopp "
    "rlcritsnow rsnowlin1 rsnowlin2 ricehi1 ricehi2 riceinit rvice rvrain rvsnow "
    "rthomo rcovpmin rccn rnice rccnom rccnss rccnsu rcldtopcf rdepliqrefrate "
    "rdepliqrefdepth rcl_kkaac rcl_kkbac rcl_kkaau rcl_kkbauq rcl_kkbaun "
    "rcl_kk_cloud_num_sea rcl_kk_cloud_num_land rcl_ai rcl_bi rcl_ci rcl_di "
    "rcl_x1i rcl_x2i rcl_x3i rcl_x4i rcl_const1i rcl_const2i rcl_const3i rcl_const4i "
    "rcl_const5i rcl_const6i rcl_apb1 rcl_apb2 rcl_apb3 rcl_as rcl_bs rcl_cs rcl_ds "
    "rcl_x1s rcl_x2s rcl_x3s rcl_x4s rcl_const1s rcl_const2s rcl_const3s rcl_const4s "
    "rcl_const5s rcl_const6s rcl_const7s rcl_const8s rdenswat rdensref rcl_ar rcl_br "
    "rcl_cr rcl_dr rcl_x1r rcl_x2r rcl_x4r rcl_ka273 rcl_cdenom1 rcl_cdenom2 rcl_cdenom3 "
    "rcl_schmidt rcl_dynvisc rcl_const1r rcl_const2r rcl_const3r rcl_const4r rcl_fac1 "
    "rcl_fac2 rcl_const5r rcl_const6r rcl_fzrab rcl_fzrbb nshapep nshapeq"
).split()
PARAM_INTS = (
    "lcldextra lcldbudget nssopt ncldtop naeclbc naecldu naeclom naeclss naeclsu nclddiag "
    "naercld laerliqautolsp laerliqautocp laerliqautocpb laerliqcoll laericesed laericeauto nbeta"
).split()


class Params(C.Structure):
    _fields_ = [(n, C.c_double) for n in PARAM_DOUBLES] + [(n, C.c_int) for n in PARAM_INTS]

    @classmethod
    def from_dict(cls, d: Dict[str, float]) -> "Params":
        p = cls()
        for n in PARAM_DOUBLES:
            setattr(p, n, float(d[n]))
        for n in PARAM_INTS:
            setattr(p, n, int(d[n]))
        return p

    def to_dict(self) -> Dict[str, float]:
        return {n: getattr(self, n) for n in PARAM_DOUBLES + PARAM_INTS}


# ---------------------------------------------------------------------------
# field inventory
# ---------------------------------------------------------------------------
# kind: "2d" [lev][klon], "2dh" [lev+1][klon], "3d" [nclv][lev][klon], "1d" [klon]
INPUT_FIELDS = {
    "pt": "2d", "pq": "2d", "tendency_tmp_t": "2d", "tendency_tmp_q": "2d", "tendency_tmp_a": "2d",
    "tendency_tmp_cld": "3d", "pvfl": "2d", "pvfi": "2d", "phrsw": "2d", "phrlw": "2d",
    "pvervel": "2d", "pap": "2d", "paph": "2dh", "plsm": "1d", "ktype": "1d", "plu": "2d",
    "psnde": "2d", "pmfu": "2d", "pmfd": "2d", "pa": "2d", "pclv": "3d", "psupsat": "2d",
}
AEROSOL_FIELDS = {"plcrit_aer": "2d", "picrit_aer": "2d", "pre_ice": "2d", "pccn": "2d", "pnice": "2d"}
INOUT_FIELDS = {"plude": "2d"}
OUTPUT_FIELDS = {
    "tendency_loc_t": "2d", "tendency_loc_q": "2d", "tendency_loc_a": "2d", "tendency_loc_cld": "3d",
    "pcovptot": "2d", "prainfrac_toprfz": "1d",
    "pfsqlf": "2dh", "pfsqif": "2dh", "pfcqnng": "2dh", "pfcqlng": "2dh", "pfsqrf": "2dh",
    "pfsqsf": "2dh", "pfcqrng": "2dh", "pfcqsng": "2dh", "pfsqltur": "2dh", "pfsqitur": "2dh",
    "pfplsl": "2dh", "pfplsn": "2dh", "pfhpsl": "2dh", "pfhpsn": "2dh",
}
ALL_FIELDS = {**INPUT_FIELDS, **AEROSOL_FIELDS, **INOUT_FIELDS, **OUTPUT_FIELDS}

# The 21 validated fields in the dwarf's print order (cloudsc_validate.c:193-216).
VALIDATED = [
    ("PLUDE", "plude"), ("PCOVPTOT", "pcovptot"), ("PRAINFRAC_TOPRFZ", "prainfrac_toprfz"),
    ("PFSQLF", "pfsqlf"), ("PFSQIF", "pfsqif"), ("PFCQLNG", "pfcqlng"), ("PFCQNNG", "pfcqnng"),
    ("PFSQRF", "pfsqrf"), ("PFSQSF", "pfsqsf"), ("PFCQRNG", "pfcqrng"), ("PFCQSNG", "pfcqsng"),
    ("PFSQLTUR", "pfsqltur"), ("PFSQITUR", "pfsqitur"), ("PFPLSL", "pfplsl"), ("PFPLSN", "pfplsn"),
    ("PFHPSL", "pfhpsl"), ("PFHPSN", "pfhpsn"), ("TENDENCY_LOC%A", "tendency_loc_a"),
    ("TENDENCY_LOC%Q", "tendency_loc_q"), ("TENDENCY_LOC%T", "tendency_loc_t"),
    ("TENDENCY_LOC%CLD", "tendency_loc_cld"),
]
# Fortran NDIM printed by ERROR_PRINT (VALIDATE_R1/R2/R3)
VALIDATED_NDIM = {n: (1 if ALL_FIELDS[k] == "1d" else 3 if ALL_FIELDS[k] == "3d" else 2) for n, k in VALIDATED}

class Fields(C.Structure):
    """cloudsc_fields_t (pointer order == include/cloudsc_amd.h)."""
    _fields_ = [(n, C.c_void_p) for n in (
        "pt pq tendency_tmp_t tendency_tmp_q tendency_tmp_a tendency_tmp_cld "
        "pvfl pvfi phrsw phrlw pvervel pap paph plsm ktype "
        "plu psnde pmfu pmfd pa pclv psupsat "
        "plcrit_aer picrit_aer pre_ice pccn pnice plude "
        "tendency_loc_t tendency_loc_q tendency_loc_a tendency_loc_cld pcovptot prainfrac_toprfz "
        "pfsqlf pfsqif pfcqnng pfcqlng pfsqrf pfsqsf pfcqrng pfcqsng "
        "pfsqltur pfsqitur pfplsl pfplsn pfhpsl pfhpsn").split()]


class Placement(C.Structure):
    """cloudsc_placement_t: what a placement search cost and found."""
    _fields_ = [("probe_first_ms", C.c_float), ("probe_final_ms", C.c_float), ("tries", C.c_int),
                ("moves", C.c_int), ("launches", C.c_int), ("method", C.c_int), ("search_ms", C.c_double),
                ("peak_transient_bytes", C.c_longlong), ("transient_budget_bytes", C.c_longlong)]

    def to_dict(self) -> dict:
        return {"probe_first_ms": round(self.probe_first_ms, 4), "probe_final_ms": round(self.probe_final_ms, 4),
                "tries": self.tries, "moves": self.moves, "launches": self.launches,
                "method": {0: "none", 1: "kernel", 2: "write-probe", 3: "rw-probe"}.get(self.method, self.method),
                "search_ms": round(self.search_ms, 1), "peak_transient_bytes": self.peak_transient_bytes,
                "transient_budget_bytes": self.transient_budget_bytes}


PLACE_NONE = 1
ALLOC_AEROSOLS = 2


class Template(C.Structure):
    _fields_ = [("klon", C.c_int), ("klev", C.c_int)] + [(n, C.c_void_p) for n in (
        "pt pq tendency_tmp_t tendency_tmp_q tendency_tmp_a tendency_tmp_cld "
        "pvfl pvfi phrsw phrlw pvervel pap paph plsm ktype "
        "plu plude psnde pmfu pmfd pa pclv psupsat "
        "plcrit_aer picrit_aer pre_ice pccn pnice").split()]


class Reference(C.Structure):
    _fields_ = [("klon", C.c_int), ("klev", C.c_int), ("field", C.c_void_p * 21)]


class Stats(C.Structure):
    _fields_ = [("minval", C.c_double), ("maxval", C.c_double), ("maxerr", C.c_double),
                ("errsum", C.c_double), ("refsum", C.c_double),
                ("errsum_lo", C.c_double), ("refsum_lo", C.c_double)]


# ---------------------------------------------------------------------------
# dataset (template) I/O
# ---------------------------------------------------------------------------
def field_shape(kind: str, klev: int, klon: int):
    return {"2d": (klev, klon), "2dh": (klev + 1, klon), "3d": (NCLV, klev, klon), "1d": (klon,)}[kind]


def read_params_txt(path: str) -> Dict[str, float]:
    out: Dict[str, float] = {}
    with open(path) as fh:
        for line in fh:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            name, val = line.split("=")
            name, val = name.strip(), val.strip()
            out[name] = int(val) if name in PARAM_INTS else float(val)
    return out


def write_params_txt(path: str, params: Dict[str, float]) -> None:
    with open(path, "w") as fh:
        fh.write("# CLOUDSC parameter block (YOMCST, YOETHF, TECLDP, PTSPHY); %.17g = exact\n")
        for n in PARAM_DOUBLES:
            fh.write("%s = %.17g\n" % (n, params[n]))
        for n in PARAM_INTS:
            fh.write("%s = %d\n" % (n, int(params[n])))


@dataclass
class Dataset:
    """KLON template columns + parameters (+ optional reference outputs)."""
    klon: int
    klev: int
    params: Dict[str, float]
    inputs: Dict[str, np.ndarray]
    reference: Dict[str, np.ndarray] = field(default_factory=dict)

    def copy(self) -> "Dataset":
        return Dataset(self.klon, self.klev, dict(self.params),
                       {k: v.copy() for k, v in self.inputs.items()},
                       {k: v.copy() for k, v in self.reference.items()})


def read_serialbox_params(path: str) -> Dict[str, float]:
    """The parameter block from a Serialbox store's MetaData-input.json
    (global_meta_info, the input.h5 scalar names: RG, ..., YRECLDP_<NAME>;
    logicals as 0/1), keyed like params.txt (lower case, no YRECLDP_ prefix)."""
    g = json.load(open(os.path.join(path, "MetaData-input.json")))["global_meta_info"]
    by_key = {}
    for name, v in g.items():
        key = (name[8:] if name.startswith("YRECLDP_") else name).lower()
        by_key[key] = v["value"]
    out: Dict[str, float] = {}
    for n in PARAM_DOUBLES:
        out[n] = float(by_key[n])
    for n in PARAM_INTS:
        out[n] = int(by_key[n])
    return out


def load_dataset(path: str = DATA_DIR, with_reference: bool = True) -> Dataset:
    """Read a data directory: a Serialbox store (the reference's data/:
    MetaData-input.json + input_<NAME>.dat, reference_<NAME>.dat) or the raw
    form written by tools/make_fixtures.py (manifest.json + params.txt + the
    same .dat arrays)."""
    if os.path.exists(os.path.join(path, "MetaData-input.json")):
        g = json.load(open(os.path.join(path, "MetaData-input.json")))["global_meta_info"]
        klon, klev = int(g["KLON"]["value"]), int(g["KLEV"]["value"])
        params = read_serialbox_params(path)
    else:
        man = json.load(open(os.path.join(path, "manifest.json")))
        klon, klev = man["klon"], man["klev"]
        params = read_params_txt(os.path.join(path, "params.txt"))
    inputs = {}
    for name, kind in {**INPUT_FIELDS, **AEROSOL_FIELDS, **INOUT_FIELDS}.items():
        fn = os.path.join(path, "input_%s.dat" % name.upper())
        if not os.path.exists(fn):
            continue
        dt = np.int32 if name == "ktype" else np.float64
        inputs[name] = np.fromfile(fn, dtype=dt).reshape(field_shape(kind, klev, klon))
    ref = {}
    if with_reference:
        for vname, key in VALIDATED:
            fn = os.path.join(path, "reference_%s.dat" % key.upper())
            if os.path.exists(fn):
                ref[key] = np.fromfile(fn, dtype=np.float64).reshape(field_shape(ALL_FIELDS[key], klev, klon))
    return Dataset(klon, klev, params, inputs, ref)


# ---------------------------------------------------------------------------
# NPROMA-block expansion / contraction (host, numpy)
# ---------------------------------------------------------------------------
def nblocks_of(ngptot: int, nproma: int) -> int:
    return ngptot // nproma + (1 if ngptot % nproma else 0)


def global_columns(ngptot: int, nproma: int, col_offset: int = 0) -> np.ndarray:
    """[nblocks, nproma] global column index of every block lane (lanes past
    ngptot replicate the map, like the C loader's expand_* which fills them)."""
    nb = nblocks_of(ngptot, nproma)
    return col_offset + np.arange(nb * nproma, dtype=np.int64).reshape(nb, nproma)


def expand(arr: np.ndarray, kind: str, ngptot: int, nproma: int, col_offset: int = 0,
           dtype=None) -> np.ndarray:
    """Template ``[..][klon]`` -> block layout ``[nblocks][..][nproma]`` with g % klon."""
    klon = arr.shape[-1]
    src = global_columns(ngptot, nproma, col_offset) % klon            # [nb, nproma]
    out = np.take(arr, src, axis=-1)                                   # [..., nb, nproma]
    out = np.moveaxis(out, -2, 0)                                      # [nb, ..., nproma]
    return np.ascontiguousarray(out, dtype=dtype or arr.dtype)


def blocks_to_columns(arr: np.ndarray, ngptot: int) -> np.ndarray:
    """Block layout ``[nb][..][nproma]`` -> column-last ``[..][ngptot]``."""
    x = np.moveaxis(arr, 0, -2)                                        # [..., nb, nproma]
    x = x.reshape(x.shape[:-2] + (-1,))
    return x[..., :ngptot]


@dataclass
class HostState:
    """All kernel fields in block layout on the host (used with the oracle)."""
    ngptot: int
    nproma: int
    klev: int
    precision: int
    arrays: Dict[str, np.ndarray]

    def fields(self) -> Fields:
        f = Fields()
        for name, _ in Fields._fields_:
            a = self.arrays.get(name)
            setattr(f, name, a.ctypes.data if a is not None else None)
        return f


_KIND_CODE = {"2d": 0, "2dh": 1, "3d": 2, "1d": 3}
_io = None


def io_lib():
    """libcloudsc_io.so (host-only dataset plumbing of the C driver), or None if
    it is not built -- then the numpy forms below are used (same results)."""
    global _io
    if _io is None:
        path = os.path.join(HERE, "libcloudsc_io.so")
        if not os.path.exists(path):
            return None
        lib = C.CDLL(path)
        lib.cloudsc_io_expand.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.c_longlong, C.c_int, C.c_void_p]
        lib.cloudsc_io_field_stats.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                               C.c_int, C.c_int, C.c_longlong, C.c_void_p]
        _io = lib
    return _io


def make_host_state(ds: Dataset, ngptot: int, nproma: int, precision: int = FP64,
                    col_offset: int = 0) -> HostState:
    real = np.float64 if precision == FP64 else np.float32
    nb = nblocks_of(ngptot, nproma)
    arrays = {}
    io = io_lib()
    for name, arr in ds.inputs.items():
        kind = ALL_FIELDS[name]
        dt = np.int32 if name == "ktype" else real
        if io is not None and arr.dtype == (np.int32 if name == "ktype" else np.float64):
            src = np.ascontiguousarray(arr)
            out = np.empty((nb,) + field_shape(kind, ds.klev, nproma), dtype=dt)
            io.cloudsc_io_expand(src.ctypes.data, _KIND_CODE[kind], int(name == "ktype"), ds.klev, ds.klon,
                                 ngptot, nproma, col_offset, out.itemsize, out.ctypes.data)
            arrays[name] = out
        else:
            arrays[name] = expand(arr, kind, ngptot, nproma, col_offset, dtype=dt)
    for name, kind in OUTPUT_FIELDS.items():
        shp = (nb,) + field_shape(kind, ds.klev, nproma)
        arrays[name] = np.full(shp, np.nan, dtype=real)                # callee must write all
    return HostState(ngptot, nproma, ds.klev, precision, arrays)


# ---------------------------------------------------------------------------
# validation (Fortran ERROR_PRINT semantics, validate_mod.F90:118-296)
# ---------------------------------------------------------------------------
def field_stats(field: np.ndarray, ref: np.ndarray) -> tuple:
    f = field.astype(np.float64).ravel()
    r = ref.astype(np.float64).ravel()
    d = np.abs(f - r)
    return (float(f.min()), float(f.max()), float(d.max()), float(d.sum()), float(np.abs(r).sum()))


def rel_error(errsum: float, refsum: float, eps: float = np.finfo(np.float64).eps):
    """(zrelerr, iopt) exactly as ERROR_PRINT (validate_mod.F90:273-283)."""
    if errsum < eps:
        return 0.0, 1
    if refsum < eps:
        return errsum / (1.0 + refsum), 2
    return errsum / refsum, 3


def format_row(name: str, ndim: int, st: tuple, ngptot: int, eps: float = np.finfo(np.float64).eps) -> str:
    mn, mx, maxerr, errsum, refsum = st
    rel, iopt = rel_error(errsum, refsum, eps)
    warn = " !!!!" if rel > 10.0 * eps else "     "
    # Fortran format (1X,A20,1X,I1,'D',I1,5(1X,E20.13),A)
    return " %20s %dD%d %20.13E %20.13E %20.13E %20.13E %20.13E%s" % (
        name, ndim, iopt, mn, mx, maxerr, errsum / ngptot, 100.0 * rel, warn)


def state_outputs_to_template(arrays: Dict[str, np.ndarray], ngptot: int) -> Dict[str, np.ndarray]:
    return {k: blocks_to_columns(arrays[k], ngptot) for _, k in VALIDATED}


# ---------------------------------------------------------------------------
# GPU library (no fallback)
# ---------------------------------------------------------------------------
class CloudscError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


_lib = None


def gpu_lib(path: Optional[str] = None):
    """Load libcloudsc_amd.so.  Raises if it is missing: there is no CPU fallback."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("CLOUDSC_AMD_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise CloudscError("libcloudsc_amd.so not built (%s): run __graft_entry__.build()" % path)
    lib = C.CDLL(path)
    lib.cloudsc_strerror.restype = C.c_char_p
    lib.cloudsc_last_hip_error.restype = C.c_char_p
    lib.cloudsc_abi_sizeof.restype = C.c_longlong
    lib.cloudsc_gpu_scratch_bytes.restype = C.c_longlong
    lib.cloudsc_state_field_elems.restype = C.c_longlong
    lib.cloudsc_state_create.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_longlong, C.POINTER(Template), C.POINTER(Params)]
    lib.cloudsc_state_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float)]
    lib.cloudsc_state_run_span.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float)]
    lib.cloudsc_state_validate.argtypes = [C.c_void_p, C.POINTER(Reference), C.POINTER(Stats)]
    lib.cloudsc_state_download.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    lib.cloudsc_state_field_elems.argtypes = [C.c_void_p, C.c_int]
    lib.cloudsc_state_destroy.argtypes = [C.c_void_p]
    lib.cloudsc_state_sync.argtypes = [C.c_void_p]
    lib.cloudsc_state_reset.argtypes = [C.c_void_p]
    lib.cloudsc_state_fields.argtypes = [C.c_void_p, C.POINTER(Fields)]
    if hasattr(lib, "cloudsc_state_placement"):
        lib.cloudsc_state_placement.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                                C.POINTER(C.c_int), C.POINTER(C.c_int)]
        lib.cloudsc_debug_set_placement_search.argtypes = [C.c_int]
    if hasattr(lib, "cloudsc_debug_set_pipeline_copy"):
        lib.cloudsc_debug_set_pipeline_copy.argtypes = [C.c_int]
        lib.cloudsc_debug_host_pipeline_copy.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                                         C.POINTER(C.c_int)]
        lib.cloudsc_debug_host_pipeline_engine_check.argtypes = [C.c_void_p, C.POINTER(C.c_double),
                                                                 C.POINTER(C.c_int)]
        lib.cloudsc_host_pipeline_copy_bound.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    if hasattr(lib, "cloudsc_debug_memory_probe"):
        lib.cloudsc_debug_memory_probe.argtypes = [C.c_int] * 5 + [C.POINTER(Fields), C.c_int, C.c_int,
                                                                  C.POINTER(C.c_float)]
    if hasattr(lib, "cloudsc_fields_alloc"):
        lib.cloudsc_fields_alloc.argtypes = [C.c_int] * 6 + [C.POINTER(Fields), C.POINTER(Placement)]
        lib.cloudsc_fields_free.argtypes = [C.c_int, C.POINTER(Fields)]
        lib.cloudsc_state_placement_report.argtypes = [C.c_void_p, C.POINTER(Placement)]
    lib.cloudsc_gpu_init.argtypes = [C.c_int, C.POINTER(Params)]
    lib.cloudsc_gpu_run.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.POINTER(Fields), C.c_void_p]
    lib.cloudsc_host_pipeline_create.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int,
                                                 C.c_int, C.c_int, C.c_int, C.POINTER(Fields)]
    lib.cloudsc_host_pipeline_run.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double)]
    lib.cloudsc_host_pipeline_destroy.argtypes = [C.c_void_p]
    lib.cloudsc_gpu_check.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p]
    lib.cloudsc_hbm_copy_gbps.argtypes = [C.c_int, C.c_longlong, C.c_int, C.POINTER(C.c_double)]
    if hasattr(lib, "cloudsc_pcie_gbps"):   # (older experiment builds lack it)
        lib.cloudsc_pcie_gbps.argtypes = [C.c_int, C.c_longlong, C.c_int] + [C.POINTER(C.c_double)] * 3
    lib.cloudsc_cpu_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Params), C.POINTER(Fields),
                                    C.POINTER(C.c_double)]
    lib.cloudsc_debug_set_kseg_spin_limit.argtypes = [C.c_longlong]
    lib.cloudsc_debug_set_kseg_schedule.argtypes = [C.c_int, C.c_int]
    lib.cloudsc_debug_host_pipeline_mapping.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.cloudsc_debug_host_pinned.argtypes = [C.c_void_p, C.c_longlong]
    lib.cloudsc_debug_fp32_libm.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_longlong]
    _lib = lib
    return lib


EINVAL = -1
EHANDOFF = -7
# option bit of a variant argument: fp32 exp/pow with the glibc algorithms (bit-identical to the fp32 restatement)
FP32_EXACT_LIBM = 0x100


def kseg_schedule(nseg: int = 0, grid: int = 0) -> None:
    """Diagnostic override of the KSEG schedule (0 = default); results do not change."""
    check(gpu_lib().cloudsc_debug_set_kseg_schedule(nseg, grid))


def kseg_spin_limit(limit: int = -1) -> None:
    """Diagnostic: polls before a KSEG consumer gives up (negative = default, 0 = fail at once)."""
    check(gpu_lib().cloudsc_debug_set_kseg_spin_limit(limit))


def cpu_run(ds: "Dataset", ngptot: int, nproma: int = 32, nthreads: int = 0, col_offset: int = 0):
    """The library's CPU variant (cloudsc_cpu_run, BASELINE.json config 1) on a
    host block-layout state expanded from ds.  Returns (HostState, seconds).
    Explicitly a CPU run -- it is never used in place of a GPU run."""
    st = make_host_state(ds, ngptot, nproma, FP64, col_offset)
    return st, cpu_run_state(ds, st, nthreads)


def cpu_run_state(ds: "Dataset", st: "HostState", nthreads: int = 0) -> float:
    """cloudsc_cpu_run on an already expanded host state (plude is INOUT: the
    caller restores it between runs).  Returns seconds of the block loop."""
    p = Params.from_dict(ds.params)
    f = st.fields()
    secs = C.c_double()
    check(gpu_lib().cloudsc_cpu_run(nthreads, st.ngptot, st.nproma, st.klev, C.byref(p), C.byref(f),
                                    C.byref(secs)))
    return secs.value


def validate_host_state(ds: "Dataset", st: "HostState") -> float:
    """Worst per-field relative L1 error (ERROR_PRINT, validate_mod.F90:263-296)
    of a host state's 21 outputs against ds.reference replicated with g % klon."""
    worst = 0.0
    io = io_lib()
    cols = None
    for _, k in VALIDATED:
        if io is not None:
            ref = np.ascontiguousarray(ds.reference[k], dtype=np.float64)
            fld = np.ascontiguousarray(st.arrays[k])
            stt = Stats()
            io.cloudsc_io_field_stats(ref.ctypes.data, _KIND_CODE[ALL_FIELDS[k]], ds.klev, ds.klon, fld.ctypes.data,
                                      fld.itemsize, st.ngptot, st.nproma, 0, C.byref(stt))
            errsum, refsum = stt.errsum, stt.refsum
        else:
            cols = np.arange(st.ngptot) % ds.klon if cols is None else cols
            out = blocks_to_columns(st.arrays[k], st.ngptot)
            _, _, _, errsum, refsum = field_stats(out, np.take(ds.reference[k], cols, axis=-1))
        worst = max(worst, rel_error(errsum, refsum)[0])
    return worst


# the translation unit of the CLOUDSC kernels (cloudsc_gpu.hip and what it includes)
KERNEL_SOURCES = ("cloudsc_gpu.hip", "cloudsc_kcache.h", "cloudsc_scc.h", "cloudsc_dev.h", "cloudsc_params.h",
                  "cloudsc_libm.h", "cloudsc_libm_tab.h", "cloudsc_internal.h")


def kernel_source_hash() -> str:
    """SHA-256 (16 hex digits) of the kernels' sources and the library's build
    flags (Makefile): the key that ties a measured PMC traffic figure to the
    kernel it was measured on (bench.py drops a figure whose hash is not the
    current one)."""
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES + ("../../include/cloudsc_amd.h", "../Makefile"):
        h.update(name.encode())
        with open(os.path.normpath(os.path.join(HERE, "csrc", name)), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def hbm_copy_gbps(device: int = 0, nbytes: int = 4 << 30, reps: int = 10) -> float:
    """Achievable HBM bandwidth of the device (STREAM copy, GB/s)."""
    g = C.c_double()
    check(gpu_lib().cloudsc_hbm_copy_gbps(device, nbytes, reps, C.byref(g)))
    return g.value


def pcie_gbps(device: int = 0, nbytes: int = 1 << 30, reps: int = 3) -> Dict[str, float]:
    """Host<->device copy ceiling (cloudsc_pcie_gbps): GB/s of H2D alone, D2H
    alone, and the total of both directions at once."""
    h, d, b = C.c_double(), C.c_double(), C.c_double()
    check(gpu_lib().cloudsc_pcie_gbps(device, nbytes, reps, C.byref(h), C.byref(d), C.byref(b)))
    return {"h2d": h.value, "d2h": d.value, "both": b.value}


def device_count() -> int:
    """Visible HIP devices (through the library; raises if it is missing)."""
    n = C.c_int(0)
    check(gpu_lib().cloudsc_gpu_device_count(C.byref(n)))
    return n.value


def check(rc: int) -> None:
    if rc != 0:
        lib = gpu_lib()
        raise CloudscError("cloudsc error %d: %s (hip: %s)" % (
            rc, lib.cloudsc_strerror(rc).decode(), (lib.cloudsc_last_hip_error() or b"").decode()), rc)


def make_template(ds: Dataset, keep: list) -> Template:
    t = Template()
    t.klon, t.klev = ds.klon, ds.klev
    for name, _ in Template._fields_[2:]:
        a = ds.inputs.get(name)
        if a is not None:
            a = np.ascontiguousarray(a)
            keep.append(a)
            setattr(t, name, a.ctypes.data)
    return t


def make_reference(ds: Dataset, keep: list) -> Reference:
    r = Reference()
    r.klon, r.klev = ds.klon, ds.klev
    for i, (_, key) in enumerate(VALIDATED):
        a = np.ascontiguousarray(ds.reference[key], dtype=np.float64)
        keep.append(a)
        r.field[i] = a.ctypes.data
    return r


class GpuState:
    """Device-resident CLOUDSC problem (cloudsc_state_* of cloudsc_amd.h)."""

    def __init__(self, ds: Dataset, ngptot: int, nproma: int = 128, precision: int = FP64,
                 device: int = 0, col_offset: int = 0):
        self.lib = gpu_lib()
        self.ds, self.ngptot, self.nproma, self.precision = ds, ngptot, nproma, precision
        keep: list = []
        tmpl = make_template(ds, keep)
        self._params = Params.from_dict(ds.params)
        h = C.c_void_p()
        check(self.lib.cloudsc_state_create(C.byref(h), device, precision, ngptot, nproma,
                                            col_offset, C.byref(tmpl), C.byref(self._params)))
        self.h = h

    def run(self, variant: int = VARIANT_KCACHE, reps: int = 1) -> np.ndarray:
        ms = (C.c_float * reps)()
        check(self.lib.cloudsc_state_run(self.h, variant, reps, ms))
        return np.array(ms[:], dtype=np.float64)

    def run_span(self, variant: int = VARIANT_KCACHE, reps: int = 1) -> float:
        """`reps` plain launches timed as a whole (cloudsc_state_run_span): ms from
        the first launch's start to the last one's end."""
        ms = C.c_float()
        check(self.lib.cloudsc_state_run_span(self.h, variant, reps, C.byref(ms)))
        return float(ms.value)

    def sync(self) -> None:
        check(self.lib.cloudsc_state_sync(self.h))

    def kseg_clock(self, reset: bool = False) -> float:
        """Effective shader clock (GHz) of the KSEG launches since the last reset
        (cloudsc_state_kseg_clock); 0.0 before any KSEG launch."""
        ghz = C.c_double()
        check(self.lib.cloudsc_state_kseg_clock(self.h, int(reset), C.byref(ghz)))
        return ghz.value

    def placement(self) -> dict:
        """The output placement search of this state (cloudsc_state_placement)."""
        a, b, t, m = C.c_float(), C.c_float(), C.c_int(), C.c_int()
        check(self.lib.cloudsc_state_placement(self.h, C.byref(a), C.byref(b), C.byref(t), C.byref(m)))
        return {"probe_first_ms": round(a.value, 4), "probe_final_ms": round(b.value, 4),
                "tries": t.value, "moves": m.value}

    def placement_report(self) -> dict:
        """The placement search with its cost (cloudsc_state_placement_report)."""
        r = Placement()
        check(self.lib.cloudsc_state_placement_report(self.h, C.byref(r)))
        return r.to_dict()

    def reset(self) -> None:
        check(self.lib.cloudsc_state_reset(self.h))

    def validate(self, ds: Optional[Dataset] = None) -> list:
        ds = ds or self.ds
        keep: list = []
        ref = make_reference(ds, keep)
        st = (Stats * 21)()
        check(self.lib.cloudsc_state_validate(self.h, C.byref(ref), st))
        # (min, max, max|d|, sum|d|, sum|ref|, and the low parts of the two
        # double-double sums: cloudsc_dist.combine_stats adds partials exactly)
        return [(s.minval, s.maxval, s.maxerr, s.errsum, s.refsum, s.errsum_lo, s.refsum_lo) for s in st]

    def download(self, key: str) -> np.ndarray:
        idx = [k for _, k in VALIDATED].index(key)
        n = self.lib.cloudsc_state_field_elems(self.h, idx)
        out = np.empty(n, dtype=np.float64)
        check(self.lib.cloudsc_state_download(self.h, idx, out.ctypes.data))
        nb = nblocks_of(self.ngptot, self.nproma)
        return out.reshape((nb,) + field_shape(ALL_FIELDS[key], self.ds.klev, self.nproma))

    def outputs(self) -> Dict[str, np.ndarray]:
        """All 21 validated fields, column-last template-like order [..][ngptot]."""
        return {k: blocks_to_columns(self.download(k), self.ngptot) for _, k in VALIDATED}

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.cloudsc_state_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostPipeline:
    """Host-buffer CLOUDSC step (cloudsc_host_pipeline_* of cloudsc_amd.h): the
    block-layout arrays live in host memory (pinned in place) and every step
    copies inputs in and outputs out, chunked and overlapped over streams."""

    def __init__(self, ds: Dataset, ngptot: int, nproma: int = 128, precision: int = FP64, device: int = 0,
                 chunk_blocks: int = 128, nstreams: int = 3, col_offset: int = 0, packed: bool = False):
        """packed: all arrays carved back to back (8-byte gaps) out of ONE host
        buffer, so that neighbouring fields share pages -- the layout that
        exercises the pipeline's page-merged pinning."""
        self.lib = gpu_lib()
        self.ds, self.ngptot, self.nproma, self.precision = ds, ngptot, nproma, precision
        self._params = Params.from_dict(ds.params)
        check(self.lib.cloudsc_gpu_init(device, C.byref(self._params)))
        self.state = make_host_state(ds, ngptot, nproma, precision, col_offset)
        if packed:
            arrs = self.state.arrays
            self._buf = np.empty(sum(a.nbytes + 8 for a in arrs.values()) + 64, dtype=np.uint8)
            off = 8 - self._buf.ctypes.data % 8
            for name, a in list(arrs.items()):
                v = self._buf[off:off + a.nbytes].view(a.dtype).reshape(a.shape)
                v[...] = a
                arrs[name] = v
                off += a.nbytes + 8
        self._plude0 = self.state.arrays["plude"].copy()
        f = self.state.fields()
        if not (ds.params.get("laericesed") or ds.params.get("laericeauto")):
            for name in AEROSOL_FIELDS:            # not read by the kernel: not transferred
                setattr(f, name, None)
        self._fields = f
        h = C.c_void_p()
        check(self.lib.cloudsc_host_pipeline_create(C.byref(h), device, precision, ngptot, nproma, ds.klev,
                                                    chunk_blocks, nstreams, C.byref(f)))
        self.h = h

    def run(self, variant: int = VARIANT_KCACHE) -> float:
        """One step; plude is restored on the host first (INOUT).  Returns ms."""
        np.copyto(self.state.arrays["plude"], self._plude0)
        ms = C.c_double()
        check(self.lib.cloudsc_host_pipeline_run(self.h, variant, C.byref(ms)))
        return ms.value

    def outputs(self) -> Dict[str, np.ndarray]:
        return state_outputs_to_template(self.state.arrays, self.ngptot)

    def mapping(self):
        """(arrays, arrays NOT covered by one pinned mapping) -- the pinning
        invariant of cloudsc_host_pipeline_create (cloudsc_debug_host_pipeline_mapping)."""
        n, bad = C.c_int(), C.c_int()
        check(self.lib.cloudsc_debug_host_pipeline_mapping(self.h, C.byref(n), C.byref(bad)))
        return n.value, bad.value

    def copy_path(self):
        """(mode, H2D engine mask, D2H engine mask) of this pipeline
        (cloudsc_debug_host_pipeline_copy): mode 1 = copy engines per direction,
        0 = HIP streams."""
        m, a, b = C.c_int(), C.c_int(), C.c_int()
        check(self.lib.cloudsc_debug_host_pipeline_copy(self.h, C.byref(m), C.byref(a), C.byref(b)))
        return m.value, a.value, b.value

    def copy_bound(self) -> float:
        """ms of one step's copies without the kernels, same engines and
        arrays (cloudsc_host_pipeline_copy_bound); clobbers the host outputs
        and plude (restored by the next run())."""
        t = C.c_double()
        check(self.lib.cloudsc_host_pipeline_copy_bound(self.h, C.byref(t)))
        return t.value

    def engine_check(self):
        """(overlap, pairs tried) of the engine pair check at creation
        (cloudsc_debug_host_pipeline_engine_check): overlap = both directions at
        once / the slower alone for the kept pair (1.0 = fully concurrent)."""
        o, n = C.c_double(), C.c_int()
        check(self.lib.cloudsc_debug_host_pipeline_engine_check(self.h, C.byref(o), C.byref(n)))
        return o.value, n.value

    def host_arrays(self):
        """(pointer, bytes) of every host array handed to the pipeline."""
        out = []
        for name, _ in Fields._fields_:
            p = getattr(self._fields, name)
            if p:
                out.append((p, self.state.arrays[name].nbytes))
        return out

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.cloudsc_host_pipeline_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipDeviceSynchronize.argtypes = []
    h.hipSetDevice.argtypes = [C.c_int]
    return h


class DeviceFields:
    """Caller-owned device fields (cloudsc_fields_alloc / cloudsc_fields_free):
    the reference CUDA driver's shape -- allocate (cloudsc_driver.cu:276-328),
    copy the inputs in, launch cloudsc_gpu_run (:391-416), copy the outputs
    back (:425-447) -- with the output buffers placed by the library's
    memory-pattern search (reads + writes, no physics) unless place=False."""

    def __init__(self, ngptot: int, nproma: int, klev: int, precision: int = FP64, device: int = 0,
                 place: bool = True, aerosols: bool = False):
        self.lib = gpu_lib()
        self.ngptot, self.nproma, self.klev, self.precision, self.device = ngptot, nproma, klev, precision, device
        self.f = Fields()
        self.report = Placement()
        flags = (0 if place else PLACE_NONE) | (ALLOC_AEROSOLS if aerosols else 0)
        check(self.lib.cloudsc_fields_alloc(device, precision, ngptot, nproma, klev, flags, C.byref(self.f),
                                            C.byref(self.report)))
        self.hip = _hip()

    def nbytes(self, name: str) -> int:
        es = 4 if name == "ktype" or self.precision == FP32 else 8
        return nblocks_of(self.ngptot, self.nproma) * int(np.prod(field_shape(ALL_FIELDS[name], self.klev,
                                                                             self.nproma))) * es

    def copy_from(self, src: "Fields", names) -> None:
        """Device-to-device copy of the named fields from another field set of
        the same configuration (e.g. a state's, cloudsc_state_fields)."""
        self.hip.hipSetDevice(self.device)
        for n in names:
            rc = self.hip.hipMemcpy(getattr(self.f, n), getattr(src, n), self.nbytes(n), 3)
            if rc != 0:
                raise CloudscError("hipMemcpy %s failed (%d)" % (n, rc))

    def upload(self, arrays: Dict[str, np.ndarray]) -> None:
        """Host block-layout arrays (make_host_state(...).arrays) into the device buffers."""
        self.hip.hipSetDevice(self.device)
        for n, a in arrays.items():
            if getattr(self.f, n, None) is None:
                continue
            a = np.ascontiguousarray(a)
            assert a.nbytes == self.nbytes(n), (n, a.nbytes, self.nbytes(n))
            rc = self.hip.hipMemcpy(getattr(self.f, n), a.ctypes.data, a.nbytes, 1)
            if rc != 0:
                raise CloudscError("hipMemcpy %s failed (%d)" % (n, rc))

    def download(self, name: str) -> np.ndarray:
        """One field in block layout as float64."""
        self.hip.hipSetDevice(self.device)
        self.hip.hipDeviceSynchronize()
        dt = np.int32 if name == "ktype" else (np.float64 if self.precision == FP64 else np.float32)
        nb = nblocks_of(self.ngptot, self.nproma)
        out = np.empty((nb,) + field_shape(ALL_FIELDS[name], self.klev, self.nproma), dtype=dt)
        rc = self.hip.hipMemcpy(out.ctypes.data, getattr(self.f, name), out.nbytes, 2)
        if rc != 0:
            raise CloudscError("hipMemcpy %s failed (%d)" % (name, rc))
        return out.astype(np.float64)

    def close(self) -> None:
        if getattr(self, "f", None) is not None:
            self.lib.cloudsc_fields_free(self.device, C.byref(self.f))
            self.f = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
