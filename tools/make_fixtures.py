#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists; the GPU box only reads the result).

1. data/cloudsc100/  -- the reference's own 100-column data set:
   * input_<FIELD>.dat     raw little-endian arrays copied byte-for-byte from
                           data/input_<FIELD>.dat (Serialbox binary; C order
                           [lev][klon] / [nclv][lev][klon] / [klon], i.e. the
                           HDF5 dataset layout, serialbox2hdf5/serialbox2hdf5.py:11-33)
   * reference_<FIELD>.dat the 21 golden outputs, data/reference_<FIELD>.dat
                           (byte-identical to config-files/reference.h5)
   * params.txt            PTSPHY + YOMCST + YOETHF + YRECLDP scalars from
                           data/MetaData-input.json global_meta_info (%.17g)
   * manifest.json         klon, klev, field list
2. tests/golden/scenario_{W,M}.npz -- perturbed inputs that reach the branches the
   shipped data never exercises (rain, melting, freezing, land),
   with the outputs of the UNMODIFIED reference kernel (oracle/_ref) as expected
   values.  Inputs and outputs are both stored: RNG draw order is not relied on.
"""
import json
import os
import shutil
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cloudsc_amd as ca  # noqa: E402

REFDATA = "/root/reference/data"
OUT = os.path.join(REPO, "tests", "golden")


def json_params(meta_path):
    g = json.load(open(meta_path))["global_meta_info"]
    p = {}
    for k, v in g.items():
        name = k.lower()
        if name.startswith("yrecldp_"):
            name = name[len("yrecldp_"):]
        p[name] = v["value"]
    out = {}
    for n in ca.PARAM_DOUBLES:
        out[n] = float(p[n])
    for n in ca.PARAM_INTS:
        out[n] = int(p[n])
    return out, g["KLON"]["value"], g["KLEV"]["value"]


def make_cloudsc100():
    d = os.path.join(REPO, "data", "cloudsc100")
    os.makedirs(d, exist_ok=True)
    params, klon, klev = json_params(os.path.join(REFDATA, "MetaData-input.json"))
    ca.write_params_txt(os.path.join(d, "params.txt"), params)
    names = list(ca.INPUT_FIELDS) + list(ca.INOUT_FIELDS) + ["picrit_aer", "pre_ice", "pnice"]
    for n in names:
        shutil.copyfile(os.path.join(REFDATA, "input_%s.dat" % n.upper()),
                        os.path.join(d, "input_%s.dat" % n.upper()))
    for _, key in ca.VALIDATED:
        shutil.copyfile(os.path.join(REFDATA, "reference_%s.dat" % key.upper()),
                        os.path.join(d, "reference_%s.dat" % key.upper()))
    json.dump({"klon": klon, "klev": klev, "source": "lukasm91/dwarf-p-cloudsc data/ (Serialbox raw)",
               "inputs": sorted(n.upper() for n in names),
               "reference": [k.upper() for _, k in ca.VALIDATED]},
              open(os.path.join(d, "manifest.json"), "w"), indent=1)
    print("wrote", d)


PERTURBED = ["pt", "pq", "pclv", "plsm"]


def scenario(ds, name):
    """SURVEY.md §8c recipes, seed 20250227."""
    s = ds.copy()
    rng = np.random.default_rng(20250227)
    klev, klon = s.klev, s.klon
    if name == "W":     # warm: rain autoconversion/evaporation, melting, land
        s.inputs["pt"] = s.inputs["pt"] + 25.0 + rng.uniform(-2.0, 2.0, size=(klev, klon))
    elif name == "M":   # mixed: melting layer -> rain freezing, homogeneous freezing
        pt = s.inputs["pt"].copy()
        bump = 1.6 * np.linspace(0.0, 22.0, 30) * np.sin(np.linspace(0.0, np.pi, 30))
        pt[95:125, :] += bump[:, None] + rng.uniform(-1.0, 1.0, size=(30, klon))
        s.inputs["pt"] = pt
        pclv = s.inputs["pclv"].copy()
        pclv[2, 100:137, :] += 2e-5
        cold = pt < 233.0
        pclv[0][cold] += 1e-5
        s.inputs["pclv"] = pclv
        pq = s.inputs["pq"].copy()
        pq[pt < 235.0] *= 1.6
        s.inputs["pq"] = pq
    plsm = s.inputs["plsm"].copy()
    plsm[1::2] = 1.0
    s.inputs["plsm"] = plsm
    return s



def perturbed(ds, seed):
    """Randomly perturbed copy of the state (temperature, humidity, condensate,
    land mask, convection type, supersaturation) so that many branch
    combinations are hit.  Used by the oracle-vs-reference tests and by the GPU
    parity tests (same seed -> same inputs)."""
    rng = np.random.default_rng(seed)
    s = ds.copy()
    klev, klon = s.klev, s.klon
    s.inputs["pt"] = s.inputs["pt"] + rng.uniform(-5, 30, size=(1, klon)) + rng.normal(0, 1, size=(klev, klon))
    s.inputs["pq"] = s.inputs["pq"] * rng.uniform(0.5, 1.8, size=(klev, klon))
    pclv = s.inputs["pclv"].copy()
    pclv[:4] += rng.uniform(0, 3e-5, size=(4, klev, klon)) * (rng.random((4, klev, klon)) < 0.3)
    s.inputs["pclv"] = pclv
    s.inputs["plsm"] = (rng.random(klon) < 0.5).astype(np.float64)
    s.inputs["ktype"] = rng.integers(0, 3, size=klon).astype(np.int32)
    s.inputs["psupsat"] = s.inputs["psupsat"] + rng.uniform(0, 1e-6, size=(klev, klon)) * (rng.random((klev, klon)) < 0.2)
    s.reference = {}
    return s


def shifted(ds, kind):
    """Regime copies of the state: "cold" (every temperature 25 K lower: ice
    only, homogeneous freezing below RTHOMO, Koop-limited supersaturation),
    "dry" (humidity x0.1, no condensate: the tidy-up and evaporation paths),
    "moist" (humidity x1.6 and ten times the condensate: supersaturation
    adjustment, autoconversion, precipitation everywhere)."""
    s = ds.copy()
    if kind == "cold":
        s.inputs["pt"] = s.inputs["pt"] - 25.0
    elif kind == "dry":
        s.inputs["pq"] = s.inputs["pq"] * 0.1
        s.inputs["pclv"] = np.zeros_like(s.inputs["pclv"])
        s.inputs["pa"] = np.zeros_like(s.inputs["pa"])
    elif kind == "moist":
        s.inputs["pq"] = s.inputs["pq"] * 1.6
        s.inputs["pclv"] = s.inputs["pclv"] * 10.0
    else:
        raise ValueError(kind)
    s.reference = {}
    return s


def with_aerosols(ds, seed=11):
    """Copy of the state with LAERICESED / LAERICEAUTO on and physically sized
    aerosol inputs (the shipped PRE_ICE / PICRIT_AER / PNICE are all zero, which
    makes the aerosol branches divide by zero): ice effective radius 10-100 um
    (fall speed 0.002*re vs RVICE=0.13), critical ice content 1e-5..1e-4
    (vs RLCRITSNOW=3e-5), ice number 0.01-0.1 (vs RNICE=0.027)."""
    rng = np.random.default_rng(seed)
    s = ds.copy()
    shp = s.inputs["pt"].shape
    s.inputs["pre_ice"] = rng.uniform(10.0, 100.0, size=shp)
    s.inputs["picrit_aer"] = rng.uniform(1e-5, 1e-4, size=shp)
    s.inputs["pnice"] = rng.uniform(0.01, 0.1, size=shp)
    s.params["laericesed"] = 1
    s.params["laericeauto"] = 1
    s.reference = {}
    return s

# Input edges: states pushed beyond the shipped data's ranges (condensate down
# to 1e-200 or subnormal, or up 1000x; no water at all; full cloud cover;
# temperatures 60 K warmer or 80 K colder; tendencies, mass fluxes 100x;
# pressures 100x lower), for the parity tests at the edges of the input space.
EDGE_CASES = ("condensate_1e-200", "condensate_subnormal", "condensate_x1000", "no_water", "full_cover",
              "hot_plus60K", "cold_minus80K", "tendencies_x100", "pressure_x0.01", "mass_flux_x100")


def edge_case(ds, name):
    """Copy of the state for one of EDGE_CASES."""
    edits = {
        "condensate_1e-200": {"pclv": lambda a: a * 1e-200},
        "condensate_subnormal": {"pclv": lambda a: np.where(a > 0, 1e-310, 0.0)},
        "condensate_x1000": {"pclv": lambda a: a * 1000.0},
        "no_water": {"pclv": np.zeros_like, "pq": np.zeros_like, "pa": np.zeros_like},
        "full_cover": {"pa": np.ones_like},
        "hot_plus60K": {"pt": lambda a: a + 60.0},
        "cold_minus80K": {"pt": lambda a: a - 80.0},
        "tendencies_x100": {k: (lambda a: a * 100.0) for k in ("tendency_tmp_t", "tendency_tmp_q", "tendency_tmp_a",
                                                                "tendency_tmp_cld")},
        "pressure_x0.01": {"pap": lambda a: a * 0.01, "paph": lambda a: a * 0.01},
        "mass_flux_x100": {"pmfu": lambda a: a * 100.0, "pmfd": lambda a: a * 100.0},
    }[name]
    s = ds.copy()
    for k, f in edits.items():
        s.inputs[k] = np.ascontiguousarray(f(s.inputs[k]))
    s.reference = {}
    return s


# Parameter edges: other time steps, and the tuning parameters of YRECLDP
# jittered together (the thermodynamic constants of YOMCST / YOETHF and the
# integer switches kept), for the parity tests over the parameter space.
PARAM_CASES = ("ptsphy_60", "ptsphy_900", "ptsphy_1234.567", "ptsphy_7200", "tuning_jitter_1", "tuning_jitter_2")
THERMO_CONSTANTS = ("rg", "rd", "rcpd", "retv", "rlvtt", "rlstt", "rlmlt", "rtt", "rv", "r2es", "r3les", "r3ies",
                    "r4les", "r4ies", "r5les", "r5ies", "r5alvcp", "r5alscp", "ralvdcp", "ralsdcp", "ralfdcp",
                    "rtwat", "rtice", "rticecu", "rtwat_rtice_r", "rtwat_rticecu_r", "rkoop1", "rkoop2", "ptsphy")


def param_case(ds, name):
    """Copy of the state for one of PARAM_CASES: ptsphy_<seconds>, or every
    float YRECLDP parameter multiplied by its own factor in [0.9, 1.1]
    (tuning_jitter_<seed>)."""
    s = ds.copy()
    s.params = dict(s.params)
    if name.startswith("ptsphy_"):
        s.params["ptsphy"] = float(name[len("ptsphy_"):])
    else:
        rng = np.random.default_rng(int(name.rsplit("_", 1)[1]))
        for k in sorted(s.params):
            v = s.params[k]
            if k.startswith("r") and k not in THERMO_CONSTANTS and isinstance(v, float):
                s.params[k] = v * float(rng.uniform(0.9, 1.1))
    s.reference = {}
    return s


def sliced_levels(ds, lo_lev):
    """The bottom KLEV-lo_lev levels of the state as a standalone column
    (half-level pressures sliced to match)."""
    import cloudsc_amd as ca
    s = ds.copy()
    for name, kind in {**ca.INPUT_FIELDS, **ca.AEROSOL_FIELDS, **ca.INOUT_FIELDS}.items():
        if name not in s.inputs:
            continue
        a = s.inputs[name]
        if kind in ("2d", "2dh"):
            s.inputs[name] = np.ascontiguousarray(a[lo_lev:])
        elif kind == "3d":
            s.inputs[name] = np.ascontiguousarray(a[:, lo_lev:])
    s.klev = ds.klev - lo_lev
    s.reference = {}
    return s


def refined_levels(ds, factor=2):
    """A deeper column (KLEV * factor levels): every layer split into `factor`
    equal-pressure sublayers -- full-level fields repeated, half-level pressures
    interpolated linearly between the original interfaces."""
    import cloudsc_amd as ca
    s = ds.copy()
    kinds = {**ca.INPUT_FIELDS, **ca.AEROSOL_FIELDS, **ca.INOUT_FIELDS}
    for name, kind in kinds.items():
        if name not in s.inputs:
            continue
        a = s.inputs[name]
        if kind == "2d":
            s.inputs[name] = np.ascontiguousarray(np.repeat(a, factor, axis=0))
        elif kind == "3d":
            s.inputs[name] = np.ascontiguousarray(np.repeat(a, factor, axis=1))
        elif kind == "2dh":
            lo, hi = a[:-1], a[1:]
            sub = [lo + (hi - lo) * (j / factor) for j in range(factor)]
            inter = np.stack(sub, axis=1).reshape((a.shape[0] - 1) * factor, *a.shape[1:])
            s.inputs[name] = np.ascontiguousarray(np.concatenate([inter, a[-1:]], axis=0))
    s.klev = ds.klev * factor
    s.reference = {}
    return s


def make_scenarios():
    import oracle  # the compiled reference kernel (oracle/_ref)
    if not oracle.ref_available():
        raise SystemExit("oracle/_ref/libcloudsc_ref.so missing: make -C oracle")
    ds = ca.load_dataset(os.path.join(REPO, "data", "cloudsc100"))
    for name in ("W", "M"):
        s = scenario(ds, name)
        st, _ = oracle.run_ref(s, s.klon, s.klon, nthreads=1)
        outs = ca.state_outputs_to_template(st.arrays, s.klon)
        arrays = {"in_" + k: s.inputs[k] for k in PERTURBED}
        arrays.update({"out_" + k: v for k, v in outs.items()})
        for k, v in outs.items():
            assert np.all(np.isfinite(v)), (name, k)
        fn = os.path.join(OUT, "scenario_%s.npz" % name)
        np.savez_compressed(fn, **arrays)
        print("wrote", fn, "rain tendency nonzero points:",
              int(np.count_nonzero(outs["tendency_loc_cld"][2])),
              "prainfrac>0 columns:", int(np.count_nonzero(outs["prainfrac_toprfz"])))


def load_scenario(name, base=None):
    """Dataset with the scenario's perturbed inputs and reference outputs."""
    base = base or ca.load_dataset(os.path.join(REPO, "data", "cloudsc100"))
    z = np.load(os.path.join(OUT, "scenario_%s.npz" % name))
    s = base.copy()
    for k in z.files:
        if k.startswith("in_"):
            s.inputs[k[3:]] = z[k]
    s.reference = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return s


if __name__ == "__main__":
    make_cloudsc100()
    make_scenarios()
