"""The library's CPU variant (cloudsc_cpu_run; BASELINE.json config 1,
`dwarf-cloudsc-c 1 16384 32`) without a GPU: the same per-level phase
functions the GPU kernels are built from, compiled for the host, in the C
dwarf's block loop (src/cloudsc_c/cloudsc/cloudsc_driver.c:183-217).

Pinned bit for bit against the reference kernel itself, compiled from its
sources under /root/reference (oracle/_ref), and against the oracle
restatement and the reference's own goldens / scenario outputs."""
import numpy as np
import pytest

import cloudsc_amd as ca


def bits_equal(out, ref):
    bad = {}
    for _, k in ca.VALIDATED:
        a = np.ascontiguousarray(out[k], dtype=np.float64).view(np.uint64)
        r = np.ascontiguousarray(ref[k], dtype=np.float64).view(np.uint64)
        n = int(np.count_nonzero(a != r))
        if n:
            bad[k] = n
    return bad


def cpu_outputs(ds, ngptot, nproma, nthreads=4, col_offset=0):
    st, _ = ca.cpu_run(ds, ngptot, nproma, nthreads=nthreads, col_offset=col_offset)
    return ca.state_outputs_to_template(st.arrays, ngptot)


@pytest.mark.parametrize("ngptot,nproma", [(100, 32), (1000, 32), (1000, 16), (517, 128), (1, 1)])
def test_cpu_run_bitwise_vs_oracle(ds, oracle_mod, ngptot, nproma):
    ref_st, _ = oracle_mod.run_oracle(ds, ngptot, nproma)
    assert bits_equal(cpu_outputs(ds, ngptot, nproma), ca.state_outputs_to_template(ref_st.arrays, ngptot)) == {}


def test_cpu_run_bitwise_vs_reference_kernel(ds, oracle_mod):
    """config 1's kernel at a test size: the unmodified reference kernel
    (oracle/_ref) on the same expanded state, same NPROMA."""
    if not oracle_mod.ref_available():
        pytest.skip("oracle/_ref not built (no reference checkout)")
    st, _ = oracle_mod.run_ref(ds, 2048, 32)
    assert bits_equal(cpu_outputs(ds, 2048, 32), ca.state_outputs_to_template(st.arrays, 2048)) == {}


@pytest.mark.parametrize("name", ["W", "M"])
def test_cpu_run_scenarios_vs_reference_outputs(scenarios, name):
    # the reference kernel's own outputs of the warm / mixed-phase scenarios
    s = scenarios[name]
    assert bits_equal(cpu_outputs(s, 100, 32), s.reference) == {}


@pytest.mark.parametrize("case", ["nssopt0", "nssopt3", "aerosol", "seed2", "ncldtop2", "ncldtop40", "ncldtop138"])
def test_cpu_run_other_configurations(ds, oracle_mod, case):
    import make_fixtures as mf
    if case.startswith("ncldtop"):
        s = ds.copy()
        s.params["ncldtop"] = int(case[len("ncldtop"):])
    elif case.startswith("nssopt"):
        s = ds.copy()
        s.params["nssopt"] = int(case[-1])
    elif case == "aerosol":
        s = mf.with_aerosols(ds)
    else:
        s = mf.perturbed(ds, 2)
    ref_st, _ = oracle_mod.run_oracle(s, 300, 32)
    assert bits_equal(cpu_outputs(s, 300, 32), ca.state_outputs_to_template(ref_st.arrays, 300)) == {}


@pytest.mark.parametrize("case", __import__("make_fixtures").EDGE_CASES + __import__("make_fixtures").PARAM_CASES)
def test_cpu_run_input_and_parameter_edges(ds, oracle_mod, case):
    """The input-edge states and parameter-edge sets of make_fixtures (the oracle
    is pinned to the reference kernel on them in tests/test_oracle.py)."""
    import make_fixtures as mf
    s = mf.edge_case(ds, case) if case in mf.EDGE_CASES else mf.param_case(ds, case)
    ref_st, _ = oracle_mod.run_oracle(s, 200, 32)
    assert bits_equal(cpu_outputs(s, 200, 32), ca.state_outputs_to_template(ref_st.arrays, 200)) == {}


def test_cpu_run_threads_and_offset_invariance(ds):
    a = cpu_outputs(ds, 1000, 32, nthreads=1)
    b = cpu_outputs(ds, 1000, 32, nthreads=7)
    assert bits_equal(a, b) == {}
    c = cpu_outputs(ds, 600, 32, nthreads=3, col_offset=400)    # block-aligned shard of the same run
    assert bits_equal({k: a[k][..., 400:] for _, k in ca.VALIDATED}, c) == {}


def test_cpu_run_vs_reference_h5_dwarf_tolerance(ds):
    """Every field within the dwarf's own 10*eps line of reference.h5."""
    out = cpu_outputs(ds, 100, 32)
    eps = np.finfo(np.float64).eps
    for name, k in ca.VALIDATED:
        r = ds.reference[k]
        d = np.abs(out[k] - r).sum()
        s = np.abs(r).sum()
        rel = 0.0 if d < eps else (d / s if s >= eps else d / (1.0 + s))
        assert rel <= 10 * eps, (name, rel)


def test_cpu_run_invalid_arguments(ds):
    import ctypes as C
    lib = ca.gpu_lib()
    st = ca.make_host_state(ds, 64, 32)
    p = ca.Params.from_dict(ds.params)
    f = st.fields()
    assert lib.cloudsc_cpu_run(1, 0, 32, ds.klev, C.byref(p), C.byref(f), None) == -1
    assert lib.cloudsc_cpu_run(1, 64, 0, ds.klev, C.byref(p), C.byref(f), None) == -1
    assert lib.cloudsc_cpu_run(1, 64, 32, 1, C.byref(p), C.byref(f), None) == -1
    p.ncldtop = 1
    assert lib.cloudsc_cpu_run(1, 64, 32, ds.klev, C.byref(p), C.byref(f), None) == -1
    p = ca.Params.from_dict(ds.params)
    f.pt = None
    assert lib.cloudsc_cpu_run(1, 64, 32, ds.klev, C.byref(p), C.byref(f), None) == -1


def test_dwarf_cli_config1_cpu():
    """BASELINE.json config 1 through the product CLI: `dwarf-cloudsc-amd 1
    16384 32 --variant cpu` (the reference's `dwarf-cloudsc-c 1 16384 32`,
    src/cloudsc_c/dwarf_cloudsc.c:17-52): timing table, validation against the
    reference outputs with the dwarf's own tolerance, exit status 0."""
    import os
    import re
    import subprocess
    exe = os.path.join(os.path.dirname(ca.LIB_PATH), "dwarf-cloudsc-amd")
    if not os.path.exists(exe):
        pytest.skip("dwarf-cloudsc-amd not built")
    r = subprocess.run([exe, "1", "16384", "32", "--variant", "cpu"], capture_output=True, text=True, timeout=300)
    print(r.stdout[-3000:], r.stderr[-1000:])
    assert r.returncode == 0
    assert re.search(r"^\s+1\s+16384\s+16384\s+512\s+32\s+-1 :.*TOTAL$", r.stdout, re.M)
    assert "VALIDATION: PASSED" in r.stdout
    rows = [l for l in r.stdout.splitlines() if re.match(r"\s+\S+ \dD\d ", l)]
    assert len(rows) == 21 and not any("!!!!" in l for l in rows)
