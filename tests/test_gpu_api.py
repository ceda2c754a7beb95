"""GPU tests of the boundary's contracts beyond the numerics of one run:

* parameter sets are per state (and per host pipeline), so states with
  different physics options interleave on one device without seeing each
  other's parameters (the reference passes TECLDP by pointer per launch,
  src/cloudsc_cuda/cloudsc/cloudsc_driver.cu:312,383,411);
* a timed-out KSEG segment hand-off is reported (CLOUDSC_EHANDOFF) through
  every path: the state API, the host pipeline, and cloudsc_gpu_check after a
  low-level cloudsc_gpu_run;
* BASELINE.json configs 2 and 4 at their full size (163840 columns): SCC fp64
  (both temporaries forms) and KCACHE at NPROMA 128 bit-equal to the oracle, and
  SCC-k-caching fp32 bit-equal to the fp32 restatement (driver shape: src/cloudsc_cuda/cloudsc/cloudsc_driver.cu:391-397).
"""
import ctypes as C

import numpy as np
import pytest

import cloudsc_amd as ca
from test_gpu_parity import bitwise_mismatches, field_report, oracle_outputs, rel_l1

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    lib = ca.gpu_lib()
    assert ca.device_count() > 0
    return lib


def outputs_of(g, variant, reps=1):
    g.run(variant, reps)
    return g.outputs()


def test_interleaved_states_keep_their_parameters(lib, ds, oracle_mod):
    """Three states on device 0 -- NSSOPT 0, NSSOPT 1 (the data set's), and the
    aerosol flags on -- created first, then run interleaved with no sync in
    between; a cloudsc_gpu_init with yet another parameter set in the middle
    must not touch them.  Each matches its own oracle bit for bit."""
    import make_fixtures as mf
    s0 = ds.copy()
    s0.params["nssopt"] = 0
    s1 = ds.copy()
    s1.params["nssopt"] = 1
    s_aer = mf.with_aerosols(ds)
    cases = [("nssopt0", s0), ("nssopt1", s1), ("aerosol", s_aer)]
    ngptot, nproma = 1000, 128
    states = [(name, s, ca.GpuState(s, ngptot, nproma)) for name, s in cases]
    try:
        # enqueue on all three streams before anything is read back
        for variant in (ca.VARIANT_KSEG, ca.VARIANT_KCACHE):
            for _, _, g in states:
                ca.check(lib.cloudsc_state_run(g.h, variant, 2, None))
            other = ds.copy()
            other.params["nssopt"] = 3
            p = ca.Params.from_dict(other.params)
            ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))    # the device default set only
        results = {name: g.outputs() for name, _, g in states}
    finally:
        for _, _, g in states:
            g.close()
    for name, s in cases:
        ref = oracle_outputs(oracle_mod, s, ngptot, nproma)
        assert bitwise_mismatches(results[name], ref) == {}, name
    # the parameter sets do differ in their results
    assert not np.array_equal(results["nssopt0"]["tendency_loc_q"], results["nssopt1"]["tendency_loc_q"])


def test_gpu_run_uses_the_device_default_set(lib, ds, oracle_mod):
    """cloudsc_gpu_run runs with the set of the latest cloudsc_gpu_init."""
    s0 = ds.copy()
    s0.params["nssopt"] = 0
    g = ca.GpuState(ds, 512, 128)          # buffers; the state's own set is NSSOPT 1
    try:
        f = ca.Fields()
        ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
        for s in (s0, ds):
            p = ca.Params.from_dict(s.params)
            ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))
            ca.check(lib.cloudsc_state_reset(g.h))
            ca.check(lib.cloudsc_state_sync(g.h))
            ca.check(lib.cloudsc_gpu_run(0, None, ca.FP64, ca.VARIANT_KCACHE, 512, 128, ds.klev, C.byref(f), None))
            ca.check(lib.cloudsc_gpu_check(0, None, ca.VARIANT_KCACHE, None))
            out = g.outputs()
            assert bitwise_mismatches(out, oracle_outputs(oracle_mod, s, 512, 128)) == {}, s.params["nssopt"]
    finally:
        g.close()


@pytest.fixture
def forced_handoff_failure():
    """Spin limit 0: every KSEG consumer gives up without polling; 4 segments so
    that every column has hand-offs."""
    ca.kseg_schedule(4, 0)
    ca.kseg_spin_limit(0)
    yield
    ca.kseg_spin_limit(-1)
    ca.kseg_schedule(0, 0)


def test_handoff_timeout_state_api(lib, ds, forced_handoff_failure):
    # the output placement search's own KSEG launches time out too: the state is
    # still created, with its first placement (probe_final_ms < 0, no moves)
    g = ca.GpuState(ds, 2000, 64)
    try:
        rec = g.placement()
        assert rec["probe_final_ms"] < 0 and rec["moves"] == 0, rec
        rc = lib.cloudsc_state_run(g.h, ca.VARIANT_KSEG, 1, None)
        assert rc == ca.EHANDOFF, rc
        assert b"hand-off" in lib.cloudsc_last_hip_error()
        # the error was read and cleared: with the default bound the next run is clean
        ca.kseg_spin_limit(-1)
        ca.check(lib.cloudsc_state_run(g.h, ca.VARIANT_KSEG, 1, None))
        a = g.outputs()
        ca.check(lib.cloudsc_state_run(g.h, ca.VARIANT_KCACHE, 1, None))
        b = g.outputs()
        assert bitwise_mismatches(a, b) == {}
    finally:
        g.close()


def test_handoff_timeout_low_level(lib, ds, forced_handoff_failure):
    g = ca.GpuState(ds, 2000, 64)
    ws = None
    try:
        f = ca.Fields()
        ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
        p = ca.Params.from_dict(ds.params)
        ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))
        nbytes = lib.cloudsc_gpu_scratch_bytes(ca.FP64, ca.VARIANT_KSEG, 2000, 64, ds.klev)
        assert nbytes > 0
        # caller-owned device workspace, from the HIP runtime the library itself uses
        hip = C.CDLL("libamdhip64.so.7")
        ptr = C.c_void_p()
        assert hip.hipMalloc(C.byref(ptr), C.c_size_t(nbytes)) == 0
        ws = (hip, ptr)
        ca.check(lib.cloudsc_state_sync(g.h))
        # two launches, the first fails: the count accumulates until the check
        ca.check(lib.cloudsc_gpu_run(0, None, ca.FP64, ca.VARIANT_KSEG, 2000, 64, ds.klev, C.byref(f), ptr))
        ca.kseg_spin_limit(-1)
        ca.check(lib.cloudsc_gpu_run(0, None, ca.FP64, ca.VARIANT_KSEG, 2000, 64, ds.klev, C.byref(f), ptr))
        assert lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ptr) == ca.EHANDOFF
        assert lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ptr) == 0        # cleared by the read
    finally:
        if ws is not None:
            ws[0].hipFree(ws[1])
        g.close()


def test_handoff_timeout_host_pipeline(lib, ds, forced_handoff_failure):
    hp = ca.HostPipeline(ds, 1000, 64, chunk_blocks=4, nstreams=2)
    try:
        with pytest.raises(ca.CloudscError) as e:
            hp.run(ca.VARIANT_KSEG)
        assert e.value.code == ca.EHANDOFF
        ca.kseg_spin_limit(-1)
        hp.run(ca.VARIANT_KSEG)
    finally:
        hp.close()


@pytest.fixture(scope="module")
def oracle_163840_128(ds, oracle_mod):
    """The oracle (the restatement pinned bit for bit to the reference kernel,
    tests/test_oracle.py) at BASELINE.json config 2's full size: 163840
    columns, NPROMA 128."""
    return oracle_outputs(oracle_mod, ds, 163840, 128)


@pytest.mark.parametrize("variant", [ca.VARIANT_SCC, ca.VARIANT_SCC_PRIVATE, ca.VARIANT_KCACHE])
def test_bitwise_config2_full_size_vs_oracle(lib, ds, oracle_163840_128, variant):
    """BASELINE.json config 2 pinned directly: SCC fp64 with HBM temporaries
    (the a4 hoist form), SCC with per-thread private arrays (the reference CUDA
    SCC form, cloudsc_c.cu:60-317: 28.5 KB of private segment per thread) and
    the k-caching kernel, each at NGPTOT 163840 / NPROMA 128 -- all 21 fields
    bit-equal to the oracle at the same size and NPROMA (driver shape:
    src/cloudsc_cuda/cloudsc/cloudsc_driver.cu:391-397)."""
    g = ca.GpuState(ds, 163840, 128)
    try:
        out = outputs_of(g, variant)
    finally:
        g.close()
    assert bitwise_mismatches(out, oracle_163840_128) == {}


def test_bitwise_fp32_full_size(lib, ds, oracle_mod):
    """BASELINE.json config 4: SCC-k-caching fp32, NGPTOT 163840 (NPROMA 64, the
    fp32 bench default) -- KCACHE, KSEG and both SCC forms with the glibc
    expf/powf (CLOUDSC_FP32_EXACT_LIBM) bit-equal to the fp32 restatement at the
    same size, and the default float-internal forms within the tolerance gates;
    per-field relL1 vs reference.h5 (fp64) printed, and no worse than 2x the fp32
    CPU restatement's own (SURVEY.md §8c gate; fp32 is parity-unpinned beyond the
    restatement: the reference has no fp32 C kernel)."""
    n = 163840
    out = {}
    for variant in (ca.VARIANT_KCACHE, ca.VARIANT_KSEG, ca.VARIANT_SCC, ca.VARIANT_SCC_PRIVATE):
        g = ca.GpuState(ds, n, 64, ca.FP32)
        try:
            out[variant] = outputs_of(g, variant | ca.FP32_EXACT_LIBM)
            if variant == ca.VARIANT_KSEG:         # the default fp32 forms (float-internal exp/pow)
                fast = outputs_of(g, variant)
        finally:
            g.close()
    ref = oracle_outputs(oracle_mod, ds, n, 64, precision=ca.FP32)
    for variant, o in out.items():
        bad = {}
        for _, k in ca.VALIDATED:
            a = np.ascontiguousarray(o[k], dtype=np.float32).view(np.uint32)
            r = np.ascontiguousarray(ref[k], dtype=np.float32).view(np.uint32)
            m = int(np.count_nonzero(a != r))
            if m:
                bad[k] = m
        assert bad == {}, (variant, bad)
    gold = {k: np.take(ds.reference[k], np.arange(n) % ds.klon, axis=-1) for _, k in ca.VALIDATED}
    g_rep = field_report(out[ca.VARIANT_KCACHE], gold)
    c_rep = field_report(ref, gold)
    for k in g_rep:
        print("fp32 @163840 vs reference.h5 %-18s relL1 gpu %.3e cpu %.3e" % (k, g_rep[k][0], c_rep[k][0]))
        assert g_rep[k][0] <= 2.0 * c_rep[k][0] + 1e-6, k
    # BASELINE config 4 as the bench runs it: the float-internal exp/pow, gated
    # by tolerance (relL1 <= 1e-4 per field vs the restatement, <= 2x its error vs reference.h5)
    from test_gpu_parity import fp32_gates
    fp32_gates(fast, ref, gold, c_rep)


@pytest.mark.parametrize("nproma", [64, 128, 48])
def test_kseg_consecutive_launches_on_one_workspace(lib, ds, nproma):
    """A state zeroes its KSEG workspace once; later launches continue the
    ticket counter and the flag stamps (KsegEpoch, cloudsc_gpu.hip).  Many
    launches in one call, calls in a row, a schedule change (segments, grid)
    between calls, and a hand-off timeout (which makes the next call zero the
    workspace again): every result is bit-equal to KCACHE on the same state."""
    n = 20000 if nproma != 48 else 20001     # ragged last block in every case
    g = ca.GpuState(ds, n, nproma)
    try:
        ref = outputs_of(g, ca.VARIANT_KCACHE)
        assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KSEG, reps=7), ref) == {}
        assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KSEG, reps=2), ref) == {}
        for nseg, grid in ((4, 0), (3, 97), (1, 0), (0, 0)):
            ca.kseg_schedule(nseg, grid)
            try:
                assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KSEG, reps=3), ref) == {}, (nseg, grid)
            finally:
                ca.kseg_schedule(0, 0)
        ca.kseg_spin_limit(0)
        try:
            with pytest.raises(ca.CloudscError):
                g.run(ca.VARIANT_KSEG, 2)
        finally:
            ca.kseg_spin_limit(-1)
        assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KSEG, reps=3), ref) == {}
    finally:
        g.close()


@pytest.mark.parametrize("precision", [ca.FP64, ca.FP32])
def test_run_span_plain_launches(lib, ds, precision):
    """cloudsc_state_run_span (bench.py's timed region): plain dispatches timed
    as a whole give the same bits as the per-launch-event form, on a fresh
    workspace and continuing one; the span covers the launches (at least the
    sum of the shortest single launches, at most a few ms more than their
    per-launch sum); invalid arguments are refused; a hand-off timeout is
    reported the same way."""
    g = ca.GpuState(ds, 20000, 64, precision)
    try:
        span = g.run_span(ca.VARIANT_KSEG, 5)            # first call: zeroes the workspace
        first = g.outputs()
        per = g.run(ca.VARIANT_KSEG, 5)
        assert bitwise_mismatches(g.outputs(), first) == {}
        assert 5 * per.min() * 0.5 <= span <= per.sum() + 5.0, (span, per)
        assert g.run_span(ca.VARIANT_KSEG, 3) > 0
        assert bitwise_mismatches(g.outputs(), first) == {}
        assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KCACHE), first) == {}
        for v in (ca.VARIANT_KCACHE, ca.VARIANT_SCC, ca.VARIANT_SCC_PRIVATE):   # the other kernels, span-timed
            assert g.run_span(v, 2) > 0
            assert bitwise_mismatches(g.outputs(), first) == {}, v
        ms = C.c_float()
        assert lib.cloudsc_state_run_span(g.h, ca.VARIANT_KSEG, 0, C.byref(ms)) == ca.EINVAL
        assert lib.cloudsc_state_run_span(g.h, ca.VARIANT_KSEG, 2, None) == ca.EINVAL
        ca.kseg_spin_limit(0)
        try:
            with pytest.raises(ca.CloudscError):
                g.run_span(ca.VARIANT_KSEG, 2)
        finally:
            ca.kseg_spin_limit(-1)
        g.run_span(ca.VARIANT_KSEG, 2)
        assert bitwise_mismatches(g.outputs(), first) == {}
    finally:
        g.close()


def test_kseg_more_blocks_than_grid_y_limit(lib, ds):
    """KSEG at 163840 columns with NPROMA 2: 81,920 blocks, more than HIP's
    65,536 limit on a grid's y/z dimension.  The expansion and validation
    kernels run 1-D grids with 64-bit indices (the CUDA driver's gridDim.z
    quirk, SURVEY.md Appendix B item 7, cloudsc_driver.cu:391-397, avoided):
    every field bit-equal to the NPROMA-64 run, and the on-device validation
    statistics agree to the last bit with those of the NPROMA-64 state where
    the block partition does not enter (min, max, max|d|)."""
    out, stats = {}, {}
    for nproma in (64, 2):
        g = ca.GpuState(ds, 163840, nproma)
        try:
            out[nproma] = outputs_of(g, ca.VARIANT_KSEG)
            stats[nproma] = g.validate()
        finally:
            g.close()
    assert bitwise_mismatches(out[2], out[64]) == {}
    for a, b in zip(stats[2], stats[64]):
        assert a[:3] == b[:3]
        assert abs(a[3] - b[3]) <= 1e-12 * max(abs(b[3]), 1e-300) and abs(a[4] - b[4]) <= 1e-12 * abs(b[4])


def test_state_field_placement_is_transparent(lib, ds):
    """The diagnostic field placements of cloudsc_debug_set_state_layout (one
    arena with staggered fields) change where the state's fields live in HBM,
    never what the kernels compute: every field bit-equal across placements and
    across states of the default placement, KSEG and KCACHE, fp64 then fp32.
    Allocation flags are refused (profiles/r04/contiguous_alloc_hazard.txt)."""
    lib.cloudsc_debug_set_state_layout.argtypes = [C.c_longlong, C.c_uint]
    assert lib.cloudsc_debug_set_state_layout(-1, 4) == ca.EINVAL
    assert lib.cloudsc_debug_set_state_layout(100, 0) == ca.EINVAL      # misaligned stagger
    layouts = ((-1, 0), (0, 0), (-1, 0), (4608, 0), (-1, 0))
    for precision in (ca.FP64, ca.FP32):
        out = []
        try:
            for stagger, flags in layouts:
                ca.check(lib.cloudsc_debug_set_state_layout(stagger, flags))
                g = ca.GpuState(ds, 3000, 64, precision)
                try:
                    out.append(outputs_of(g, ca.VARIANT_KSEG))
                    out.append(outputs_of(g, ca.VARIANT_KCACHE))
                finally:
                    g.close()
        finally:
            ca.check(lib.cloudsc_debug_set_state_layout(-1, 0))
        # on a failure, name every run that differs from the first and the
        # 64-column blocks where it does (pcovptot: [klev][ngptot])
        diff = {}
        for j in range(1, len(out)):
            bad = bitwise_mismatches(out[0], out[j])
            if bad:
                d = out[0]["pcovptot"] != out[j]["pcovptot"]
                cols = np.nonzero(d.any(axis=0))[0]
                levs = np.nonzero(d.any(axis=1))[0]
                diff[(layouts[j // 2], j, "KSEG" if j % 2 == 0 else "KCACHE")] = (
                    sorted(bad), sorted(set((cols // 64).tolist())),
                    (int(levs.min()), int(levs.max())) if levs.size else None)
        assert diff == {}, (precision, diff)


def test_state_buffer_relocation_is_transparent(lib, ds):
    """The slow-state diagnostics (tools/slow_state_diag.py) move a live state's
    workspace, pristine plude copy and fields to fresh memory: the next KSEG run
    zeroes the moved workspace and every output stays bit-equal.  A buffer the
    state does not hold yet (the SCC temporaries before an SCC run) and unknown
    selectors are refused."""
    lib.cloudsc_debug_state_relocate_aux.argtypes = [C.c_void_p, C.c_int]
    lib.cloudsc_debug_state_relocate_field.argtypes = [C.c_void_p, C.c_int]
    names = [f[0] for f in ca.Fields._fields_]
    g = ca.GpuState(ds, 5000, 64)
    try:
        ref = outputs_of(g, ca.VARIANT_KSEG, reps=2)
        assert lib.cloudsc_debug_state_relocate_aux(g.h, 2) == ca.EINVAL      # no SCC scratch yet
        assert lib.cloudsc_debug_state_relocate_aux(g.h, 3) == ca.EINVAL
        assert lib.cloudsc_debug_state_relocate_aux(None, 0) == ca.EINVAL
        for which in (1, 0):                                                  # workspace, pristine plude
            ca.check(lib.cloudsc_debug_state_relocate_aux(g.h, which))
            assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KSEG, reps=2), ref) == {}, which
        for name in ("pt", "paph", "tendency_loc_cld", "pfplsn", "plude"):
            ca.check(lib.cloudsc_debug_state_relocate_field(g.h, names.index(name)))
        assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KSEG, reps=2), ref) == {}
        assert bitwise_mismatches(outputs_of(g, ca.VARIANT_KCACHE), ref) == {}
    finally:
        g.close()


@pytest.mark.parametrize("precision", [ca.FP64, ca.FP32])
def test_output_placement_search(lib, ds, precision):
    """The output placement search at state creation (cloudsc_state_placement)
    moves output buffers before anything is written to them: a state created
    with it (the default, and with 4 passes) computes exactly what a state
    created without it computes, KSEG and KCACHE; its record is consistent
    (the kept time no worse than the first, moves <= tries), and with the
    search off the record is all zero."""
    assert lib.cloudsc_debug_set_placement_search(9) == ca.EINVAL
    out, rec = [], []
    try:
        for passes in (0, -1, 4):
            ca.check(lib.cloudsc_debug_set_placement_search(passes))
            g = ca.GpuState(ds, 3000, 64, precision)
            try:
                rec.append(g.placement())
                out.append(outputs_of(g, ca.VARIANT_KSEG))
                out.append(outputs_of(g, ca.VARIANT_KCACHE))
            finally:
                g.close()
    finally:
        ca.check(lib.cloudsc_debug_set_placement_search(-1))
    for j in range(1, len(out)):
        assert bitwise_mismatches(out[0], out[j]) == {}, j
    assert rec[0] == {"probe_first_ms": 0.0, "probe_final_ms": 0.0, "tries": 0, "moves": 0}
    for r in rec[1:]:
        assert 0 < r["probe_final_ms"] <= r["probe_first_ms"]
        assert 0 <= r["moves"] <= r["tries"] and r["tries"] >= 21


@pytest.mark.parametrize("precision", [ca.FP64, ca.FP32])
def test_kseg_shared_workspace_alternating_states(lib, ds, precision):
    """Two states with different inputs (B = the template's columns rotated by
    half, so every block carries other values between its segments) run
    alternately through cloudsc_gpu_run on ONE caller-owned KSEG workspace.
    Each launch finds the other state's carried values in the hand-off slots:
    a consumer that read its slot before the producer's values were visible
    would differ.  Every launch bit-equal to that state's own state-API run
    (tools/handoff_stress.py is the long form)."""
    ngptot, nproma = 3000, 64
    ds_b = ds.copy()
    for k, v in ds_b.inputs.items():
        if v.ndim >= 1 and v.shape[-1] == ds.klon:
            ds_b.inputs[k] = np.ascontiguousarray(np.roll(v, ds.klon // 2, axis=-1))
    states = [ca.GpuState(d, ngptot, nproma, precision) for d in (ds, ds_b)]
    hip = C.CDLL("libamdhip64.so.7")
    ws = C.c_void_p()
    try:
        refs = [outputs_of(g, ca.VARIANT_KSEG) for g in states]
        assert bitwise_mismatches(refs[0], refs[1]) != {}
        fields = []
        for g in states:
            f = ca.Fields()
            ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
            fields.append(f)
        p = ca.Params.from_dict(ds.params)
        ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))
        nbytes = lib.cloudsc_gpu_scratch_bytes(precision, ca.VARIANT_KSEG, ngptot, nproma, ds.klev)
        assert hip.hipMalloc(C.byref(ws), C.c_size_t(nbytes)) == 0
        for it in range(6):
            i = it & 1
            ca.check(lib.cloudsc_state_reset(states[i].h))     # plude from the pristine copy
            ca.check(lib.cloudsc_state_sync(states[i].h))
            ca.check(lib.cloudsc_gpu_run(0, None, precision, ca.VARIANT_KSEG, ngptot, nproma, ds.klev,
                                         C.byref(fields[i]), ws))
            ca.check(lib.cloudsc_gpu_check(0, None, ca.VARIANT_KSEG, ws))
            assert bitwise_mismatches(states[i].outputs(), refs[i]) == {}, (it, i)
    finally:
        if ws.value:
            hip.hipFree(ws)
        for g in states:
            g.close()


# ---- caller-owned device fields with a placement search (cloudsc_fields_alloc, round 5) ----
def device_outputs(df, ngptot):
    return {k: ca.blocks_to_columns(df.download(k), ngptot) for _, k in ca.VALIDATED}


@pytest.mark.parametrize("precision,variant", [(ca.FP64, ca.VARIANT_KSEG), (ca.FP64, ca.VARIANT_KCACHE),
                                               (ca.FP32, ca.VARIANT_KSEG)])
def test_fields_alloc_reference_driver_shape(lib, ds, precision, variant):
    """The reference CUDA driver's shape on caller-owned buffers: allocate every
    field (cloudsc_fields_alloc, placed by the memory-pattern search), copy the
    host block-layout inputs in, cloudsc_gpu_run, copy the outputs out -- bit
    for bit what the state API computes.  The search's record is consistent,
    and cloudsc_fields_free releases every buffer it made."""
    ngptot, nproma = 3000, 64
    ref = outputs_of_state(ds, ngptot, nproma, precision, variant)
    df = ca.DeviceFields(ngptot, nproma, ds.klev, precision)
    ws = C.c_void_p()
    hip = C.CDLL("libamdhip64.so.7")
    try:
        r = df.report.to_dict()
        assert r["method"] == "rw-probe" and r["launches"] >= 30 and r["search_ms"] > 0, r
        assert 0 < r["probe_final_ms"] <= r["probe_first_ms"] and 0 <= r["moves"] <= r["tries"], r
        assert r["tries"] >= 21 and r["peak_transient_bytes"] > 0, r
        # the transient footprint stays within what the free-memory check was made for
        assert 0 < r["peak_transient_bytes"] <= r["transient_budget_bytes"], r
        # every field allocated, aerosols only on request
        assert all(getattr(df.f, n) for n in list(ca.INPUT_FIELDS) + list(ca.OUTPUT_FIELDS) + ["plude"])
        assert not any(getattr(df.f, n) for n in ca.AEROSOL_FIELDS)
        st = ca.make_host_state(ds, ngptot, nproma, precision)
        df.upload({k: v for k, v in st.arrays.items() if k in ca.INPUT_FIELDS or k == "plude"})
        p = ca.Params.from_dict(ds.params)
        ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))
        nbytes = lib.cloudsc_gpu_scratch_bytes(precision, variant, ngptot, nproma, ds.klev)
        if nbytes > 0:
            assert hip.hipMalloc(C.byref(ws), C.c_size_t(nbytes)) == 0
            assert hip.hipMemset(ws, 0, C.c_size_t(256)) == 0
        ca.check(lib.cloudsc_gpu_run(0, None, precision, variant, ngptot, nproma, ds.klev, C.byref(df.f), ws))
        ca.check(lib.cloudsc_gpu_check(0, None, variant, ws))
        assert bitwise_mismatches(device_outputs(df, ngptot), ref) == {}
    finally:
        if ws.value:
            hip.hipFree(ws)
        df.close()
    assert df.f is None


def outputs_of_state(ds, ngptot, nproma, precision, variant):
    g = ca.GpuState(ds, ngptot, nproma, precision)
    try:
        return outputs_of(g, variant)
    finally:
        g.close()


def test_fields_alloc_flags_and_free(lib, ds):
    """CLOUDSC_PLACE_NONE: no search, record zero; CLOUDSC_ALLOC_AEROSOLS
    allocates the five aerosol inputs; unknown flags and foreign pointers are
    refused; a state reports its own search with its cost."""
    f, r = ca.Fields(), ca.Placement()
    assert lib.cloudsc_fields_alloc(0, ca.FP64, 1000, 128, ds.klev, 4, C.byref(f), C.byref(r)) == ca.EINVAL
    ca.check(lib.cloudsc_fields_alloc(0, ca.FP64, 1000, 128, ds.klev, ca.PLACE_NONE | ca.ALLOC_AEROSOLS,
                                      C.byref(f), C.byref(r)))
    try:
        assert r.to_dict()["method"] == "none" and r.launches == 0 and r.tries == 0
        assert all(getattr(f, n) for n in ca.AEROSOL_FIELDS)
        own = f.pt
        g = ca.GpuState(ds, 1000, 128)
        try:
            foreign = ca.Fields()
            ca.check(lib.cloudsc_state_fields(g.h, C.byref(foreign)))
            f2 = ca.Fields(pt=foreign.pt)
            assert lib.cloudsc_fields_free(0, C.byref(f2)) == ca.EINVAL and f2.pt == foreign.pt
            rep = g.placement_report()
            assert rep["method"] == "kernel" and rep["launches"] > 0 and rep["search_ms"] > 0, rep
            assert 0 < rep["peak_transient_bytes"] <= rep["transient_budget_bytes"], rep
        finally:
            g.close()
        assert own
    finally:
        ca.check(lib.cloudsc_fields_free(0, C.byref(f)))
    assert not f.pt and not f.pfhpsn


# ---- round 6: the layout probe's addressing and cloudsc_host_run's profile ----
def _layout_module():
    import importlib.util
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools", "layout_corr.py")
    spec = importlib.util.spec_from_file_location("layout_corr", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("layout", ["B", "I"])
def test_memory_probe_layout_writes_exactly_its_elements(lib, layout):
    """cloudsc_debug_memory_probe_layout (the round-6 layout study's
    instrument, tools/layout_corr.py) over a per-block (B) or per-row (I)
    interleaved output arena: every output element the layout addresses holds
    the probe's value (block + level), and every other byte of the arena keeps
    its sentinel -- the strides keep each field inside its own chunk, with no
    overlap and no stray store.  200 columns, NPROMA 64 (a partial last block),
    KLEV 7."""
    lc = _layout_module()
    ngptot, nproma, klev = 200, 64, 7
    nblocks = (ngptot + nproma - 1) // nproma
    hip = lc.Hip()
    f, strides, owned = lc.arena_set(hip, layout, nblocks, nproma, klev, 8)
    h = hip.h
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    out_arena = owned[1]
    rows = klev + 1
    if layout == "B":
        nbytes = nblocks * strides[3] * 8
        base = out_arena
    else:
        nbytes = (nblocks * rows + 1) * strides[4] * 8
        base = out_arena
    sentinel = np.full(nbytes // 8, -7.5)
    assert h.hipMemcpy(base, sentinel.ctypes.data, nbytes, 1) == 0
    lib.cloudsc_debug_memory_probe_layout.argtypes = [C.c_int] * 5 + [C.POINTER(ca.Fields), C.c_int, C.c_int,
                                                      C.POINTER(C.c_longlong), C.POINTER(C.c_float)]
    ms = C.c_float()
    ca.check(lib.cloudsc_debug_memory_probe_layout(0, ca.FP64, ngptot, nproma, klev, C.byref(f), 0, 1,
                                                   (C.c_longlong * 6)(*strides), C.byref(ms)))
    got = np.empty(nbytes // 8)
    assert h.hipMemcpy(got.ctypes.data, base, nbytes, 2) == 0
    expect = sentinel.copy()
    bs, rs, ss = strides[3:6]
    e0 = lambda p: (p - base) // 8   # noqa: E731  element offset of a field pointer in the arena
    for b in range(nblocks):
        lanes = min(nproma, ngptot - b * nproma)
        for k in range(klev):
            v = float(b + k)
            for n in lc.OUT_LEVEL:
                o = e0(getattr(f, n)) + b * bs + k * rs
                expect[o:o + lanes] = v
            for m in range(5):
                o = e0(f.tendency_loc_cld) + b * bs + m * ss + k * rs
                expect[o:o + lanes] = v
            for n in lc.OUT_HALF:
                o = e0(getattr(f, n)) + b * bs + (k + 1) * rs
                expect[o:o + lanes] = v
        for n in lc.OUT_HALF:       # half level 0
            o = e0(getattr(f, n)) + b * bs
            expect[o:o + lanes] = float(b)
    assert np.array_equal(got, expect)
    for p in owned:
        h.hipFree(C.c_void_p(p))


def test_host_run_profile_accounts_for_each_call(lib, ds):
    """cloudsc_host_run_profile: after enabling it, N calls of cloudsc_host_run
    on one thread count as the context's first call (apart) or as profiled
    calls; the parts of the profiled calls add up to their total, and the
    device's three operations fit in the enqueue + wait span.  Results are the
    unprofiled ones, bit for bit."""
    class Prof(C.Structure):
        _fields_ = [("calls", C.c_longlong)] + [(n, C.c_double) for n in (
            "setup_ms", "pack_ms", "h2d_ms", "kernel_ms", "d2h_ms", "wait_ms", "unpack_ms", "total_ms", "alloc_ms",
            "enqueue_ms", "max_call_ms")] + [("first_calls", C.c_longlong), ("first_calls_ms", C.c_double)]
    lib.cloudsc_host_run_profile.argtypes = [C.c_int, C.POINTER(Prof)]
    ncols, nproma = 300, 64
    p = ca.Params.from_dict(ds.params)
    outs = []
    for prof in (False, True):
        st = ca.make_host_state(ds, ncols, nproma, ca.FP64)
        f = st.fields()
        if prof:
            ca.check(lib.cloudsc_host_run_profile(1, None))
        plude0 = st.arrays["plude"].copy()
        for _ in range(4):
            np.copyto(st.arrays["plude"], plude0)
            ca.check(lib.cloudsc_host_run(0, ca.FP64, ca.VARIANT_KSEG, ncols, nproma, ds.klev, C.byref(p), C.byref(f)))
        outs.append({k: st.arrays[k].copy() for k in ca.OUTPUT_FIELDS if k in st.arrays})
        if prof:
            r = Prof()
            ca.check(lib.cloudsc_host_run_profile(-1, C.byref(r)))
    # the unprofiled calls above created this thread's context: all 4 profiled calls count as calls
    assert r.calls == 4 and r.first_calls == 0
    parts = r.alloc_ms + r.setup_ms + r.pack_ms + r.enqueue_ms + r.wait_ms + r.unpack_ms
    assert abs(parts - r.total_ms) <= 0.01 * r.total_ms + 0.2, (parts, r.total_ms)
    assert 0 < r.kernel_ms and r.h2d_ms + r.kernel_ms + r.d2h_ms <= r.enqueue_ms + r.wait_ms + 0.2
    assert r.max_call_ms <= r.total_ms
    assert all(np.array_equal(outs[0][k].view(np.uint8), outs[1][k].view(np.uint8)) for k in outs[0])
    # profiling is off again: the sums no longer move
    st = ca.make_host_state(ds, ncols, nproma, ca.FP64)
    ca.check(lib.cloudsc_host_run(0, ca.FP64, ca.VARIANT_KSEG, ncols, nproma, ds.klev, C.byref(p),
                                  C.byref(st.fields())))
    r2 = Prof()
    ca.check(lib.cloudsc_host_run_profile(0, C.byref(r2)))
    assert r2.calls == r.calls and r2.total_ms == r.total_ms
