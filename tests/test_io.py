"""Host plumbing of the dwarf driver (no GPU): the C dataset readers/writer of
dwarf-p-cloudsc_amd/csrc/cloudsc_io.c through libcloudsc_io.so, and the
dwarf-cloudsc-amd CLI paths that need no device.

Pinned against the reference's own files: data/cloudsc100 holds the
Serialbox arrays of the reference's data/, tests/golden/reference.h5 is
config-files/reference.h5.  The HDF5 writer must reproduce that file exactly
from the raw arrays (the input.h5 regeneration tool of SURVEY.md §8f-1)."""
import ctypes as C
import os
import shutil
import stat
import subprocess

import numpy as np
import pytest

import cloudsc_amd as ca

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dwarf-p-cloudsc_amd")
IO_LIB = os.path.join(PKG, "libcloudsc_io.so")
DWARF = os.path.join(PKG, "dwarf-cloudsc-amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
DATA = os.path.join(REPO, "data", "cloudsc100")
REF_H5_UPSTREAM = "/root/reference/config-files/reference.h5"

NIN = 28
INPUT_NAMES = ["pt", "pq", "tendency_tmp_t", "tendency_tmp_q", "tendency_tmp_a", "tendency_tmp_cld", "pvfl",
               "pvfi", "phrsw", "phrlw", "pvervel", "pap", "paph", "plsm", "ktype", "plu", "plude", "psnde",
               "pmfu", "pmfd", "pa", "pclv", "psupsat", "plcrit_aer", "picrit_aer", "pre_ice", "pccn", "pnice"]


class Dataset(C.Structure):
    _fields_ = [("klon", C.c_int), ("klev", C.c_int), ("params", ca.Params),
                ("inp", C.POINTER(C.c_double) * NIN), ("ktype", C.POINTER(C.c_int)),
                ("ref", C.POINTER(C.c_double) * 21), ("has_reference", C.c_int), ("source", C.c_char * 512)]


@pytest.fixture(scope="module")
def io():
    # the CLI links libcloudsc_amd.so; building it is __graft_entry__.build()'s job
    if not os.path.exists(IO_LIB):
        subprocess.check_call(["make", "-s", "-C", PKG, "libcloudsc_io.so"])
    lib = C.CDLL(IO_LIB)
    lib.cloudsc_io_load_raw.argtypes = [C.c_char_p, C.c_int, C.POINTER(Dataset)]
    lib.cloudsc_io_load_serialbox.argtypes = [C.c_char_p, C.c_int, C.POINTER(Dataset)]
    lib.cloudsc_io_load_dir.argtypes = [C.c_char_p, C.c_int, C.POINTER(Dataset)]
    lib.cloudsc_io_load_hdf5.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(Dataset)]
    lib.cloudsc_io_load_hdf5_reference.argtypes = [C.c_char_p, C.POINTER(Dataset)]
    lib.cloudsc_io_write_hdf5.argtypes = [C.POINTER(Dataset), C.c_char_p, C.c_char_p]
    lib.cloudsc_io_free.argtypes = [C.POINTER(Dataset)]
    lib.cloudsc_io_last_error.restype = C.c_char_p
    return lib


def need_hdf5(io):
    if not io.cloudsc_io_hdf5_available():
        pytest.skip("no libhdf5 on this host: %s" % io.cloudsc_io_last_error().decode())


def arrays(d: Dataset):
    """numpy copies of a loaded dataset, keyed like cloudsc_amd.Dataset"""
    klev, klon = d.klev, d.klon
    kinds = {**ca.INPUT_FIELDS, **ca.AEROSOL_FIELDS, **ca.INOUT_FIELDS}
    inp = {}
    for i, name in enumerate(INPUT_NAMES):
        shp = ca.field_shape(kinds[name], klev, klon)
        n = int(np.prod(shp))
        if name == "ktype":
            if d.ktype:
                inp[name] = np.ctypeslib.as_array(d.ktype, (n,)).reshape(shp).copy()
        elif d.inp[i]:
            inp[name] = np.ctypeslib.as_array(d.inp[i], (n,)).reshape(shp).copy()
    ref = {}
    for i, (_, key) in enumerate(ca.VALIDATED):
        if d.ref[i]:
            shp = ca.field_shape(ca.ALL_FIELDS[key], klev, klon)
            ref[key] = np.ctypeslib.as_array(d.ref[i], (int(np.prod(shp)),)).reshape(shp).copy()
    return inp, ref


def load_raw(io, path=DATA):
    d = Dataset()
    rc = io.cloudsc_io_load_raw(path.encode(), 1, C.byref(d))
    assert rc == 0, io.cloudsc_io_last_error()
    return d


def test_raw_reader_matches_python_loader(io, ds):
    d = load_raw(io)
    try:
        assert (d.klon, d.klev) == (ds.klon, ds.klev)
        inp, ref = arrays(d)
        for k, v in ds.inputs.items():
            assert np.array_equal(inp[k], v), k
        for k, v in ds.reference.items():
            assert np.array_equal(ref[k], v), k
        assert d.params.to_dict() == ca.Params.from_dict(ds.params).to_dict()
    finally:
        io.cloudsc_io_free(C.byref(d))


def test_raw_reader_errors(io, tmp_path):
    d = Dataset()
    assert io.cloudsc_io_load_raw(str(tmp_path).encode(), 1, C.byref(d)) == -6     # no manifest
    shutil.copytree(DATA, tmp_path / "ds")
    with open(tmp_path / "ds" / "input_PT.dat", "r+b") as fh:                     # truncated field
        fh.truncate(100)
    assert io.cloudsc_io_load_raw(str(tmp_path / "ds").encode(), 1, C.byref(d)) == -6
    assert b"input_PT.dat" in io.cloudsc_io_last_error()


def test_hdf5_writer_reproduces_reference_h5(io, tmp_path):
    """Raw arrays -> reference.h5 through our writer == the reference's file."""
    need_hdf5(io)
    d = load_raw(io)
    try:
        out = tmp_path / "reference.h5"
        assert io.cloudsc_io_write_hdf5(C.byref(d), None, str(out).encode()) == 0, io.cloudsc_io_last_error()
        for fixture in (os.path.join(GOLDEN, "reference.h5"), REF_H5_UPSTREAM):
            if not os.path.exists(fixture):
                continue
            h5diff = shutil.which("h5diff") or "/opt/conda/bin/h5diff"
            if os.path.exists(h5diff):
                r = subprocess.run([h5diff, str(out), fixture], capture_output=True, text=True)
                assert r.returncode == 0, r.stdout[-2000:]
            # and through our own read-only reader
            e = Dataset()
            e.klon, e.klev = d.klon, d.klev
            assert io.cloudsc_io_load_hdf5_reference(fixture.encode(), C.byref(e)) == 0
            _, ref_a = arrays(d)
            _, ref_b = arrays(e)
            for k in ref_a:
                assert np.array_equal(ref_a[k], ref_b[k]), k
            io.cloudsc_io_free(C.byref(e))
    finally:
        io.cloudsc_io_free(C.byref(d))


def test_hdf5_input_roundtrip_readonly(io, tmp_path):
    """input.h5 written from the raw state reads back identically, from a
    read-only file (the C reference opens it RDWR: load_state.c:499)."""
    need_hdf5(io)
    d = load_raw(io)
    try:
        inp_h5, ref_h5 = tmp_path / "input.h5", tmp_path / "reference.h5"
        assert io.cloudsc_io_write_hdf5(C.byref(d), str(inp_h5).encode(), str(ref_h5).encode()) == 0
        for p in (inp_h5, ref_h5):
            os.chmod(p, stat.S_IRUSR | stat.S_IRGRP | stat.S_IROTH)
        e = Dataset()
        rc = io.cloudsc_io_load_hdf5(str(inp_h5).encode(), str(ref_h5).encode(), C.byref(e))
        assert rc == 0, io.cloudsc_io_last_error()
        a_in, a_ref = arrays(d)
        b_in, b_ref = arrays(e)
        assert a_in.keys() == b_in.keys() and a_ref.keys() == b_ref.keys()
        for k in a_in:
            assert np.array_equal(a_in[k], b_in[k]), k
        for k in a_ref:
            assert np.array_equal(a_ref[k], b_ref[k]), k
        assert d.params.to_dict() == e.params.to_dict()
        assert b"read-only" in e.source
        io.cloudsc_io_free(C.byref(e))
    finally:
        io.cloudsc_io_free(C.byref(d))


def test_hdf5_missing_dataset_reported(io, tmp_path):
    need_hdf5(io)
    d = load_raw(io)
    try:
        ref_only = tmp_path / "r.h5"
        assert io.cloudsc_io_write_hdf5(C.byref(d), None, str(ref_only).encode()) == 0
        e = Dataset()
        # a reference file is not an input file: KLON exists, PT does not
        assert io.cloudsc_io_load_hdf5(str(ref_only).encode(), None, C.byref(e)) == -6
        assert b"/PT" in io.cloudsc_io_last_error()
        assert io.cloudsc_io_load_hdf5(str(tmp_path / "nope.h5").encode(), None, C.byref(e)) == -6
    finally:
        io.cloudsc_io_free(C.byref(d))


def test_cli_argument_errors():
    """dwarf_cloudsc.c:45-48: wrong argument count -> message, EXIT_FAILURE;
    needs no device."""
    if not os.path.exists(DWARF):
        pytest.skip("dwarf-cloudsc-amd not built (needs libcloudsc_amd.so: __graft_entry__.build())")
    r = subprocess.run([DWARF, "1", "100"], capture_output=True, text=True)
    assert r.returncode == 1 and "right number of arguments" in r.stdout
    # nproma > 256 with a one-workgroup-per-block variant (KSEG takes any NPROMA)
    r = subprocess.run([DWARF, "--variant", "kcache", "1", "100", "300"], capture_output=True, text=True)
    assert r.returncode == 1 and "invalid sizes" in r.stderr
    r = subprocess.run([DWARF, "--variant", "nope"], capture_output=True, text=True)
    assert r.returncode == 1


def test_cli_write_h5(tmp_path, io):
    """dwarf-cloudsc-amd --write-h5 regenerates input.h5 + reference.h5 (no device)."""
    need_hdf5(io)
    if not os.path.exists(DWARF):
        pytest.skip("dwarf-cloudsc-amd not built")
    r = subprocess.run([DWARF, "--write-h5", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "input.h5").exists() and (tmp_path / "reference.h5").exists()


def test_host_expand_and_stats_match_python(io, ds):
    """cloudsc_io_expand / cloudsc_io_field_stats (the host-buffer path of the
    driver) == the numpy plumbing (ca.expand, ca.field_stats)."""
    io.cloudsc_io_expand.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_longlong, C.c_int, C.c_void_p]
    io.cloudsc_io_field_stats.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                          C.c_int, C.c_longlong, C.POINTER(ca.Stats)]
    kind_id = {"2d": 0, "2dh": 1, "3d": 2, "1d": 3}
    ngptot, nproma, off = 1000, 128, 37
    for name in ("pt", "paph", "pclv", "plsm", "ktype"):
        src = np.ascontiguousarray(ds.inputs[name])
        kind = ca.ALL_FIELDS[name]
        is_int = name == "ktype"
        for es, dt in ((8, np.float64), (4, np.float32)):
            want = ca.expand(src, kind, ngptot, nproma, off, dtype=np.int32 if is_int else dt)
            got = np.empty_like(want)
            io.cloudsc_io_expand(src.ctypes.data, kind_id[kind], int(is_int), ds.klev, ds.klon, ngptot, nproma,
                                 off, 4 if is_int else es, got.ctypes.data)
            assert np.array_equal(got, want), (name, es)
    for _, key in ca.VALIDATED[:6]:
        ref = np.ascontiguousarray(ds.reference[key])
        kind = ca.ALL_FIELDS[key]
        fld = ca.expand(ref * (1 + 1e-9), kind, ngptot, nproma, 0)
        st = ca.Stats()
        io.cloudsc_io_field_stats(ref.ctypes.data, kind_id[kind], ds.klev, ds.klon, fld.ctypes.data, 8, ngptot,
                                  nproma, 0, C.byref(st))
        want = ca.field_stats(ca.blocks_to_columns(fld, ngptot), np.take(ref, np.arange(ngptot) % 100, axis=-1))
        got = (st.minval, st.maxval, st.maxerr, st.errsum, st.refsum)
        assert got[:3] == tuple(want[:3]), key
        assert got[3] == pytest.approx(want[3], rel=1e-12) and got[4] == pytest.approx(want[4], rel=1e-12), key


# ---- Serialbox store (the reference's data/ directory) ----
REF_DATA_UPSTREAM = "/root/reference/data"


def load_serialbox(io, path):
    d = Dataset()
    rc = io.cloudsc_io_load_serialbox(path.encode(), 1, C.byref(d))
    assert rc == 0, io.cloudsc_io_last_error()
    return d


def assert_same_dataset(a: Dataset, b: Dataset):
    assert (a.klon, a.klev) == (b.klon, b.klev)
    ia, ra = arrays(a)
    ib, rb = arrays(b)
    assert sorted(ia) == sorted(ib) and sorted(ra) == sorted(rb)
    for k in ia:
        assert ia[k].dtype == ib[k].dtype and np.array_equal(ia[k], ib[k]), k
    for k in ra:
        assert np.array_equal(ra[k], rb[k]), k
    pa, pb = a.params.to_dict(), b.params.to_dict()
    assert pa == pb, {k: (pa[k], pb[k]) for k in pa if pa[k] != pb[k]}


def test_serialbox_reader_equals_committed_conversion(io):
    """data/cloudsc100 is a Serialbox store (the reference's MetaData-*.json,
    ArchiveMetaData-*.json and .dat arrays): reading it natively gives exactly the
    dataset of the committed conversion (manifest.json + params.txt), every array
    and every parameter bit for bit (serialbox2hdf5/serialbox2hdf5.py:11-33 is the
    reference's converter; load_state.c:538-690 its reader of the result)."""
    a, b = load_serialbox(io, DATA), load_raw(io, DATA)
    try:
        assert_same_dataset(a, b)
        assert a.has_reference and b"Serialbox" in a.source
    finally:
        io.cloudsc_io_free(C.byref(a))
        io.cloudsc_io_free(C.byref(b))


def test_serialbox_reader_on_the_reference_data_dir(io):
    """`--data /root/reference/data`: the reference's own directory, unconverted."""
    if not os.path.exists(os.path.join(REF_DATA_UPSTREAM, "MetaData-input.json")):
        pytest.skip("no reference checkout")
    a, b = load_serialbox(io, REF_DATA_UPSTREAM), load_raw(io, DATA)
    try:
        ia, _ = arrays(a)
        # the reference directory also holds the two aerosol inputs the kernel never reads
        assert {"plcrit_aer", "pccn"} <= set(ia)
        for k in ("plcrit_aer", "pccn"):
            a.inp[INPUT_NAMES.index(k)] = C.POINTER(C.c_double)()
        assert_same_dataset(a, b)
    finally:
        io.cloudsc_io_free(C.byref(b))


def test_load_dir_dispatch_and_errors(io, tmp_path):
    d = Dataset()
    assert io.cloudsc_io_load_dir(DATA.encode(), 1, C.byref(d)) == 0
    assert b"Serialbox" in d.source
    io.cloudsc_io_free(C.byref(d))
    shutil.copytree(DATA, tmp_path / "sb")
    # a field whose metadata disagrees with the file / the expected shape is rejected
    with open(tmp_path / "sb" / "input_PAP.dat", "r+b") as fh:
        fh.truncate(800)
    assert io.cloudsc_io_load_serialbox(str(tmp_path / "sb").encode(), 1, C.byref(d)) == -6
    assert b"input_PAP.dat" in io.cloudsc_io_last_error()
    # a missing parameter scalar is an error, not a silent zero
    import json
    shutil.copy(os.path.join(DATA, "input_PAP.dat"), tmp_path / "sb" / "input_PAP.dat")
    meta = json.load(open(tmp_path / "sb" / "MetaData-input.json"))
    del meta["global_meta_info"]["YRECLDP_RTHOMO"]
    os.chmod(tmp_path / "sb" / "MetaData-input.json", 0o644)
    json.dump(meta, open(tmp_path / "sb" / "MetaData-input.json", "w"))
    assert io.cloudsc_io_load_serialbox(str(tmp_path / "sb").encode(), 1, C.byref(d)) == -6
    assert b"YRECLDP_RTHOMO" in io.cloudsc_io_last_error()


def test_python_loader_reads_serialbox(ds):
    """cloudsc_amd.load_dataset reads the Serialbox metadata too: same parameters
    as params.txt (the committed conversion)."""
    txt = ca.read_params_txt(os.path.join(DATA, "params.txt"))
    sb = ca.read_serialbox_params(DATA)
    assert txt == sb
    assert ds.params == sb


def _corruptions(seed=20261016):
    """(file, description, mutator(bytes) -> bytes) for the metadata and data files."""
    import random
    rng = random.Random(seed)
    cases = []
    for name in ("MetaData-input.json", "ArchiveMetaData-input.json", "MetaData-reference.json",
                 "ArchiveMetaData-reference.json", "manifest.json"):
        size = os.path.getsize(os.path.join(DATA, name))
        for frac in (0.0, 0.1, 0.5, 0.9, 0.999):
            n = int(size * frac)
            cases.append((name, "truncated at %d" % n, lambda b, n=n: b[:n]))
        for _ in range(4):
            pos = rng.randrange(size)
            junk = bytes(rng.choice(b'{}[]":,0123456789-eE.xyz \x00\xff') for _ in range(rng.randint(1, 8)))
            cases.append((name, "junk at %d" % pos, lambda b, pos=pos, junk=junk: b[:pos] + junk + b[pos + len(junk):]))
        cases.append((name, "digits doubled", lambda b: b.replace(b"1", b"11")))
        cases.append((name, "numbers as strings", lambda b: b.replace(b": 1", b': "1"')))
        cases.append((name, "empty", lambda b: b""))
        # cut exactly inside a number and inside a literal: the parser's
        # look-ahead (strtod, the true/false/null compares) must stop at the end
        # of the buffer, which has no NUL terminator
        digits = [i for i in range(1, size) if chr(open(os.path.join(DATA, name), "rb").read()[i - 1]).isdigit()]
        for n in (digits[len(digits) // 2], digits[-1]) if digits else ():
            cases.append((name, "truncated after a digit at %d" % n, lambda b, n=n: b[:n]))
        cases.append((name, "ends in 'tr'", lambda b: b[:max(0, len(b) // 2)] + b' "x": tr'))
        cases.append((name, "ends in 'fals'", lambda b: b[:max(0, len(b) // 3)] + b'[fals'))
        cases.append((name, "ends in a long number", lambda b: b[:len(b) // 4] + b"1" * 200))
    for name in ("input_PT.dat", "input_KTYPE.dat", "input_PCLV.dat", "reference_PLUDE.dat"):
        cases.append((name, "empty", lambda b: b""))
        cases.append((name, "one byte more", lambda b: b + b"\x00"))
        cases.append((name, "one value less", lambda b: b[:-8]))
    return cases


def test_readers_survive_corrupted_metadata(io, tmp_path):
    """I/O hardening: every reader returns 0 or CLOUDSC_EIO (-6)
    with a message -- never a crash -- on truncated, garbled, empty and
    mis-sized metadata and data files (each case in a child process, so a
    crash is seen as a signal)."""
    import sys
    child = os.path.join(REPO, "tests", "io_fuzz_child.py")
    base = tmp_path / "sb"
    shutil.copytree(DATA, base)
    for p in base.iterdir():
        os.chmod(p, 0o644)
    bad = []
    for name, what, mutate in _corruptions():
        f = base / name
        orig = f.read_bytes()
        try:
            f.write_bytes(mutate(orig))
            r = subprocess.run([sys.executable, child, str(base)], capture_output=True, text=True, timeout=120)
            rcs = r.stdout.split()
            if r.returncode != 0 or len(rcs) != 3 or any(x not in ("0", "-6") for x in rcs):
                bad.append((name, what, r.returncode, r.stdout.strip(), r.stderr.strip()[-300:]))
        finally:
            f.write_bytes(orig)
    assert bad == [], bad[:5]


def test_hdf5_reader_survives_corrupted_files(io, tmp_path):
    """The read-only HDF5 reader on truncated and bit-flipped input.h5 /
    reference.h5: 0 or CLOUDSC_EIO, never a crash (child process per case)."""
    import random
    import sys
    need_hdf5(io)
    child = os.path.join(REPO, "tests", "io_fuzz_child.py")
    d = load_raw(io)
    try:
        inp, ref = tmp_path / "input.h5", tmp_path / "reference.h5"
        assert io.cloudsc_io_write_hdf5(C.byref(d), str(inp).encode(), str(ref).encode()) == 0
    finally:
        io.cloudsc_io_free(C.byref(d))
    rng = random.Random(7)
    bad = []
    for target in (inp, ref):
        orig = target.read_bytes()
        cases = [("truncated at %d" % n, orig[:n]) for n in (0, 100, 2048, len(orig) // 2, len(orig) - 1)]
        for _ in range(8):
            pos = rng.randrange(len(orig))
            cases.append(("byte %d flipped" % pos, orig[:pos] + bytes([orig[pos] ^ 0xFF]) + orig[pos + 1:]))
        for what, data in cases:
            target.write_bytes(data)
            r = subprocess.run([sys.executable, child, "--hdf5", str(inp), str(ref)], capture_output=True, text=True,
                               timeout=120)
            if r.returncode != 0 or r.stdout.strip() not in ("0", "-6"):
                bad.append((target.name, what, r.returncode, r.stdout.strip(), r.stderr.strip()[-300:]))
        target.write_bytes(orig)
    assert bad == [], bad[:5]


def test_io_readers_under_address_sanitizer(io, tmp_path):
    """The readers built with -fsanitize=address,undefined (leak checking on)
    in a C driver (tests/io_sanitize_driver.c), on the clean data set and on
    every corruption of test_readers_survive_corrupted_metadata plus truncated
    HDF5 files: no out-of-bounds access, no undefined behaviour, no leak on any
    success or error path."""
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("no gcc")
    exe = str(tmp_path / "io_san")
    build = subprocess.run([cc, "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-std=gnu11",
                            "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(PKG, "csrc"),
                            os.path.join(REPO, "tests", "io_sanitize_driver.c"), os.path.join(PKG, "csrc", "cloudsc_io.c"),
                            "-o", exe, "-ldl", "-lm"], capture_output=True, text=True)
    if build.returncode != 0:
        pytest.skip("no sanitizer runtime: " + build.stderr[-300:])
    dirs = [DATA]
    for i, (name, what, mutate) in enumerate(_corruptions()):
        d = tmp_path / ("c%03d" % i)
        shutil.copytree(DATA, d)
        os.chmod(d / name, 0o644)
        (d / name).write_bytes(mutate((d / name).read_bytes()))
        dirs.append(str(d))
    if io.cloudsc_io_hdf5_available():
        d = load_raw(io)
        try:
            inp = tmp_path / "input.h5"
            assert io.cloudsc_io_write_hdf5(C.byref(d), str(inp).encode(), None) == 0
        finally:
            io.cloudsc_io_free(C.byref(d))
        data = inp.read_bytes()
        for n in (0, 100, len(data) // 2, len(data)):
            p = tmp_path / ("t%d.h5" % n)
            p.write_bytes(data[:n])
            dirs.append(str(p))
    supp = tmp_path / "lsan.supp"
    supp.write_text("leak:libhdf5\nleak:H5\n")     # the HDF5 library's own caches, not ours
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:exitcode=99", UBSAN_OPTIONS="halt_on_error=1:exitcode=98",
               LSAN_OPTIONS="suppressions=%s" % supp)
    r = subprocess.run([exe] + dirs, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr, r.stderr[-3000:]
    lines = r.stdout.split("\n")
    assert lines[0].split() == ["0", "0", "0"]
