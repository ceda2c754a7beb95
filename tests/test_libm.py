"""The device exp/pow (dwarf-p-cloudsc_amd/csrc/cloudsc_libm.h) compiled for the
host must reproduce the host C library's exp/pow -- the functions the reference
kernel calls -- bit for bit (tools/libm_check.cc), and the lookup tables must
be what tools/gen_libm_tables.py derives from their definitions."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "dwarf-p-cloudsc_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("libm") / "libm_check")
    subprocess.check_call([cxx, "-O2", "-mfma", "-ffp-contract=off", "-std=c++20", "-I" + CSRC,
                           os.path.join(REPO, "tools", "libm_check.cc"), "-o", exe])
    return exe


def has_fma():
    try:
        with open("/proc/cpuinfo") as f:
            return " fma " in f.read()
    except OSError:
        return False


@pytest.mark.skipif(not has_fma(), reason="the host C library's non-FMA variant rounds differently in rare cases")
@pytest.mark.parametrize("seed", [20250227, 7])
def test_exp_pow_bitwise_vs_host_libm(checker, seed):
    r = subprocess.run([checker, "1", str(seed)], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    for line in r.stdout.splitlines():
        assert "mismatches        0" in line, line


def test_tables_are_generated(tmp_path):
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_libm_tables", os.path.join(REPO, "tools", "gen_libm_tables.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    exp_rows = gen.exp_table()
    log_rows = gen.log_table()
    # spot values of the published tables: 2^(1/128) ~= H(1 + T), first log row
    assert exp_rows[1] == (0x3C9B3B4F1A88BF6E, 0x3FEFF63DA9FB3335)
    assert log_rows[0][0] == 1.4140625 and log_rows[0][1] == float.fromhex("-0x1.62c82f2b9c800p-2")
    # the committed header is the generator's output
    with open(os.path.join(CSRC, "cloudsc_libm_tab.h")) as f:
        text = f.read()
    for t, s in exp_rows:
        assert "0x%016xULL, 0x%016xULL" % (t, s) in text
    for invc, logc, tail in log_rows:
        assert "%s, %s, %s, 0.0" % (invc.hex(), logc.hex(), tail.hex()) in text


def test_known_divisor_division(tmp_path):
    """cl_div_known / cl_div_lit (cloudsc_dev.h): with the host's r = RN(1/d)
    the one-correction quotient (two in fp32) is the IEEE n/d, for CLOUDSC's
    constant divisors and random ones (tools/div_const_check.c)."""
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("no gcc")
    exe = str(tmp_path / "div_const_check")
    subprocess.check_call([cc, "-O2", "-ffp-contract=off", os.path.join(REPO, "tools", "div_const_check.c"),
                           "-lm", "-o", exe])
    r = subprocess.run([exe, "2"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0 and "total mismatches 0" in r.stdout, r.stdout + r.stderr
