"""The dwarf's stdout contract, checked the way the reference's benchmark
harness reads it: JUBE's `timing_pattern` and `results_pattern`
(benchmark/include/include_patternset.yml:2-171) applied to captured
`dwarf-cloudsc-amd` output.

The patterns are restated here, not copied: the per-field result patterns are
generated from the field list (the yml spells out one block of five per field,
:10-134), and JUBE's default `$jube_pat_*` macros are expanded to their
documented regexes.  The reference C validator prints the tendency rows in
upper case (`TENDENCY_LOC%A`, src/cloudsc_c/cloudsc/cloudsc_validate.c:213-216)
while the yml spells the Fortran dwarf's `tendency_loc%a`; those four rows are
matched case-insensitively, the P* rows exactly.

CPU: the `--variant cpu` run prints one `@ core#` row per host thread like the
C dwarf (cloudsc_driver.c:238-253).  GPU (tests/test_gpu_driver.py): the
`--gpus N` shard rows end in `@ core#` like the reference GPU driver
(src/cloudsc_cuda/cloudsc/cloudsc_driver.cu:475)."""
import os
import re
import subprocess

import pytest

import cloudsc_amd as ca

# JUBE's built-in pattern macros (JUBE documentation, "Predefined patterns")
JUBE = {
    "jube_pat_int": r"([+-]?\d+)",
    "jube_pat_nint": r"(?:[+-]?\d+)",
    "jube_pat_fp": r"([+-]?(?:\d*\.?\d+(?:[eE][-+]?\d+)?|\d+\.))",
    "jube_pat_nfp": r"(?:[+-]?(?:\d*\.?\d+(?:[eE][-+]?\d+)?|\d+\.))",
}


def jube(pat):
    """Expand $jube_pat_* macros (longest names first: nint before int)."""
    for k in sorted(JUBE, key=len, reverse=True):
        pat = pat.replace("$" + k, JUBE[k])
    return pat


# timing_pattern (include_patternset.yml:159-171)
TIMING = {
    "thr_time": r"(?:$jube_pat_nint\s+){6}:\s+$jube_pat_int\s+(?:$jube_pat_nint\s+){2}@\s+(?:rank#$jube_pat_nint:)?core#",
    "thr_mflops": r"(?:$jube_pat_nint\s+){6}:\s+$jube_pat_nint\s+$jube_pat_int\s+$jube_pat_nint\s+@\s+(?:rank#$jube_pat_nint:)?core#",
    "tot_time": r"(?:$jube_pat_nint\s*x\s*)?(?:$jube_pat_nint\s+){6}:\s+$jube_pat_int\s+(?:$jube_pat_nint\s+){2}(?::\s+)?TOTAL(?!\s@)",
    "tot_mflops": r"(?:$jube_pat_nint\s*x\s*)?(?:$jube_pat_nint\s+){6}:\s+$jube_pat_nint\s+$jube_pat_int\s+$jube_pat_nint\s+(?::\s+)?TOTAL(?!\s@)",
    "tot_numomp": r"(?:$jube_pat_nint\s*x\s*)?$jube_pat_int\s+(?:$jube_pat_nint\s+){5}:\s+(?:$jube_pat_nint\s+){3}(?::\s+)?TOTAL(?!\s@)",
    "tot_ngptot": r"(?:$jube_pat_nint\s*x\s*)?$jube_pat_nint\s+$jube_pat_int\s+(?:$jube_pat_nint\s+){4}:\s+(?:$jube_pat_nint\s+){3}(?::\s+)?TOTAL(?!\s@)",
    "tot_ngpblks": r"(?:$jube_pat_nint\s*x\s*)?(?:$jube_pat_nint\s+){3}$jube_pat_int\s+(?:$jube_pat_nint\s+){2}:\s+(?:$jube_pat_nint\s+){3}(?::\s+)?TOTAL(?!\s@)",
    "tot_nproma": r"(?:$jube_pat_nint\s*x\s*)?(?:$jube_pat_nint\s+){4}$jube_pat_int\s+$jube_pat_nint\s+:\s+(?:$jube_pat_nint\s+){3}(?::\s+)?TOTAL(?!\s@)",
}

FIELDS = ["PLUDE", "PCOVPTOT", "PRAINFRAC_TOPRFZ", "PFSQLF", "PFSQIF", "PFCQLNG", "PFCQNNG", "PFSQRF", "PFSQSF",
          "PFCQRNG", "PFCQSNG", "PFSQLTUR", "PFSQITUR", "PFPLSL", "PFPLSN", "PFHPSL", "PFHPSN", "tendency_loc%a",
          "tendency_loc%q", "tendency_loc%T", "tendency_loc%cld"]
COLUMNS = ["min", "max", "abs_max_err", "avg_abs_err", "max_rel_err"]


def result_patterns():
    """results_pattern (include_patternset.yml:3-134): for each field, five
    patterns that capture one of MinValue .. MaxRelErr-% on its row."""
    out = {}
    for f in FIELDS:
        for i, col in enumerate(COLUMNS):
            nums = [r"$jube_pat_fp" if j == i else r"$jube_pat_nfp" for j in range(5)]
            out[(f, col)] = re.escape(f) + r"\s+\dD\d\s+" + r"\s+".join(nums)
    return out


def check_timing(out, nthreads, ngptot, nproma, nblocks):
    """Apply the timing patterns; returns the captured per-thread times."""
    thr = [int(m.group(1)) for m in re.finditer(jube(TIMING["thr_time"]), out)]
    thr_mf = [int(m.group(1)) for m in re.finditer(jube(TIMING["thr_mflops"]), out)]
    assert len(thr) == nthreads and len(thr_mf) == nthreads, (thr, thr_mf)
    tot = {k: [int(m.group(1)) for m in re.finditer(jube(v), out)] for k, v in TIMING.items() if k.startswith("tot")}
    assert all(len(v) == 1 for v in tot.values()), tot
    assert tot["tot_ngptot"] == [ngptot] and tot["tot_nproma"] == [nproma] and tot["tot_ngpblks"] == [nblocks]
    assert tot["tot_time"][0] >= 0 and tot["tot_mflops"][0] >= 0
    return thr, tot


def check_results(out):
    """Apply the result patterns: every field's five values are captured, and
    the dwarf's tolerance holds (MaxRelErr-% <= 100 * 10 eps)."""
    got = {}
    for (f, col), pat in result_patterns().items():
        flags = re.IGNORECASE if f.startswith("tendency") else 0
        m = re.findall(jube(pat), out, flags)
        assert len(m) == 1, (f, col, m)
        got[(f, col)] = float(m[0])
    for f in FIELDS:
        assert got[(f, "max_rel_err")] <= 100 * 10 * 2.220446049250313e-16, f
    return got


def test_jube_macros_expand():
    assert re.fullmatch(jube("$jube_pat_fp"), "-0.1026720108982E-03")
    assert re.fullmatch(jube("$jube_pat_nint"), "-1")
    assert "$" not in jube(TIMING["thr_time"])


def test_jube_patterns_on_cpu_dwarf():
    """`dwarf-cloudsc-amd 3 2000 32 --variant cpu`: three `@ core#` thread rows,
    one TOTAL row with NUMOMP/NGPTOT/#BLKS/NPROMA, and all 21 x 5 result values."""
    exe = os.path.join(os.path.dirname(ca.LIB_PATH), "dwarf-cloudsc-amd")
    if not os.path.exists(exe):
        pytest.skip("dwarf-cloudsc-amd not built")
    r = subprocess.run([exe, "3", "2000", "32", "--variant", "cpu", "--reps", "2"], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout[-4000:], r.stderr[-1000:])
    assert r.returncode == 0
    _, tot = check_timing(r.stdout, 3, 2000, 32, 63)
    assert tot["tot_numomp"] == [3]
    # the threads' columns add up to NGPTOT (the #GP-cols column of the thread rows)
    rows = re.findall(r"^\s+3\s+2000\s+(\d+)\s+(\d+)\s+32\s+(\d) :.*@ core#$", r.stdout, re.M)
    assert sorted(int(t) for _, _, t in rows) == [0, 1, 2]
    assert sum(int(c) for c, _, _ in rows) == 2000 and sum(int(b) for _, b, _ in rows) == 63
    check_results(r.stdout)
