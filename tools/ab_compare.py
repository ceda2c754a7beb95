#!/usr/bin/env python3
"""A/B bit-identity check between two builds of libcloudsc_amd.so: run a fixed
set of cases with the library named by CLOUDSC_AMD_LIB and write one SHA-256
per (case, field) to a JSON file; --compare A.json B.json lists differences.
Cases: reference state, scenarios W/M, three random perturbations, NSSOPT 0/2/3,
aerosol flags, fp32, and the full 163840-column state."""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))


def cases(ca, mf):
    base = ca.load_dataset()
    yield "ref_1000", base, 1000, ca.FP64
    yield "W", mf.load_scenario("W", base), 1000, ca.FP64
    yield "M", mf.load_scenario("M", base), 1000, ca.FP64
    for seed in (1, 2, 3):
        yield "perturbed_%d" % seed, mf.perturbed(base, seed), 1000, ca.FP64
    for n in (0, 2, 3):
        s = base.copy()
        s.params["nssopt"] = n
        yield "nssopt_%d" % n, s, 300, ca.FP64
    yield "aerosol", mf.with_aerosols(base), 300, ca.FP64
    yield "fp32_1000", base, 1000, ca.FP32
    yield "fp32_W", mf.load_scenario("W", base), 1000, ca.FP32
    yield "full_163840", base, 163840, ca.FP64


def run(out_path, variant_name):
    import cloudsc_amd as ca
    import make_fixtures as mf
    variant = {"kseg": ca.VARIANT_KSEG, "kcache": ca.VARIANT_KCACHE, "scc": ca.VARIANT_SCC}[variant_name]
    res = {}
    for name, ds, ngptot, prec in cases(ca, mf):
        g = ca.GpuState(ds, ngptot, 128, prec)
        try:
            g.run(variant, 1)
            for _, k in ca.VALIDATED:
                res["%s/%s" % (name, k)] = hashlib.sha256(g.download(k).tobytes()).hexdigest()
        finally:
            g.close()
        print("done", name, flush=True)
    json.dump(res, open(out_path, "w"), indent=0, sort_keys=True)


def compare(a, b):
    A, B = json.load(open(a)), json.load(open(b))
    diff = sorted(k for k in A if A[k] != B.get(k))
    print("%d of %d (case, field) pairs differ" % (len(diff), len(A)))
    for k in diff:
        print("  ", k)
    return 1 if diff else 0


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--out")
    p.add_argument("--variant", default="kcache")
    p.add_argument("--compare", nargs=2)
    a = p.parse_args()
    if a.compare:
        sys.exit(compare(*a.compare))
    run(a.out, a.variant)
