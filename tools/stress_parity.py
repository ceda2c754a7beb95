#!/usr/bin/env python3
"""Parity at the edges of the input space (diagnostic): states pushed beyond the
shipped data's ranges -- condensate scaled down to 1e-200 or up 1000x, no
condensate and no humidity at all, temperatures 60 K warmer or 80 K colder,
tendencies 100x, pressures scaled down 100x, subnormal condensate -- each run
through the KSEG kernel (fp64) and the oracle, every validated field compared
bit for bit.  One JSON line per case: the fields that differ and how many
elements, and whether the outputs are finite.

usage (GPU box): python tools/stress_parity.py [--ngptot 300] [--nproma 64]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cloudsc_amd as ca  # noqa: E402
import make_fixtures as mf  # noqa: E402
import oracle  # noqa: E402


def cases(ds):
    for name in mf.EDGE_CASES:
        yield name, mf.edge_case(ds, name)
    yield "perturbed_seed7", mf.perturbed(ds, 7)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ngptot", type=int, default=300)
    ap.add_argument("--nproma", type=int, default=64)
    a = ap.parse_args()
    ds = ca.load_dataset()
    for name, s in cases(ds):
        st, _ = oracle.run_oracle(s, a.ngptot, a.nproma)
        ref = ca.state_outputs_to_template(st.arrays, a.ngptot)
        g = ca.GpuState(s, a.ngptot, a.nproma, ca.FP64)
        try:
            g.run(ca.VARIANT_KSEG, 1)
            out = g.outputs()
        finally:
            g.close()
        bad = {}
        finite_gpu = finite_ref = True
        for _, k in ca.VALIDATED:
            x = np.ascontiguousarray(out[k], dtype=np.float64)
            r = np.ascontiguousarray(ref[k], dtype=np.float64)
            finite_gpu &= bool(np.all(np.isfinite(x)))
            finite_ref &= bool(np.all(np.isfinite(r)))
            n = int(np.count_nonzero(x.view(np.uint64) != r.view(np.uint64)))
            if n:
                bad[k] = n
        print(json.dumps({"case": name, "fields_differing": bad, "finite_gpu": finite_gpu,
                          "finite_oracle": finite_ref}), flush=True)


if __name__ == "__main__":
    main()
