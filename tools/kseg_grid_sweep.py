#!/usr/bin/env python3
"""KSEG schedule sweep (persistent grid size x level segments) through the
library's diagnostic setter, against KCACHE on the same state: kernel ms
(median of --reps after --warmup) per (precision, grid, nseg)."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--precision", default="fp32")
p.add_argument("--nproma", type=int, default=64)
p.add_argument("--grids", default="0,2048,2560,3072")
p.add_argument("--nsegs", default="0,2,3,4")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--warmup", type=int, default=3)
a = p.parse_args()
prec = ca.FP64 if a.precision == "fp64" else ca.FP32
g = ca.GpuState(ca.load_dataset(), 163840, a.nproma, prec)
try:
    g.run(ca.VARIANT_KCACHE, a.warmup)
    kc = float(np.median(g.run(ca.VARIANT_KCACHE, a.reps)))
    print(json.dumps({"variant": "kcache", "precision": a.precision, "kernel_ms_median": round(kc, 4)}), flush=True)
    for grid in [int(x) for x in a.grids.split(",")]:
        for nseg in [int(x) for x in a.nsegs.split(",")]:
            ca.kseg_schedule(nseg, grid)
            g.run(ca.VARIANT_KSEG, a.warmup)
            ms = float(np.median(g.run(ca.VARIANT_KSEG, a.reps)))
            print(json.dumps({"variant": "kseg", "precision": a.precision, "grid": grid, "nseg": nseg,
                              "kernel_ms_median": round(ms, 4)}), flush=True)
finally:
    ca.kseg_schedule(0, 0)
    g.close()
