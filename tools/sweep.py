#!/usr/bin/env python3
"""Kernel-time sweep over variant / precision / NPROMA on one GPU (HIP events on
the launch stream; median of --reps steps after --warmup)."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

BYTES = {ca.FP64: 56036, ca.FP32: 28020}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("--nproma", default="64,128,256")
    p.add_argument("--variants", default="kcache,scc")
    p.add_argument("--precisions", default="fp64,fp32")
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--cfgs", default="", help="comma list of CLOUDSC_KCACHE_CFG values to sweep (kcache/kseg)")
    p.add_argument("--nsegs", default="", help="comma list of CLOUDSC_KSEG_NSEG values to sweep (kseg only)")
    a = p.parse_args()
    ds = ca.load_dataset()
    rows = []
    for prec_s in a.precisions.split(","):
        prec = ca.FP64 if prec_s == "fp64" else ca.FP32
        for npr in [int(x) for x in a.nproma.split(",")]:
            g = ca.GpuState(ds, a.ngptot, npr, prec)
            combos = []
            for var_s in a.variants.split(","):
                cfgs = a.cfgs.split(",") if (var_s in ("kcache", "kseg") and a.cfgs) else [""]
                nsegs = a.nsegs.split(",") if (var_s == "kseg" and a.nsegs) else [""]
                combos += [(var_s, c, n) for c in cfgs for n in nsegs]
            for var_s, cfg, nseg in combos:
                for key, val in (("CLOUDSC_KCACHE_CFG", cfg), ("CLOUDSC_KSEG_NSEG", nseg)):
                    if val:
                        os.environ[key] = val
                    else:
                        os.environ.pop(key, None)
                var = {"kcache": ca.VARIANT_KCACHE, "scc": ca.VARIANT_SCC, "kseg": ca.VARIANT_KSEG,
               "scc-private": ca.VARIANT_SCC_PRIVATE}[var_s]
                g.run(var, a.warmup)
                ms = g.run(var, a.reps)
                med = float(np.median(ms))
                st = g.validate()
                worst = max((s[3] / s[4] if s[4] > 0 else s[3]) for s in st)
                row = {"variant": var_s, "cfg": cfg, "nseg": nseg, "precision": prec_s, "nproma": npr, "ngptot": a.ngptot,
                       "kernel_ms_median": round(med, 4), "kernel_ms_min": round(float(np.min(ms)), 4),
                       "Mcol_per_s": round(a.ngptot / med / 1e3, 2),
                       "algo_GBs": round(BYTES[prec] * a.ngptot / (med * 1e-3) / 1e9, 1),
                       "worst_rel_l1_vs_reference": worst}
                print(json.dumps(row), flush=True)
                rows.append(row)
            g.close()


if __name__ == "__main__":
    main()
