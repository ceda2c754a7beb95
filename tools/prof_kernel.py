#!/usr/bin/env python3
"""Minimal driver for rocprofv3 counter passes: build one device state and run
the chosen kernel a few times (no validation, no CPU work)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--precision", default="fp64")
p.add_argument("--variant", default="kcache")
p.add_argument("--ngptot", type=int, default=163840)
p.add_argument("--nproma", type=int, default=128)
p.add_argument("--reps", type=int, default=3)
p.add_argument("--cfg", default="")
a = p.parse_args()
if a.cfg:
    os.environ["CLOUDSC_KCACHE_CFG"] = a.cfg
ds = ca.load_dataset()
g = ca.GpuState(ds, a.ngptot, a.nproma, ca.FP64 if a.precision == "fp64" else ca.FP32)
ms = g.run({"kseg": ca.VARIANT_KSEG, "kcache": ca.VARIANT_KCACHE, "scc": ca.VARIANT_SCC,
      "scc-private": ca.VARIANT_SCC_PRIVATE}[a.variant], a.reps)
print("kernel ms:", ms)
g.close()
