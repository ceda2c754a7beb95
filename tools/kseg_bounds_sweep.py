#!/usr/bin/env python3
"""KSEG segment boundaries sweep (CLOUDSC_KSEG_BOUNDS) at NGPTOT 163840."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

nproma = int(sys.argv[1]) if len(sys.argv) > 1 else 64
sets = sys.argv[2].split(";") if len(sys.argv) > 2 else []
ds = ca.load_dataset()
g = ca.GpuState(ds, 163840, nproma)
for rnd in range(2):
    for b in sets:
        if b:
            os.environ["CLOUDSC_KSEG_BOUNDS"] = b
        else:
            os.environ.pop("CLOUDSC_KSEG_BOUNDS", None)
        g.run(ca.VARIANT_KSEG, 3)
        ms = g.run(ca.VARIANT_KSEG, 20)
        print(json.dumps({"round": rnd, "bounds": b or "default", "nproma": nproma,
                          "ms": round(float(np.median(ms)), 4)}), flush=True)
g.close()
