#!/usr/bin/env python3
"""Host-buffer path (H2D -> kernel -> D2H per chunk, overlapped on streams):
time per step over chunk sizes and stream counts."""
import itertools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

ngptot = int(sys.argv[1]) if len(sys.argv) > 1 else 163840
nproma = 64
ds = ca.load_dataset()
for chunk, ns in itertools.product((32, 64, 128, 320), (2, 3, 4, 6)):
    hp = ca.HostPipeline(ds, ngptot, nproma, ca.FP64, chunk_blocks=chunk, nstreams=ns)
    try:
        hp.run(ca.VARIANT_KSEG)
        ms = min(hp.run(ca.VARIANT_KSEG) for _ in range(3))
    finally:
        hp.close()
    print(json.dumps({"chunk_blocks": chunk, "nstreams": ns, "ms": round(ms, 2),
                      "Mcol_per_s": round(ngptot / ms / 1e3, 3),
                      "GBs_both_dirs": round(56036 * ngptot / ms / 1e6, 1)}), flush=True)
