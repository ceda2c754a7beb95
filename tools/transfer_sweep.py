#!/usr/bin/env python3
"""Host-buffer path (H2D -> kernel -> D2H per chunk, pipelined over an input,
a kernel and an output stream): time per step over chunk sizes and device
chunk-slot counts (the `nstreams` argument of cloudsc_host_pipeline_create).
usage: transfer_sweep.py [ngptot] [chunks,..] [slots,..]"""
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
chunks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else (32, 64, 128, 256, 640)
slots = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else (2, 3, 4)
for chunk, ns in itertools.product(chunks, slots):
    hp = ca.HostPipeline(ds, ngptot, nproma, ca.FP64, chunk_blocks=chunk, nstreams=ns)
    try:
        hp.run(ca.VARIANT_KSEG)
        ms = min(hp.run(ca.VARIANT_KSEG) for _ in range(3))
    finally:
        hp.close()
    print(json.dumps({"chunk_blocks": chunk, "slots": ns, "ms": round(ms, 2),
                      "Mcol_per_s": round(ngptot / ms / 1e3, 3),
                      "GBs_both_dirs": round(56036 * ngptot / ms / 1e6, 1)}), flush=True)
