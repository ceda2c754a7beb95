#!/usr/bin/env python3
"""Diagnostic: step-to-step spread of the host-buffer pipeline
(cloudsc_host_pipeline_run) -- every step's time, for host arrays from numpy
(pinned in place by the pipeline with hipHostRegister) and for the same arrays
in hipHostMalloc memory (already pinned; the pipeline uses them as they are),
and by copy path (cloudsc_debug_set_pipeline_copy): engines pinned per
direction (the default), HIP streams with the runtime's engine choice, or HIP
streams with the outputs written back by a copy kernel.
usage: pipeline_steps.py [steps] [chunk_blocks] [slots] [modes]
modes: comma-separated of reg, reg-hip, reg-blit, hm, hm-hip (default: reg, reg-hip, hm, hm-hip, reg)"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 128
slots = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ds = ca.load_dataset()
hip = C.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostFree.argtypes = [C.c_void_p]


def host_nodes(arrays, per_array=8):
    """NUMA node of sampled pages of the host arrays (move_pages(2) query
    form, nothing is moved): {node: pages}."""
    libc = C.CDLL(None, use_errno=True)
    pages = []
    for a in arrays.values():
        if a.nbytes >= 4096:
            base = a.ctypes.data
            pages += [base + i * (a.nbytes // per_array) // 4096 * 4096 for i in range(per_array)]
    n = len(pages)
    pa = (C.c_void_p * n)(*pages)
    st = (C.c_int * n)()
    if libc.syscall(279, 0, C.c_ulong(n), pa, None, st, 0) != 0:   # SYS_move_pages (x86_64)
        return None
    out = {}
    for v in st:
        out[str(v)] = out.get(str(v), 0) + 1
    return out


def gpu_numa_node():
    bus = C.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(bus, 64, 0) != 0:
        return None
    try:
        return int(open("/sys/bus/pci/devices/%s/numa_node" % bus.value.decode().lower()).read())
    except (OSError, ValueError):
        return None


GPU_NODE = gpu_numa_node()

COPY = {0: "hip streams", 1: "engines per direction", 2: "hip streams, D2H by copy kernel"}


def run(kind, copy=1):
    ca.check(ca.gpu_lib().cloudsc_debug_set_pipeline_copy(copy))
    hp = ca.HostPipeline.__new__(ca.HostPipeline)
    if kind == "registered":
        hp = ca.HostPipeline(ds, 163840, 64, ca.FP64, chunk_blocks=chunk, nstreams=slots)
        keep = []
    else:
        # the same state, every array moved into hipHostMalloc memory before the pipeline is created
        lib = ca.gpu_lib()
        params = ca.Params.from_dict(ds.params)
        ca.check(lib.cloudsc_gpu_init(0, C.byref(params)))
        st = ca.make_host_state(ds, 163840, 64, ca.FP64)
        keep = []
        for name, a in list(st.arrays.items()):
            p = C.c_void_p()
            assert hip.hipHostMalloc(C.byref(p), a.nbytes, 0) == 0
            keep.append(p)
            v = np.ctypeslib.as_array((C.c_byte * a.nbytes).from_address(p.value)).view(a.dtype).reshape(a.shape)
            v[...] = a
            st.arrays[name] = v
        hp.lib, hp.ds, hp.ngptot, hp.nproma, hp.precision = lib, ds, 163840, 64, ca.FP64
        hp._params, hp.state, hp._plude0 = params, st, st.arrays["plude"].copy()
        f = st.fields()
        for name in ca.AEROSOL_FIELDS:
            setattr(f, name, None)
        hp._fields = f
        h = C.c_void_p()
        ca.check(lib.cloudsc_host_pipeline_create(C.byref(h), 0, ca.FP64, 163840, 64, ds.klev, chunk, slots,
                                                  C.byref(f)))
        hp.h = h
    try:
        mode, e_in, e_out = hp.copy_path()
        overlap, pairs = hp.engine_check()
        nodes = host_nodes(hp.state.arrays)
        hp.run(ca.VARIANT_KSEG)
        ms = [round(hp.run(ca.VARIANT_KSEG), 2) for _ in range(steps)]
    finally:
        hp.close()
        for p in keep:
            hip.hipHostFree(p)
    print(json.dumps({"host_memory": kind, "copy": COPY[copy], "engines": [e_in, e_out], "engine_overlap": round(overlap, 3),
                      "pairs_tried": pairs,
                      "host_numa_nodes": nodes, "gpu_numa_node": GPU_NODE,
                      "chunk_blocks": chunk, "slots": slots, "ms": ms,
                      "median": float(np.median(ms)), "min": min(ms)}), flush=True)


MODES = {"reg": ("registered", 1), "reg-hip": ("registered", 0), "reg-blit": ("registered", 2),
         "hm": ("hostmalloc", 1), "hm-hip": ("hostmalloc", 0)}
modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["reg", "reg-hip", "hm", "hm-hip", "reg"]
for m in modes:
    run(*MODES[m])
ca.check(ca.gpu_lib().cloudsc_debug_set_pipeline_copy(-1))
