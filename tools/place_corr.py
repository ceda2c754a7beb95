#!/usr/bin/env python3
"""Placement study, round 5.

Question 1: does the memory-pattern probe (cloudsc_debug_memory_probe: the KSEG
kernel's loads and stores with no physics) rank output placements the way the
physics kernel does?  If it does, a placement can be chosen before the caller's
inputs exist (cloudsc_fields_alloc).

  N states of one configuration, placement search off, so their output
  placements are whatever hipMalloc gave.  Interleaved over R rounds, per
  state: the KSEG kernel time (state_run), the write-only probe (mode 0) and
  the read+write probe (mode 1) on the state's own pointers.  Pearson and
  Spearman correlation of the probes with the kernel.

Question 2 (--pairs): which output fields collide?  For the slowest and the
fastest state, the write probe of every output field alone and of every pair.

Usage (GPU box): python tools/place_corr.py [--states 10] [--rounds 5] [--pairs] > out.jsonl
"""
import argparse
import ctypes as C
import itertools
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

OUT_NAMES = ["plude", "tendency_loc_t", "tendency_loc_q", "tendency_loc_a", "tendency_loc_cld", "pcovptot",
             "prainfrac_toprfz", "pfsqlf", "pfsqif", "pfcqnng", "pfcqlng", "pfsqrf", "pfsqsf", "pfcqrng",
             "pfcqsng", "pfsqltur", "pfsqitur", "pfplsl", "pfplsn", "pfhpsl", "pfhpsn"]


def rank(x):
    r = np.empty(len(x))
    r[np.argsort(x)] = np.arange(len(x))
    return r


def probe(lib, prec, ngptot, nproma, klev, f, mode, reps=2):
    ms = C.c_float()
    ca.check(lib.cloudsc_debug_memory_probe(0, prec, ngptot, nproma, klev, C.byref(f), mode, reps, C.byref(ms)))
    return ms.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--ngptot", type=int, default=163840)
    ap.add_argument("--nproma", type=int, default=64)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--pairs", action="store_true")
    a = ap.parse_args()
    prec = ca.FP32 if a.fp32 else ca.FP64
    lib = ca.gpu_lib()
    ds = ca.load_dataset()
    ca.check(lib.cloudsc_debug_set_placement_search(0))
    states = [ca.GpuState(ds, a.ngptot, a.nproma, prec) for _ in range(a.states)]
    fields = []
    for g in states:
        f = ca.Fields()
        ca.check(lib.cloudsc_state_fields(g.h, C.byref(f)))
        fields.append(f)
    # warm the clock (bench.py prewarm): ~40 launches
    for _ in range(4):
        for g in states:
            g.run(ca.VARIANT_KSEG, 1)
    kt = [[] for _ in states]
    w = [[] for _ in states]
    rw = [[] for _ in states]
    for r in range(a.rounds):
        order = range(a.states) if r % 2 == 0 else reversed(range(a.states))
        for i in order:
            kt[i].append(float(min(states[i].run(ca.VARIANT_KSEG, 2))))
            w[i].append(probe(lib, prec, a.ngptot, a.nproma, ds.klev, fields[i], 0))
            rw[i].append(probe(lib, prec, a.ngptot, a.nproma, ds.klev, fields[i], 1))
        print(json.dumps({"round": r, "kernel_ms": [round(x[-1], 4) for x in kt]}), flush=True)
    K = np.array([np.median(x) for x in kt])
    W = np.array([np.median(x) for x in w])
    RW = np.array([np.median(x) for x in rw])
    for i in range(a.states):
        print(json.dumps({"state": i, "kernel_ms": round(K[i], 4), "write_probe_ms": round(W[i], 4),
                          "rw_probe_ms": round(RW[i], 4),
                          "first_output": hex(C.cast(fields[i].tendency_loc_t, C.c_void_p).value or 0)}),
              flush=True)
    res = {"states": a.states, "rounds": a.rounds, "precision": prec,
           "kernel_spread": round(float(K.max() / K.min() - 1), 4),
           "pearson_write": round(float(np.corrcoef(K, W)[0, 1]), 3),
           "pearson_rw": round(float(np.corrcoef(K, RW)[0, 1]), 3),
           "spearman_write": round(float(np.corrcoef(rank(K), rank(W))[0, 1]), 3),
           "spearman_rw": round(float(np.corrcoef(rank(K), rank(RW))[0, 1]), 3),
           "argmin_kernel": int(K.argmin()), "argmin_write": int(W.argmin()), "argmin_rw": int(RW.argmin())}
    print(json.dumps(res), flush=True)
    if a.pairs:
        for label, i in (("slowest", int(K.argmax())), ("fastest", int(K.argmin()))):
            src = fields[i]
            single = {}
            for n in OUT_NAMES:
                f = ca.Fields()
                setattr(f, n, getattr(src, n))
                single[n] = probe(lib, prec, a.ngptot, a.nproma, ds.klev, f, 0, 3)
            pair = {}
            for x, y in itertools.combinations(OUT_NAMES, 2):
                f = ca.Fields()
                setattr(f, x, getattr(src, x))
                setattr(f, y, getattr(src, y))
                pair[x + "+" + y] = probe(lib, prec, a.ngptot, a.nproma, ds.klev, f, 0, 3)
            # excess of a pair over its two fields written one after the other
            exc = {k: v / (single[k.split("+")[0]] + single[k.split("+")[1]]) for k, v in pair.items()}
            worst = sorted(exc.items(), key=lambda kv: -kv[1])[:12]
            addr = {n: hex(C.cast(getattr(src, n), C.c_void_p).value or 0) for n in OUT_NAMES}
            print(json.dumps({"pairs": label, "state": i, "kernel_ms": round(K[i], 4),
                              "single_us": {k: round(v * 1e3, 1) for k, v in single.items()},
                              "pair_ratio_median": round(float(np.median(list(exc.values()))), 3),
                              "worst_pairs": [(k, round(v, 3)) for k, v in worst], "addresses": addr}),
                  flush=True)
    for g in states:
        g.close()


if __name__ == "__main__":
    main()
