#!/usr/bin/env python3
"""Per-step overlap of the two copy directions in a rocprofv3 memory-copy trace
of tools/pipeline_steps.py (one pipeline, `steps` steps after one warm step,
each of nchunks chunks): busy time per direction, the time both run at once,
and the gaps of the H2D stream.
usage: copy_trace_overlap.py <dir with *_memory_copy_trace.csv> [steps incl. warm-up = 7]"""
import csv
import glob
import sys

d = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = list(csv.DictReader(open(glob.glob(d + "/*memory_copy_trace.csv")[0])))
h = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
           if r["Direction"].endswith("HOST_TO_DEVICE"))
o = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
           if r["Direction"].endswith("DEVICE_TO_HOST"))
nh, nd = len(h) // nsteps, len(o) // nsteps


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


for s in range(nsteps):
    H, D = union(h[s * nh:(s + 1) * nh]), union(o[s * nd:(s + 1) * nd])
    ov, i, j = 0, 0, 0
    while i < len(H) and j < len(D):
        a, b = max(H[i][0], D[j][0]), min(H[i][1], D[j][1])
        ov += max(0, b - a)
        if H[i][1] < D[j][1]:
            i += 1
        else:
            j += 1
    span = max(H[-1][1], D[-1][1]) - min(H[0][0], D[0][0])
    print("step %d: span %.1f ms  H2D busy %.1f ms  D2H busy %.1f ms  both at once %.1f ms" % (
        s, span / 1e6, sum(b - a for a, b in H) / 1e6, sum(b - a for a, b in D) / 1e6, ov / 1e6))
