#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table from the compiler's
kernel-resource-usage remarks (make -C dwarf-p-cloudsc_amd resources)."""
import re
import subprocess
import os

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dwarf-p-cloudsc_amd")
out = subprocess.run(["make", "-s", "-C", PKG, "resources"], capture_output=True, text=True).stdout
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
print("%-60s %5s %5s %8s %4s" % ("kernel", "VGPR", "AGPR", "scratch", "occ"))
for r, d in zip(rows, dem):
    d = re.sub(r"\(.*", "", d)
    print("%-60s %5d %5d %8d %4d" % (d[:60], r.get("vgpr", -1), r.get("agpr", -1), r.get("scratch", -1), r.get("occ", -1)))
