#!/usr/bin/env python3
"""Static instruction mix of the KSEG level loop (diagnostic, host only).

Compiles cloudsc_gpu.hip for gfx950 to assembly (one precision's KSEG kernel,
-DCLOUDSC_ONLY_KSEG), finds the product kernel's level loop (the innermost
loop with the most instructions) and prints its instruction count by mnemonic,
the VALU share and where the register moves come from (VGPR copies, SGPR
materialisations, constants).  Static counts: code inside branches counts
once whether or not a wave takes it.

usage: isa_mix.py fp64|fp32 [extra hipcc flags...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
    es = 8 if prec == "fp64" else 4
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-ffp-contract=off", "-std=c++17", "--offload-arch=gfx950",
                           "-mllvm", "-disable-machine-licm", "-I" + os.path.join(REPO, "include"),
                           "-I" + os.path.join(REPO, "dwarf-p-cloudsc_amd", "csrc"), "-DCLOUDSC_ONLY_KSEG=%d" % es,
                           "--cuda-device-only", "-S", os.path.join(REPO, "dwarf-p-cloudsc_amd", "csrc", "cloudsc_gpu.hip"),
                           "-o", out] + sys.argv[2:], stderr=subprocess.DEVNULL)
    L = open(out).read().split("\n")
    # the product kernel: no aerosols, no LDS carry; fp32 FAST (last flag 1), fp64 exact (0)
    name = r"^_Z10kseg_entryI%sLi2ELi%dELb0ELb0ELb%dE.*:" % ("d" if es == 8 else "f", 3 if es == 8 else 1,
                                                             0 if es == 8 else 1)
    st = next(i for i, l in enumerate(L) if re.match(name, l))
    en = next(i for i in range(st, len(L)) if L[i].startswith(".Lfunc_end"))
    L = L[st:en]
    labels = {m.group(1): i for i, l in enumerate(L) for m in [re.match(r"^(\.LBB\d+_\d+):", l)] if m}
    loops = {}
    for i, l in enumerate(L):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            h = m.group(1)
            loops[h] = (labels[h], max(i, loops.get(h, (0, 0))[1]))
    # innermost big loop: the largest loop that contains no other loop header of comparable size
    cands = sorted(loops.values(), key=lambda ab: ab[1] - ab[0], reverse=True)
    a, b = cands[1] if len(cands) > 1 else cands[0]
    cnt, moves = collections.Counter(), collections.Counter()
    for l in L[a:b + 1]:
        t = l.strip()
        if not t or t[0] in ";." or t.endswith(":"):
            continue
        op = t.split()[0]
        cnt[op] += 1
        if op.startswith("v_mov_b"):
            src = t.split(",")[1].strip().split()[0]
            moves["vgpr" if src.startswith("v") else "sgpr" if src.startswith("s") else "constant"] += 1
    tot = sum(cnt.values())
    valu = sum(c for o, c in cnt.items() if o.startswith("v_"))
    print("%s KSEG level loop: %d instructions, %d VALU, %d SALU, %d vector memory, %d LDS" % (
        prec, tot, valu, sum(c for o, c in cnt.items() if o.startswith("s_")),
        sum(c for o, c in cnt.items() if o.startswith("global_")), sum(c for o, c in cnt.items() if o.startswith("ds_"))))
    print("register moves by source:", dict(moves), "of", sum(moves.values()))
    for o, c in cnt.most_common(30):
        print("  %-28s %d" % (o, c))


if __name__ == "__main__":
    main()
