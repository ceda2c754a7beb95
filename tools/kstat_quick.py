#!/usr/bin/env python3
"""Static instruction histogram of one kernel of a csrc tree (diagnostic).
usage: kstat_quick.py <csrc dir> <kernel-name-substring> [extra hipcc flags]"""
import collections
import re
import subprocess
import sys

src, pat = sys.argv[1], sys.argv[2]
out = "/tmp/kstat_quick.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-ffp-contract=off", "-std=c++17", "--offload-arch=gfx950",
                       "-mllvm", "-disable-machine-licm", "-I/root/repo/include", "-I" + src, "--cuda-device-only",
                       "-S", src + "/cloudsc_gpu.hip", "-o", out] + sys.argv[3:])
s = open(out).read()
for f in re.split(r'\n(?=\S+:\s*; @)', s):
    name = f.split(':')[0].strip()
    if pat in name and not name.startswith('.'):
        ops = collections.Counter()
        for l in f.splitlines():
            l = l.strip()
            if not l or l.startswith((';', '.')) or l.endswith(':'):
                continue
            ops[l.split()[0]] += 1
        v = sum(c for o, c in ops.items() if o.startswith('v_'))
        mov = sum(c for o, c in ops.items() if o.startswith('v_mov'))
        f64 = sum(c for o, c in ops.items() if o.endswith(('f64', 'f64_e32', 'f64_e64')))
        print("%s: total %d VALU %d (f64 %d, v_mov %d) s_mov %d lanes %d" % (
            name[:60], sum(ops.values()), v, f64, mov, ops['s_mov_b32'] + ops['s_mov_b64'],
            ops['v_readlane_b32'] + ops['v_writelane_b32']))
