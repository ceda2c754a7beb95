#!/usr/bin/env python3
"""Experiment builds: copy the library sources to a scratch tree, apply textual
edits, and build build/lib<name>.so (not the product library).

usage: exp_variant.py <name> <edits.py> [extra hipcc flags...]
  edits.py defines EDITS = [(relative_file, old_text, new_text), ...]"""
import os
import runpy
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, edits_file = sys.argv[1], sys.argv[2]
    extra = sys.argv[3:]
    edits = runpy.run_path(edits_file)["EDITS"] if edits_file != "-" else []
    tmp = os.path.join("/tmp", "exp_" + name)
    shutil.rmtree(tmp, ignore_errors=True)
    shutil.copytree(os.path.join(REPO, "dwarf-p-cloudsc_amd", "csrc"), os.path.join(tmp, "csrc"))
    for rel, old, new in edits:
        p = os.path.join(tmp, "csrc", rel)
        s = open(p).read()
        if old not in s:
            sys.exit("edit does not apply to %s: %r" % (rel, old[:80]))
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(REPO, "build", "lib%s.so" % name)
    srcs = [os.path.join(tmp, "csrc", f) for f in ("cloudsc_gpu.hip", "cloudsc_state.hip", "cloudsc_pipeline.hip",
                                                     "cloudsc_cpu.hip", "cloudsc_hbm.hip", "cloudsc_place.hip")]
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-ffp-contract=off", "-fPIC", "-std=c++17", "--offload-arch=gfx950",
           "-Wno-unused-result", "-mllvm", "-disable-machine-licm", "-Xarch_host", "-mfma",
           "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(tmp, "csrc"), "-shared"] + extra + srcs + \
          ["-o", out]
    subprocess.check_call(cmd)
    # resource report of the main kernels
    r = subprocess.run(cmd[:-2 - len(srcs)] + [os.path.join(tmp, "csrc", "cloudsc_gpu.hip"), "-S",
                        "--cuda-device-only", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
    cur = None
    for line in r.stderr.splitlines():
        if "Function Name:" in line:
            cur = line.split("Function Name:")[1].split()[0]
        elif cur and ("kseg_entryId" in cur or "kcache_entryId" in cur or "kseg_entryIf" in cur) and \
                ("VGPRs:" in line or "ScratchSize" in line or "Occupancy" in line):
            print(cur[:40], line.split("remark:")[1].split("[-R")[0].strip())
    print("built", out)


if __name__ == "__main__":
    main()
