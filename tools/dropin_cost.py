#!/usr/bin/env python3
"""What the GPU drop-in cloudsc_c() costs inside the reference C dwarf
(VERDICT r04 weak 7 / next 8).

The unmodified reference dwarf (dwarf_cloudsc.c + cloudsc_driver.c + load_state.c
+ cloudsc_validate.c, oracle/Makefile target `dwarf`, in oracle/_ref/) is run
twice per configuration: linked with the reference kernel cloudsc_c.c
(dwarf-cloudsc-c, CPU) and with libcloudsc_c_amd_gpu.so (dwarf-cloudsc-c-amd-gpu:
every cloudsc_c() block call of the OpenMP loop -- cloudsc_driver.c:183-217 --
becomes H2D + kernel + D2H of that block on the MI355X through
cloudsc_host_run).  Per run: the driver's own TOTAL row (cloudsc_driver.c:
231-262: time of the block loop, MFlops/s, col/s) and whether its validation
table equals the reference kernel's.  One JSON line per run.

With the profiling build (dwarf-cloudsc-c-amd-gpu-prof, round 6) a third run
reports where each call's time goes: setup, pack, H2D, kernel, D2H, wait and
unpack (cloudsc_host_run_profile).

usage (GPU box): python tools/dropin_cost.py [cfg ...]   (cfg like "1 16384 32"; default: 1 16384 32, 4 163840 512)
"""
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(REPO, "oracle", "_ref")
DWARF_AMD = os.path.join(REPO, "dwarf-p-cloudsc_amd", "dwarf-cloudsc-amd")
DATA = os.path.join(REPO, "data", "cloudsc100")


def run(binary, args, cwd, want_stderr=False):
    env = dict(os.environ, OMP_NUM_THREADS=args.split()[0], OMP_SCHEDULE="static", OMP_STACKSIZE="512M")
    cmd = "ulimit -s unlimited && exec %s %s" % (binary, args)
    r = subprocess.run(["bash", "-c", cmd], cwd=cwd, capture_output=True, text=True, env=env, timeout=900)
    if r.returncode != 0:
        raise SystemExit("%s %s failed: %s" % (binary, args, (r.stdout + r.stderr)[-2000:]))
    return (r.stdout, r.stderr) if want_stderr else r.stdout


def profile_row(err):
    """The CLOUDSC_C_DROPIN_PROFILE line of the profiling build: per-call means
    (ms) of each part and its share of the calls' total."""
    m = re.search(r"CLOUDSC_C_DROPIN_PROFILE (.*)$", err, re.M)
    if not m:
        return None
    kv = {k: float(v) for k, v in (x.split("=") for x in m.group(1).split())}
    n = kv.pop("calls")
    mx = kv.pop("max_call_ms", None)
    first = {"calls": int(kv.pop("first_calls", 0)), "ms": kv.pop("first_calls_ms", None)}
    tot = kv["total_ms"]
    parts = ["alloc_ms", "setup_ms", "pack_ms", "enqueue_ms", "h2d_ms", "kernel_ms", "d2h_ms", "unpack_ms"]
    row = {"calls": int(n), "per_call_ms": {k: round(v / n, 4) for k, v in kv.items()},
           "share_of_total": {k: round(kv[k] / tot, 4) for k in parts + ["wait_ms"]}, "max_call_ms": mx,
           "first_calls": first}
    # host-side work (everything but the device's three operations) and the device's, over the calls
    # after each thread's first (which creates its context and starts the runtime: first_calls)
    host = kv["setup_ms"] + kv["pack_ms"] + kv["enqueue_ms"] + kv["unpack_ms"] + kv["alloc_ms"]
    row["host_side_share"] = round(host / tot, 4)
    row["device_side_share"] = round((kv["h2d_ms"] + kv["kernel_ms"] + kv["d2h_ms"]) / tot, 4)
    return row


def total_row(out):
    m = re.search(r"^\s*(\d+)\s+(\d+)\s+(\d+)\s+(\d+)\s+(\d+)\s+(-?\d+)\s*:\s*(\d+)\s+(\d+)\s+(\d+)\s+TOTAL", out, re.M)
    return None if not m else {"time_ms": int(m.group(7)), "mflops": int(m.group(8)), "col_s": int(m.group(9))}


def table(out):
    lines = out.splitlines()
    i = [k for k, l in enumerate(lines) if "Variable Dim" in l][0]
    return [l for l in lines[i + 1:] if l.strip()][:21]


def main():
    cfgs = sys.argv[1:] or ["1 16384 32", "4 163840 512"]
    with tempfile.TemporaryDirectory() as wd:
        r = subprocess.run([DWARF_AMD, "--data", DATA, "--write-h5", wd], capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stdout + r.stderr)
        for cfg in cfgs:
            ref = run(os.path.join(REF_BIN, "dwarf-cloudsc-c"), cfg, wd)
            gpu = run(os.path.join(REF_BIN, "dwarf-cloudsc-c-amd-gpu"), cfg, wd)
            prof_bin = os.path.join(REF_BIN, "dwarf-cloudsc-c-amd-gpu-prof")
            prof = run(prof_bin, cfg, wd, want_stderr=True) if os.path.exists(prof_bin) else None
            n = cfg.split()
            blocks = -(-int(n[1]) // int(n[2]))
            for kind, out in (("reference kernel cloudsc_c.c (CPU)", ref),
                              ("drop-in libcloudsc_c_amd_gpu.so (MI355X, per-block H2D + kernel + D2H)", gpu)):
                print(json.dumps({"cmd": cfg, "kernel": kind, "total": total_row(out), "blocks": blocks,
                                  "cloudsc_c_calls_per_thread": -(-blocks // int(n[0])),
                                  "validation_table_equal_to_reference": table(out) == table(ref)}), flush=True)
            if prof:
                print(json.dumps({"cmd": cfg, "kernel": "drop-in libcloudsc_c_amd_gpu_prof.so (the GPU form with "
                                  "cloudsc_host_run_profile on)", "total": total_row(prof[0]),
                                  "validation_table_equal_to_reference": table(prof[0]) == table(ref),
                                  "per_call_breakdown": profile_row(prof[1])}), flush=True)


if __name__ == "__main__":
    main()
