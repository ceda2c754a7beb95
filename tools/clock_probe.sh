#!/bin/bash
# Effective shader clock of this box while the fp64 KSEG kernel runs: one
# rocprofv3 pass counting GRBM_GUI_ACTIVE (busy cycles, summed over the 8 XCDs)
# with the kernel trace of the same dispatches -> gpurun_out/clock_probe.json
# (kernel ms and GHz per dispatch).  usage: tools/clock_probe.sh [reps] [-- program args...]
# (with "-- bench.py ...": the clock of every KSEG dispatch of that bench run)
reps=${1:-10}
shift
[ "$1" == "--" ] && shift
prog=("$@")
[ ${#prog[@]} -eq 0 ] && prog=(tools/prof_kernel.py --variant kseg --precision fp64 --nproma 64 --reps $reps)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
out=$R/gpurun_out/clock_probe
rm -rf $out && mkdir -p $out
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $out -o run --output-format csv \
  -- python3 $R/"${prog[0]}" "${prog[@]:1}" > $out/run.log 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, json, os, re, sys
d = sys.argv[1]
grbm, dur = {}, {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and "kseg_entry" in r["Kernel_Name"]:
            grbm[r["Dispatch_Id"]] = grbm.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "kseg_entry" in r["Kernel_Name"]:
            dur[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
rows = [{"dispatch": k, "kernel_ms": round(dur[k] / 1e6, 4), "sclk_ghz": round(grbm[k] / 8 / dur[k], 3)}
        for k in sorted(grbm, key=int) if dur.get(k)]
res = {"rows": rows, "median_kernel_ms": sorted(r["kernel_ms"] for r in rows)[len(rows) // 2],
       "median_sclk_ghz": sorted(r["sclk_ghz"] for r in rows)[len(rows) // 2]}
json.dump(res, open(os.path.join(os.path.dirname(d), "clock_probe.json"), "w"), indent=1)
print(json.dumps({k: res[k] for k in ("median_kernel_ms", "median_sclk_ghz")}))
PY
