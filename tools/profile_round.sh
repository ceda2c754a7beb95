#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace stats of the default
# bench command, then FETCH_SIZE / WRITE_SIZE passes (each its own run, --pmc
# with --kernel-trace only) for the bench kernel -> gpurun_out/prof/.
# usage: tools/profile_round.sh [variant] [precision] [nproma]
variant=${1:-kseg}; prec=${2:-fp64}; nproma=${3:-64}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
out=$R/gpurun_out/prof
mkdir -p $out
# the FETCH pass also counts GRBM_GUI_ACTIVE (GPU busy cycles, summed over the 8 XCDs): with the
# dispatch durations of the same pass it gives the effective shader clock of the box
for c in FETCH_SIZE WRITE_SIZE; do
  pmc=$c; [ $c == FETCH_SIZE ] && pmc="FETCH_SIZE GRBM_GUI_ACTIVE"
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-trace -d $out/pmc_${c}_${variant}_${prec} -o run --output-format csv \
    -- python3 $R/tools/prof_kernel.py --variant $variant --precision $prec --nproma $nproma --reps 3 \
    > $out/pmc_${c}_${variant}_${prec}.log 2>&1 || exit $?
done
python3 $R/tools/pmc_traffic.py ${variant}_${prec}_163840_${nproma} $out/pmc_FETCH_SIZE_${variant}_${prec} \
  $out/pmc_WRITE_SIZE_${variant}_${prec} $out/traffic.json
# the bench line reads its roofline.traffic from profiles/traffic_latest.json
python3 - <<PY
import json, os
src, dst = "$out/traffic.json", "$R/profiles/traffic_latest.json"
d = json.load(open(dst)) if os.path.exists(dst) else {}
d.update(json.load(open(src)))
json.dump(d, open(dst, "w"), indent=1, sort_keys=True)
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats_${variant}_${prec} -o bench --output-format csv \
  -- python3 $R/bench.py --steps 100 --warmup 5 --no-transfer --no-cpu-baseline --variant $variant --precision $prec \
  --nproma $nproma > $out/bench_under_rocprof_${variant}_${prec}.log 2>&1 || exit $?
# the --stats summary averages every launch of the kernel (placement probes, first step, prewarm, energy
# window); the timed launches alone, selected with the counts the bench line reports:
python3 $R/tools/timed_stats.py $(find $out/stats_${variant}_${prec} -name "*kernel_trace.csv" -print -quit) \
  $out/bench_under_rocprof_${variant}_${prec}.log $out/${variant}_${prec}_bench_kernel \
  > $out/timed_stats_${variant}_${prec}.json || exit $?
# counter calibration at the kernels' access widths (FETCH_SIZE and WRITE_SIZE passes of a known byte count)
if [ "${CALIB:-1}" == 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace -d $out/calib_$c -o calib --output-format csv \
      -- python3 $R/tools/calib_counters.py run > $out/calib_$c.log 2>&1 || exit $?
  done
  python3 $R/tools/calib_counters.py analyse $out/calib_FETCH_SIZE $out/calib_WRITE_SIZE $R/profiles/traffic_latest.json \
    > $out/calib.json || exit $?
fi
cp $R/profiles/traffic_latest.json $out/traffic_latest.json
