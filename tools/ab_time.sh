#!/bin/bash
# Same-box timing A/B of several library builds (box-to-box clock differences
# are ~5 %, so compare only within one call).  usage:
#   tools/ab_time.sh "<sweep args>" lib1.so lib2.so ...   (interleaved, 2 rounds)
args=$1; shift
mkdir -p gpurun_out
for round in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    CLOUDSC_AMD_LIB=$(realpath $lib) timeout -k 10 300 python tools/sweep.py $args --reps 20 > gpurun_out/abt_${tag}_$round.log 2>&1 || exit $?
    python3 -c "
import json,sys
for l in open('gpurun_out/abt_${tag}_$round.log'):
    if l.startswith('{'):
        r=json.loads(l); print('%-28s round $round %-7s %-4s %s %-5s %8.4f ms %7.2f Mcol/s' % ('$tag', r['variant'], r['cfg'], r['precision'], r['nproma'], r['kernel_ms_median'], r['Mcol_per_s']))
"
  done
done
