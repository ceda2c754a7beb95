#!/bin/bash
# interleaved config A/B with the knob library: cfgab.sh <precision> <rounds> cfg...
prec=$1; rounds=$2; shift 2
for r in $(seq 1 $rounds); do
  for c in "$@"; do
    CLOUDSC_AMD_LIB=ab/libcloudsc_knobs.so timeout -k 10 200 python tools/sweep.py --variants kseg --precisions $prec --nproma 64 --cfgs $c --reps 20 > gpurun_out/cfgab_${prec}_${c}_$r.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/cfgab_${prec}_${c}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print('round $r', d['precision'], 'cfg', d['cfg'], d['kernel_ms_median'])"
  done
done
