#!/bin/bash
# KSEG kernel time for a list of segment counts, for each given library build
# usage: tools/nseg_quick.sh "1,2,4" lib1.so lib2.so ...
nsegs=$1; shift
for lib in "$@"; do
  CLOUDSC_AMD_LIB=$(realpath $lib) timeout -k 10 300 python tools/sweep.py --variants kseg --precisions fp64 \
    --nproma 64 --nsegs $nsegs --reps 20 > gpurun_out/nq_$(basename $lib .so).log 2>&1 || exit $?
  python3 -c "
import json
for l in open('gpurun_out/nq_$(basename $lib .so).log'):
    if l.startswith('{'):
        r=json.loads(l); print('%-16s nseg %-3s %8.4f ms' % ('$(basename $lib .so)', r['nseg'], r['kernel_ms_median']))
"
done
