#!/bin/bash
# A/B of the bench line between libraries: rounds x libs, one JSON summary line per run
for round in 1 2 3; do
  for lib in "$@"; do
    CLOUDSC_AMD_LIB=$(realpath $lib) timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bab_$(basename $lib .so)_$round.log 2>&1 || exit 1
    python3 -c "
import json
l=[x for x in open('gpurun_out/bab_$(basename $lib .so)_$round.log') if x.startswith('{')][-1]
r=json.loads(l); print('$(basename $lib .so) round $round ms_per_step %.4f kernel_ms %.4f value %.1f' % (r['ms_per_step'], r['kernel_ms'], r['value']/1e6))"
  done
done
