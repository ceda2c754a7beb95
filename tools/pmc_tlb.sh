#!/bin/bash
# Address-translation counters of the KSEG kernel (rocprofv3, one --pmc group
# per run, --kernel-trace only): UTCL1 requests / hits / misses, the UTCL1
# stalls, and how busy the UTCL2 is.  usage: tools/pmc_tlb.sh <tag> <prof_kernel.py args...>
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_$tag
mkdir -p $out
passes=(
 "TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_PERMISSION_MISS_sum"
 "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
 "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-trace --kernel-include-regex "${KREGEX:-kseg_entry|place_probe}" \
     -d $out/p$i -o run --output-format csv -- python3 $R/tools/${PROF_SCRIPT:-prof_kernel.py} "$@" > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $p"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
done
