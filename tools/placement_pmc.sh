#!/bin/bash
# PMC passes of tools/placement_pmc.py (one rocprofv3 run per counter group);
# outputs under gpurun_out/ppmc_<pass>/.  Each pass is a new process, so a new
# placement: compare slow and fast states WITHIN a pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
passes=(
  "A TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum"
  "B TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_64B_sum"
  "C TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_PERMISSION_MISS_sum"
)
for p in "${passes[@]}"; do
  set -- $p; name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/ppmc_$name -o p \
    -- python3 -u tools/placement_pmc.py "${PLACE_ARGS[@]}" > gpurun_out/ppmc_$name.log 2>&1 || { echo "pass $name rc=$?"; exit 1; }
  echo "pass $name ok"
done
