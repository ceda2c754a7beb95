#!/bin/bash
# Static statistics of the main kernels for a set of extra compile flags:
#   tools/kstat.sh "<flags>"
# VGPR / scratch / occupancy from the compiler remarks, and instruction counts
# (VALU, SALU, scalar loads, scratch ops, vmcnt(0) waits, SGPR-spill lane ops)
# from the assembly.  The assembly stays in /tmp/kstat.s.
cd "$(dirname "$0")/../dwarf-p-cloudsc_amd" || exit 1
hipcc -O3 -ffp-contract=off -fPIC -std=c++17 --offload-arch=gfx950 -mllvm -disable-machine-licm -I../include -Icsrc \
  --cuda-device-only -S csrc/cloudsc_gpu.hip -o /tmp/kstat.s $1 -Rpass-analysis=kernel-resource-usage 2> /tmp/kstat.err || exit 1
declare -A NAMES=(
  [_Z10kseg_entryIdLi2ELi0ELb0ELb0EEvN7cloudsc5KArgsIT_EENS0_11PersistArgsIS2_EE]="kseg<double,2,0>"
  [_Z12kcache_entryIdLi2ELi0ELb0ELb0EEvN7cloudsc5KArgsIT_EE]="kcache<double,2,0>"
  [_Z12kcache_entryIfLi4ELi0ELb0ELb1EEvN7cloudsc5KArgsIT_EE]="kcache<float,4,0,lds>"
)
for k in "${!NAMES[@]}"; do
  awk "/^$k:/,/s_endpgm/" /tmp/kstat.s > /tmp/kstat_k.s
  res=$(grep -A12 "Function Name: $k" /tmp/kstat.err | grep -E "VGPRs:|ScratchSize|Occupancy" | head -3 |
        sed 's/.*remark: //;s/ \[-Rpass.*//;s/ \[bytes\/lane\]//;s/ \[waves\/SIMD\]//' | tr -s ' ' | tr '\n' ' ')
  printf "%-24s %s valu=%d salu=%d sload=%d lgkm=%d scratch=%d vmcnt0=%d lane=%d\n" "${NAMES[$k]}" "$res" \
    "$(grep -cE '^\s+v_' /tmp/kstat_k.s)" "$(grep -cE '^\s+s_' /tmp/kstat_k.s)" "$(grep -c 's_load' /tmp/kstat_k.s)" \
    "$(grep -c 'lgkmcnt' /tmp/kstat_k.s)" "$(grep -c 'scratch_' /tmp/kstat_k.s)" "$(grep -c 'vmcnt(0)' /tmp/kstat_k.s)" \
    "$(grep -c 'lane_b32' /tmp/kstat_k.s)"
done
