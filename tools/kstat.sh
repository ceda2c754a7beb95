#!/bin/bash
# static statistics of the main kernels for a set of extra compile flags:
# tools/kstat.sh "<flags>"
cd $(dirname $0)/../dwarf-p-cloudsc_amd
hipcc -O3 -ffp-contract=off -fPIC -std=c++17 --offload-arch=gfx950 -mllvm -disable-machine-licm -I../include -Icsrc \
  --cuda-device-only -S csrc/cloudsc_gpu.hip -o /tmp/kstat.s $1 -Rpass-analysis=kernel-resource-usage 2> /tmp/kstat.err || exit 1
for k in _Z10kseg_entryIdLi2ELi0ELb0EEvN7cloudsc5KArgsIT_EENS0_11PersistArgsIS2_EE _Z12kcache_entryIfLi3ELi1ELb0EEvN7cloudsc5KArgsIT_EE; do
  awk "/^$k:/,/s_endpgm/" /tmp/kstat.s > /tmp/kstat_k.s
  res=$(grep -A12 "Function Name: $k" /tmp/kstat.err | grep -E "VGPRs:|ScratchSize|Occupancy" | sed 's/.*remark: //;s/ \[-Rpass.*//' | tr '\n' ' ')
  echo "$k: $res valu=$(grep -cE '^\s+v_' /tmp/kstat_k.s) salu=$(grep -cE '^\s+s_' /tmp/kstat_k.s) sload=$(grep -c 's_load' /tmp/kstat_k.s) scratch=$(grep -c 'scratch_' /tmp/kstat_k.s) vmcnt0=$(grep -c 'vmcnt(0)' /tmp/kstat_k.s) lane=$(grep -c 'lane_b32' /tmp/kstat_k.s)" | sed 's/_Z10kseg_entryIdLi2ELi0ELb0EEvN7cloudsc5KArgsIT_EENS0_11PersistArgsIS2_EE/kseg<d,2,0>/;s/_Z12kcache_entryIfLi3ELi1ELb0EEvN7cloudsc5KArgsIT_EE/kcache<f,3,1>/'
done
