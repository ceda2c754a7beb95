#!/bin/bash
# Per-phase cost of the fp64 KSEG kernel: build the kernel
# with one section of the physics ablated at a time (CLOUDSC_ABLATE bits,
# csrc/cloudsc_kcache.h), plus the full kernel and the memory-only one
# (CLOUDSC_ABLATE_PHYSICS), each as a one-kernel experiment library
# (CLOUDSC_ONLY_KSEG=8).  CPU side only; tools/ablation_gpu.sh measures them.
#   tools/ablation.sh [outdir] [element size: 8 (fp64, default) | 4 (fp32)]
set -e
out=${1:-build/abl}
es=${2:-8}
mkdir -p $out
declare -A masks=([full]=0 [supsat]=1 [conv]=2 [erosion]=4 [newton]=8 [cond]=16 [depos]=32 [sedim]=64
                  [auto]=128 [melt]=256 [evap]=512 [trunc]=1024 [solve]=2048 [sat]=4096)
cd "$(dirname "$0")/../dwarf-p-cloudsc_amd"
pids=()
for name in "${!masks[@]}"; do
  make -s variant "VFLAGS=-DCLOUDSC_ONLY_KSEG=$es -DCLOUDSC_ABLATE=${masks[$name]}" OUT=../$out/$name.so \
      > /tmp/abl_$name.log 2>&1 &
  pids+=($!)
  if [ ${#pids[@]} -ge 6 ]; then wait ${pids[0]}; pids=("${pids[@]:1}"); fi
done
make -s variant "VFLAGS=-DCLOUDSC_ONLY_KSEG=$es -DCLOUDSC_ABLATE_PHYSICS" OUT=../$out/memonly.so > /tmp/abl_memonly.log 2>&1
wait
ls ../$out
