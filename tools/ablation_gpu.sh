#!/bin/bash
# GPU side of tools/ablation.sh: (1) interleaved kernel time of every build on
# one set of device fields (tools/ab_interleave.py, full kernel first);
# (2) one rocprofv3 counter pass per build: wave count, VALU / SALU
# instructions, the fp64 VALU classes, busy cycles and the GRBM clock pair
# (effective clock = GRBM_GUI_ACTIVE / kernel time).  Output under
# gpurun_out/<tag>/.   usage: tools/ablation_gpu.sh [libdir] [fp64|fp32] [tag]
dir=${1:-build/abl}
prec=${2:-fp64}
P=$([ "$prec" = fp32 ] && echo F32 || echo F64)
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/${3:-abl}
mkdir -p $out
libs=($dir/full.so)
for f in $dir/*.so; do [ "$f" != "$dir/full.so" ] && libs+=($f); done
timeout -k 10 300 python3 -u $R/tools/ab_interleave.py --precision $prec --rounds 30 --warmup 10 "${libs[@]}" > $out/times.txt 2>&1
rc=$?; echo "interleave rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/times.txt; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for f in "${libs[@]}"; do
  n=$(basename $f .so)
  CLOUDSC_AMD_LIB=$R/$f timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FMA_$P \
      SQ_INSTS_VALU_MUL_$P SQ_INSTS_VALU_ADD_$P SQ_INSTS_VALU_TRANS_$P SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
      --kernel-trace --kernel-include-regex kseg_entry -d $out/pmc_$n -o run --output-format csv \
      -- python3 $R/tools/prof_kernel.py --precision $prec --variant kseg --nproma 64 --reps 5 > $out/pmc_$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/pmc_$n.log; exit $rc; }
done
exit 0
