#!/bin/bash
# rocprofv3 counter passes for one kernel configuration (each pass its own run,
# --pmc with --kernel-trace only).  usage: tools/pmc_session.sh <tag> <prof_kernel.py args...>
# PMC_PREC=F32 counts the fp32 VALU instruction classes instead of the fp64 ones.
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_$tag
mkdir -p $out
passes=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_LDS"
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_IFETCH"
 "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_INST_REQ"
 "FETCH_SIZE"
 "WRITE_SIZE"
 "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU_TRANS_${PMC_PREC:-F64} SQ_INSTS_VALU_FMA_${PMC_PREC:-F64} SQ_INSTS_VALU_MUL_${PMC_PREC:-F64} SQ_INSTS_VALU_ADD_${PMC_PREC:-F64}"
 "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-trace --kernel-include-regex "kcache_entry|scc_entry|kseg_entry" \
     -d $out/p$i -o run --output-format csv -- python3 $R/tools/prof_kernel.py "$@" > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $p"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
done
