// Diagnostic: how many waves execute each physics branch body (per level-wave).
// build: make -C dwarf-p-cloudsc_amd variant VFLAGS=-DCLOUDSC_BRANCH_STATS OUT=../build/libbranch_stats.so \
//          LIB_SRCS="../tools/branch_stats.hip csrc/cloudsc_state.hip csrc/cloudsc_pipeline.hip"
#include "../dwarf-p-cloudsc_amd/csrc/cloudsc_gpu.hip"
extern "C" int cloudsc_branch_stats(unsigned long long* out) {
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_branch_count), sizeof(unsigned long long) * 32));
  return 0;
}
