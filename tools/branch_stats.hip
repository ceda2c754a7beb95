// Diagnostic: how many waves execute each physics branch body (per level-wave).
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -DCLOUDSC_BRANCH_STATS -I include
//        -I dwarf-p-cloudsc_amd/csrc tools/branch_stats.hip -shared -fPIC -o build/libbranch_stats.so
#include "../dwarf-p-cloudsc_amd/csrc/cloudsc_gpu.hip"
extern "C" int cloudsc_branch_stats(unsigned long long* out) {
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_branch_count), sizeof(unsigned long long) * 32));
  return 0;
}
