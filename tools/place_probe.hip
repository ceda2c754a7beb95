// tools/place_probe.hip -- does the physical placement of a set of output
// fields decide their write rate?  (placement study)
//
// tools/placement_fields.py found the KSEG kernel up to 19 % slower for some
// states, the whole difference carried by the 21 OUTPUT fields (moving them to
// fresh allocations one by one recovered it; moving inputs did nothing), and
// the slow states show 5-10x the L2->memory write stalls for DRAM credits
// (TCC_EA0_WRREQ_DRAM_CREDIT_STALL, tools/placement_pmc.sh).  This probe takes
// the kernel out of it: NSETS sets of 21 fields of the fp64 half-level size
// (hipMalloc each), and a kernel that writes a set the way the KSEG kernel
// writes its outputs -- one wave per NPROMA block, level by level, one 512-byte
// nontemporal row per field and level.  The sets are timed round-robin; one
// JSON line per set, then the spread.
//   hipcc -O3 --offload-arch=gfx950 tools/place_probe.hip -o build/place_probe
//   build/place_probe [nsets] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(2);                                                                                \
    }                                                                                              \
  } while (0)

constexpr int kFields = 21, kNproma = 64, kLev = 138, kBlocks = 2560;
struct Set { double* f[kFields]; };

// grid: 2048 workgroups of 4 waves; wave w of the grid takes blocks w, w + nwaves, ...
__global__ void __launch_bounds__(256) write_set(const Set s) {
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  for (int b = wave; b < kBlocks; b += nwaves) {
    const size_t base = (size_t)b * kLev * kNproma + lane;
    for (int k = 0; k < kLev; k++) {
      const double v = (double)(b + k);
#pragma unroll
      for (int q = 0; q < kFields; q++) __builtin_nontemporal_store(v, s.f[q] + base + (size_t)k * kNproma);
    }
  }
}

// one field alone, the same pattern (one wave per block, level rows)
__global__ void __launch_bounds__(256) write_one(double* f) {
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  for (int b = wave; b < kBlocks; b += nwaves) {
    const size_t base = (size_t)b * kLev * kNproma + lane;
    for (int k = 0; k < kLev; k++) __builtin_nontemporal_store((double)(b + k), f + base + (size_t)k * kNproma);
  }
}

int main(int argc, char** argv) {
  const int nsets = argc > 1 ? atoi(argv[1]) : 12, rounds = argc > 2 ? atoi(argv[2]) : 20;
  const size_t bytes = (size_t)kBlocks * kLev * kNproma * sizeof(double);
  std::vector<Set> sets(nsets);
  for (auto& s : sets)
    for (auto& p : s.f) CK(hipMalloc((void**)&p, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(nsets);
  for (int r = 0; r < rounds + 3; r++)
    for (int i = 0; i < nsets; i++) {
      const int s = (r & 1) ? nsets - 1 - i : i;
      CK(hipEventRecord(e0, nullptr));
      hipLaunchKernelGGL(write_set, dim3(2048), dim3(256), 0, nullptr, sets[s]);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float t = 0.f;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r >= 3) ms[s].push_back(t);
    }
  float lo = 1e30f, hi = 0.f;
  for (int s = 0; s < nsets; s++) {
    std::sort(ms[s].begin(), ms[s].end());
    const float med = ms[s][ms[s].size() / 2];
    lo = std::min(lo, med);
    hi = std::max(hi, med);
    std::printf("{\"set\": %d, \"ms_median\": %.4f, \"GBs\": %.1f, \"first_field\": \"%p\"}\n", s, med,
                kFields * bytes / (med * 1e-3) / 1e9, (void*)sets[s].f[0]);
  }
  std::printf("{\"sets\": %d, \"bytes_per_set\": %zu, \"spread\": %.4f}\n", nsets, kFields * bytes, hi / lo - 1.0);
  // every field alone: median of 7 launches, in us, per set
  for (int s = 0; s < nsets; s++) {
    std::printf("{\"set\": %d, \"field_us\": [", s);
    for (int q = 0; q < kFields; q++) {
      std::vector<float> t1;
      for (int r = 0; r < 8; r++) {
        CK(hipEventRecord(e0, nullptr));
        hipLaunchKernelGGL(write_one, dim3(2048), dim3(256), 0, nullptr, sets[s].f[q]);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float t = 0.f;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (r) t1.push_back(t);
      }
      std::sort(t1.begin(), t1.end());
      std::printf("%s%.1f", q ? ", " : "", t1[t1.size() / 2] * 1e3);
    }
    std::printf("]}\n");
  }
  return 0;
}
