// tools/layout_probe.hip -- does an interleaved output layout take the kernel
// out of the placement lottery?  (round 6)
//
// The KSEG kernel writes 24 output planes per wave and level (5 level fields,
// the 5 species planes of tendency_loc_cld, 14 half-level fluxes), each a
// 512-byte run of a different allocation.  Output sets of the same shape run up
// to 15-19 % apart depending on where their pages land.
// This probe writes (and optionally reads) field sets exactly in the kernel's
// order -- one wave per 64-column block, level by level, one level of input
// lookahead, write-through (sc1) or non-temporal stores -- over several output
// LAYOUTS, NSETS fresh sets each, allocated alternately, timed round-robin:
//   P  planar: one hipMalloc per field, [block][level][64] (the reference layout)
//   I  interleaved rows: one hipMalloc per set, [block][row][24 planes][64]; row
//      k holds level k's 10 level/species planes then half level k+1's 14
//      fluxes, so a wave-level's 24 stores are ONE contiguous 12 KiB run
//   B  block-major: one hipMalloc per set, [block][field plane][row][64]
// Per layout: the median of every set and the spread (slowest / fastest - 1).
// A layout whose spread stays within the timing noise is placement-free.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/layout_probe.hip -o build/layout_probe
//   build/layout_probe [nsets=6] [rounds=12] [read=1] [pace=0] [store=sc1|nt] [layouts=SP,SB,PP,PB,BB]
// A layout is <inputs><outputs>, each P, I or B as above; inputs S = one shared planar
// input set for every output set (what the first runs used).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(2);                                                                                \
    }                                                                                              \
  } while (0)

constexpr int kLanes = 64, kLev = 137, kRows = kLev + 1, kBlocks = 2560;
constexpr int kOutLevel = 5, kOutSpecies = 5, kOutHalf = 14, kPlanes = kOutLevel + kOutSpecies + kOutHalf;
constexpr int kInLevel = 17, kInSpecies = 8;   // + paph: the kernel's 26 input planes per level
constexpr size_t kPlane = (size_t)kBlocks * kRows * kLanes;   // elements of one plane (rows padded to 138)

// one output set: 24 plane bases + the element stride between consecutive rows
// and between consecutive blocks of each plane (the layouts differ only there)
struct OutSet {
  double* p[kPlanes];
  long long row_stride, block_stride;
};
constexpr int kIn = kInLevel + kInSpecies + 1;
struct InSet {
  const double* p[kIn];
  long long row_stride, block_stride;
};

template <bool WT>
__device__ __forceinline__ void st(double* p, double v) {
  if constexpr (WT)
    __hip_atomic_store((unsigned long long*)p, __double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    __builtin_nontemporal_store(v, p);
}

template <bool WT, bool READ>
__global__ void __launch_bounds__(64) probe(const OutSet o, const InSet in, int pace) {
  constexpr int NL = kInLevel + kInSpecies + 1;
  const int lane = threadIdx.x;
  for (int b = blockIdx.x; b < kBlocks; b += gridDim.x) {
    const size_t ob = (size_t)b * o.block_stride + lane;
    const size_t ib = (size_t)b * in.block_stride + lane;
    double nxt[NL], acc = 0.0;
    auto load = [&](int k) {
      if constexpr (READ) {
#pragma unroll
        for (int q = 0; q < NL; q++) nxt[q] = __builtin_nontemporal_load(in.p[q] + ib + (size_t)k * in.row_stride);
      }
    };
    load(0);
    // half level 0 (flux_top): row 0's flux planes
#pragma unroll
    for (int q = kOutLevel + kOutSpecies; q < kPlanes; q++) st<WT>(o.p[q] + ob, (double)b);
    for (int k = 0; k < kLev; k++) {
      double cur[NL];
#pragma unroll
      for (int q = 0; q < NL; q++) cur[q] = READ ? nxt[q] : 0.0;
      if (k + 1 < kLev) load(k + 1);
      double v = (double)(b + k);
      for (int i = 0; i < pace; i++) v = __builtin_fma(v, 0.999999, 1e-9);   // compute stand-in
      const size_t r0 = ob + (size_t)k * o.row_stride, r1 = r0 + o.row_stride;
#pragma unroll
      for (int q = 0; q < kOutLevel + kOutSpecies; q++) st<WT>(o.p[q] + r0, v);
#pragma unroll
      for (int q = kOutLevel + kOutSpecies; q < kPlanes; q++) st<WT>(o.p[q] + r1, v);
#pragma unroll
      for (int q = 0; q < NL; q++) acc += cur[q];
    }
    if (READ) st<WT>(o.p[0] + ob + (size_t)kLev * o.row_stride, acc);   // (row 137 of a level plane: padding)
  }
}

// A layout of np planes: P = one hipMalloc per plane ([block][row][64] each);
// I = one hipMalloc, [block][row][np planes][64]; B = one hipMalloc,
// [block][plane][row][64].  Returns the plane bases and the two strides.
void make_planes(char layout, int np, double** p, long long* row_stride, long long* block_stride,
                 std::vector<void*>& owned) {
  const size_t pb = kPlane * sizeof(double);
  if (layout == 'P') {
    for (int q = 0; q < np; q++) {
      void* a;
      CK(hipMalloc(&a, pb));
      CK(hipMemset(a, 0, pb));
      owned.push_back(a);
      p[q] = (double*)a;
    }
    *row_stride = kLanes;
    *block_stride = (long long)kRows * kLanes;
    return;
  }
  void* a;
  CK(hipMalloc(&a, pb * np));
  CK(hipMemset(a, 0, pb * np));
  owned.push_back(a);
  double* base = (double*)a;
  if (layout == 'I') {
    // outputs: row k = planes 0..9 (level k) then 10..23 (half level k); a wave
    // at level k stores 0..9 of row k and 10..23 of row k+1: one contiguous run
    for (int q = 0; q < np; q++) p[q] = base + (size_t)q * kLanes;
    *row_stride = (long long)np * kLanes;
    *block_stride = (long long)kRows * np * kLanes;
  } else {   // 'B'
    for (int q = 0; q < np; q++) p[q] = base + (size_t)q * kRows * kLanes;
    *row_stride = kLanes;
    *block_stride = (long long)np * kRows * kLanes;
  }
}

int main(int argc, char** argv) {
  const int nsets = argc > 1 ? atoi(argv[1]) : 6, rounds = argc > 2 ? atoi(argv[2]) : 12;
  const bool read = argc > 3 ? atoi(argv[3]) != 0 : true;
  const int pace = argc > 4 ? atoi(argv[4]) : 0;
  const bool wt = argc > 5 ? std::strcmp(argv[5], "nt") != 0 : true;
  // layouts: comma-separated pairs <inputs><outputs>; input S = one shared planar input set
  const std::string spec = argc > 6 ? argv[6] : "SP,SB,PP,PB,BB";
  std::vector<std::string> layouts;
  for (size_t a = 0; a <= spec.size();) {
    size_t e = spec.find(',', a);
    if (e == std::string::npos) e = spec.size();
    layouts.push_back(spec.substr(a, e - a));
    a = e + 1;
  }
  std::vector<void*> owned;
  InSet shared;
  {
    double* p[kIn];
    make_planes('P', kIn, p, &shared.row_stride, &shared.block_stride, owned);
    for (int q = 0; q < kIn; q++) shared.p[q] = p[q];
  }
  // sets allocated alternately across layouts, so each layout sees the allocator in the same states
  std::vector<OutSet> outs;
  std::vector<InSet> ins;
  std::vector<int> lay;
  for (int i = 0; i < nsets; i++)
    for (int L = 0; L < (int)layouts.size(); L++) {
      InSet in = shared;
      if (layouts[L][0] != 'S') {
        double* p[kIn];
        make_planes(layouts[L][0], kIn, p, &in.row_stride, &in.block_stride, owned);
        for (int q = 0; q < kIn; q++) in.p[q] = p[q];
      }
      OutSet o;
      make_planes(layouts[L][1], kPlanes, o.p, &o.row_stride, &o.block_stride, owned);
      ins.push_back(in);
      outs.push_back(o);
      lay.push_back(L);
    }
  const int n = (int)outs.size();
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&](int s) {
    const OutSet& o = outs[s];
    const InSet& in = ins[s];
    if (wt && read) hipLaunchKernelGGL((probe<true, true>), dim3(2048), dim3(64), 0, nullptr, o, in, pace);
    else if (wt) hipLaunchKernelGGL((probe<true, false>), dim3(2048), dim3(64), 0, nullptr, o, in, pace);
    else if (read) hipLaunchKernelGGL((probe<false, true>), dim3(2048), dim3(64), 0, nullptr, o, in, pace);
    else hipLaunchKernelGGL((probe<false, false>), dim3(2048), dim3(64), 0, nullptr, o, in, pace);
  };
  for (int w = 0; w < 30; w++) launch(w % n);   // clock warm-up
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> ms(n);
  for (int r = 0; r < rounds; r++)
    for (int i = 0; i < n; i++) {
      const int s = (r & 1) ? n - 1 - i : i;
      CK(hipEventRecord(e0, nullptr));
      launch(s);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float t = 0.f;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[s].push_back(t);
    }
  for (int L = 0; L < (int)layouts.size(); L++) {
    std::vector<float> med;
    for (int s = 0; s < n; s++) {
      if (lay[s] != L) continue;
      auto v = ms[s];
      std::sort(v.begin(), v.end());
      med.push_back(v[v.size() / 2]);
    }
    std::printf("{\"layout\": \"%s\", \"read\": %d, \"pace\": %d, \"store\": \"%s\", \"set_medians_ms\": [",
                layouts[L].c_str(), (int)read, pace, wt ? "sc1" : "nt");
    for (size_t i = 0; i < med.size(); i++) std::printf("%s%.4f", i ? ", " : "", med[i]);
    auto sorted = med;
    std::sort(sorted.begin(), sorted.end());
    std::printf("], \"median_ms\": %.4f, \"fastest_ms\": %.4f, \"slowest_ms\": %.4f, \"spread\": %.4f}\n",
                sorted[sorted.size() / 2], sorted.front(), sorted.back(), sorted.back() / sorted.front() - 1.0);
  }
  for (void* p : owned) CK(hipFree(p));
  return 0;
}
