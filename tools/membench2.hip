// membench2.hip -- does the load width matter for the k-caching access pattern?
// Same layout as the kernel ([nblocks][klev][64] per field, NPROMA 64 = one
// wave per workgroup, 30 input planes + 24 output planes per level):
//  (a) every lane loads 8 B of every field (global_load_dwordx2), as the kernel;
//  (b) half-wave 16 B loads: lanes 0-31 load 16 B of field f, lanes 32-63 of
//      field f+1 (global_load_dwordx4), one instruction per two fields;
//  (c) as (b) but into LDS with global_load_lds_dwordx4, then ds_read_b64.
// build: hipcc --offload-arch=gfx950 -O3 tools/membench2.hip -o build/membench2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int NIN = 30, NOUT = 24, NP = 64;
struct Ptrs { const double* in[NIN]; double* out[NOUT]; };

__global__ void __launch_bounds__(64) pat_a(Ptrs p, int klev) {
  const int b = blockIdx.x, jl = threadIdx.x;
  double acc = 0.0;
  for (int k = 0; k < klev; k++) {
    const size_t i = ((size_t)b * klev + k) * NP + jl;
    double s = acc;
#pragma unroll
    for (int f = 0; f < NIN; f++) s += p.in[f][i];
#pragma unroll
    for (int f = 0; f < NOUT; f++) p.out[f][i] = s + f;
    acc = s * 1e-3;
  }
}

// (a2) as (a) in the kernel's addressing: uniform row index + lane byte offset
__global__ void __launch_bounds__(64) pat_a2(Ptrs p, int klev) {
  const int b = blockIdx.x, jl = threadIdx.x;
  const unsigned lo = jl * 8u;
  double acc = 0.0;
  for (int k = 0; k < klev; k++) {
    int kk = k;
    asm volatile("" : "+s"(kk));
    const size_t row = ((size_t)b * klev + kk) * NP;
    double s = acc;
#pragma unroll
    for (int f = 0; f < NIN; f++) s += *(const double*)((const char*)(p.in[f] + row) + lo);
#pragma unroll
    for (int f = 0; f < NOUT; f++) *(double*)((char*)(p.out[f] + row) + lo) = s + f;
    acc = s * 1e-3;
  }
}

__global__ void __launch_bounds__(64) pat_b(Ptrs p, int klev) {
  const int b = blockIdx.x, jl = threadIdx.x;
  const int half = jl >> 5, l2 = jl & 31;
  double acc = 0.0;
  for (int k = 0; k < klev; k++) {
    const size_t row = ((size_t)b * klev + k) * NP;
    double s = acc;
#pragma unroll
    for (int f = 0; f < NIN; f += 2) {
      const double* pa = p.in[f];
      const double* pb = p.in[f + 1];
      const double2 v = *(const double2*)((half ? pb : pa) + row + 2 * l2);
      s += v.x + v.y;          // not the lane's own column, but the same bytes move
    }
#pragma unroll
    for (int f = 0; f < NOUT; f++) p.out[f][row + jl] = s + f;
    acc = s * 1e-3;
  }
}

__global__ void __launch_bounds__(64) pat_c(Ptrs p, int klev) {
  __shared__ double buf[NIN * NP];
  const int b = blockIdx.x, jl = threadIdx.x;
  const int half = jl >> 5, l2 = jl & 31;
  double acc = 0.0;
  for (int k = 0; k < klev; k++) {
    const size_t row = ((size_t)b * klev + k) * NP;
#pragma unroll
    for (int f = 0; f < NIN; f += 2) {
      const double* pa = p.in[f];
      const double* pb = p.in[f + 1];
      __builtin_amdgcn_global_load_lds((const void*)((half ? pb : pa) + row + 2 * l2),
                                       (__attribute__((address_space(3))) void*)(buf + f * NP), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double s = acc;
#pragma unroll
    for (int f = 0; f < NIN; f++) s += buf[f * NP + jl];
#pragma unroll
    for (int f = 0; f < NOUT; f++) p.out[f][row + jl] = s + f;
    acc = s * 1e-3;
  }
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  f(); CHK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < reps; r++) {
    CHK(hipEventRecord(a)); f(); CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int ngptot = argc > 1 ? atoi(argv[1]) : 163840;
  const int klev = 137, nblocks = ngptot / NP;
  const size_t plane = (size_t)nblocks * klev * NP;
  Ptrs p;
  std::vector<void*> allocs;
  for (int f = 0; f < NIN; f++) { void* q; CHK(hipMalloc(&q, plane * 8)); CHK(hipMemset(q, 0, plane * 8)); p.in[f] = (const double*)q; allocs.push_back(q); }
  for (int f = 0; f < NOUT; f++) { void* q; CHK(hipMalloc(&q, plane * 8)); p.out[f] = (double*)q; allocs.push_back(q); }
  const double bytes = (double)(NIN + NOUT) * plane * 8;
  float ms;
  ms = time_it([&] { hipLaunchKernelGGL(pat_a, dim3(nblocks), dim3(NP), 0, 0, p, klev); }, 10);
  printf("{\"test\": \"a_dwordx2_per_lane\", \"ms\": %.4f, \"GBs\": %.1f}\n", ms, bytes / ms / 1e6);
  ms = time_it([&] { hipLaunchKernelGGL(pat_a2, dim3(nblocks), dim3(NP), 0, 0, p, klev); }, 10);
  printf("{\"test\": \"a2_dwordx2_saddr\", \"ms\": %.4f, \"GBs\": %.1f}\n", ms, bytes / ms / 1e6);
  ms = time_it([&] { hipLaunchKernelGGL(pat_b, dim3(nblocks), dim3(NP), 0, 0, p, klev); }, 10);
  printf("{\"test\": \"b_dwordx4_half_wave\", \"ms\": %.4f, \"GBs\": %.1f}\n", ms, bytes / ms / 1e6);
  ms = time_it([&] { hipLaunchKernelGGL(pat_c, dim3(nblocks), dim3(NP), 0, 0, p, klev); }, 10);
  printf("{\"test\": \"c_glds_dwordx4\", \"ms\": %.4f, \"GBs\": %.1f}\n", ms, bytes / ms / 1e6);
  for (void* q : allocs) CHK(hipFree(q));
  return 0;
}
