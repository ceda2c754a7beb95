// membench3.hip -- a synthetic model of the KSEG schedule: how memory traffic and
// per-level arithmetic overlap at 2 waves per SIMD.
//
// Same layout and traffic as the CLOUDSC k-caching kernel (26 input planes and
// 24 output planes per level of a [nblocks][klev][nproma] block, NPROMA 64 =
// one wave per workgroup), a persistent grid of 2048 one-wave workgroups (LDS
// caps residency at 2 waves per SIMD, as the real kernel's registers do)
// dequeuing whole blocks from an atomic counter, and per level a synthetic
// fp64 workload: `ilp` independent chains of `len` dependent FMAs each, seeded
// by the level's loads, feeding the level's stores.
//
//   ./membench3 <len> <ilp> [ngptot] [mode: 0 = persistent, 1 = one-shot grid] [waves per SIMD: 2]
// mode 2 = persistent, two adjacent levels per load/store step (len ignored).
// prints one JSON line: ms, algorithmic TB/s, FMAs per wave-level.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/membench3.hip -o build/membench3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                         \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                  \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int NIN = 26, NOUT = 24, MAXILP = 8;

struct Ptrs {
  const double* in[NIN];
  double* out[NOUT];
};

template <int ILP>
__device__ __forceinline__ void level(const Ptrs& p, size_t i, int len, double& carry) {
  double v[NIN];
#pragma unroll
  for (int f = 0; f < NIN; f++) v[f] = p.in[f][i];
  double x[ILP];
#pragma unroll
  for (int c = 0; c < ILP; c++) x[c] = v[c] + carry;
  const double y0 = v[4], y1 = v[5];
  for (int n = 0; n < len; n += 2) {
#pragma unroll
    for (int c = 0; c < ILP; c++) x[c] = __builtin_fma(x[c], 0.999999, y0);
#pragma unroll
    for (int c = 0; c < ILP; c++) x[c] = __builtin_fma(x[c], 0.999998, y1);
  }
  double s = carry;
#pragma unroll
  for (int f = 0; f < NIN; f++) s += v[f];
#pragma unroll
  for (int c = 0; c < ILP; c++) s += x[c];
#pragma unroll
  for (int f = 0; f < NOUT; f++) p.out[f][i] = s + f;
  carry = s * 1e-3;
}

template <int ILP>
__global__ void __launch_bounds__(64) persistent(Ptrs p, int klev, int nblocks, unsigned* counter, int len) {
  extern __shared__ double pad[];
  __shared__ int s_item;
  const int jl = threadIdx.x;
  for (;;) {
    if (jl == 0) s_item = (int)atomicAdd(counter, 1u);
    __syncthreads();
    const int b = s_item;
    __syncthreads();
    if (b >= nblocks) break;
    double carry = 0.0;
    for (int k = 0; k < klev; k++) level<ILP>(p, ((size_t)b * klev + k) * 64 + jl, len, carry);
  }
  if (jl == 1000) pad[0] = 0.0;   // keeps the dynamic LDS allocation
}

// mode 2: the persistent schedule, but each step loads and stores two adjacent
// levels together (1 KB contiguous per field and access pair instead of 512 B)
__device__ __forceinline__ void level_pair(const Ptrs& p, size_t i, double& carry) {
  double v[NIN], w[NIN];
#pragma unroll
  for (int f = 0; f < NIN; f++) { v[f] = p.in[f][i]; w[f] = p.in[f][i + 64]; }
  double s = carry, t;
#pragma unroll
  for (int f = 0; f < NIN; f++) s += v[f];
  t = s * 1e-3;
#pragma unroll
  for (int f = 0; f < NIN; f++) t += w[f];
#pragma unroll
  for (int f = 0; f < NOUT; f++) { p.out[f][i] = s + f; p.out[f][i + 64] = t + f; }
  carry = t * 1e-3;
}

__global__ void __launch_bounds__(64) persistent_pair(Ptrs p, int klev, int nblocks, unsigned* counter) {
  extern __shared__ double pad[];
  __shared__ int s_item;
  const int jl = threadIdx.x;
  for (;;) {
    if (jl == 0) s_item = (int)atomicAdd(counter, 1u);
    __syncthreads();
    const int b = s_item;
    __syncthreads();
    if (b >= nblocks) break;
    double carry = 0.0;
    int k = 0;
    for (; k + 1 < klev; k += 2) level_pair(p, ((size_t)b * klev + k) * 64 + jl, carry);
    if (k < klev) level<1>(p, ((size_t)b * klev + k) * 64 + jl, 0, carry);
  }
  if (jl == 1000) pad[0] = 0.0;
}

template <int ILP>
__global__ void __launch_bounds__(64) oneshot(Ptrs p, int klev, int len) {
  extern __shared__ double pad[];
  const int b = blockIdx.x, jl = threadIdx.x;
  double carry = 0.0;
  for (int k = 0; k < klev; k++) level<ILP>(p, ((size_t)b * klev + k) * 64 + jl, len, carry);
  if (jl == 1000) pad[0] = 0.0;
}

template <int ILP>
float run(Ptrs p, int klev, int nblocks, unsigned* counter, int len, int mode, size_t lds, int grid) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 6; rep++) {
    CHK(hipMemset(counter, 0, 4));
    CHK(hipEventRecord(a));
    if (mode == 2)
      hipLaunchKernelGGL(persistent_pair, dim3(grid), dim3(64), lds, 0, p, klev, nblocks, counter);
    else if (mode == 0)
      hipLaunchKernelGGL(persistent<ILP>, dim3(grid), dim3(64), lds, 0, p, klev, nblocks, counter, len);
    else
      hipLaunchKernelGGL(oneshot<ILP>, dim3(nblocks), dim3(64), lds, 0, p, klev, len);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (rep > 0 && ms < best) best = ms;
  }
  return best;
}

int main(int argc, char** argv) {
  const int len = argc > 1 ? atoi(argv[1]) : 0;
  const int ilp = argc > 2 ? atoi(argv[2]) : 1;
  const int ngptot = argc > 3 ? atoi(argv[3]) : 163840;
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  const int wps = argc > 5 ? atoi(argv[5]) : 2;   // waves per SIMD (LDS-capped residency)
  const int klev = 137, nblocks = ngptot / 64;
  const size_t plane = (size_t)nblocks * klev * 64;
  Ptrs p;
  std::vector<double*> bufs;
  for (int f = 0; f < NIN + NOUT; f++) {
    double* d;
    CHK(hipMalloc(&d, plane * sizeof(double)));
    CHK(hipMemset(d, 0, plane * sizeof(double)));
    bufs.push_back(d);
    if (f < NIN) p.in[f] = d;
    else p.out[f - NIN] = d;
  }
  unsigned* counter;
  CHK(hipMalloc(&counter, 4));
  // dynamic LDS per one-wave workgroup: 160 KB / (4 SIMDs * wps) caps residency at wps waves per SIMD
  const size_t lds = (160 * 1024) / (4 * wps) - 512;
  const int grid = 256 * 4 * wps;
  float ms = 0.0f;
  switch (ilp) {
    case 1: ms = run<1>(p, klev, nblocks, counter, len, mode, lds, grid); break;
    case 2: ms = run<2>(p, klev, nblocks, counter, len, mode, lds, grid); break;
    case 4: ms = run<4>(p, klev, nblocks, counter, len, mode, lds, grid); break;
    case 8: ms = run<8>(p, klev, nblocks, counter, len, mode, lds, grid); break;
    default: printf("ilp must be 1, 2, 4 or 8\n"); return 1;
  }
  const double bytes = (double)ngptot * klev * (NIN + NOUT) * 8.0;
  printf("{\"len\": %d, \"ilp\": %d, \"mode\": \"%s\", \"waves_per_simd\": %d, \"fma_per_wave_level\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n",
         len, ilp, mode == 0 ? "persistent" : (mode == 2 ? "persistent_pair" : "oneshot"), wps, len * ilp, ms, bytes / (ms * 1e-3) / 1e12);
  for (double* d : bufs) CHK(hipFree(d));
  CHK(hipFree(counter));
  return 0;
}
