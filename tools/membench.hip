// membench.hip -- memory ceiling of the CLOUDSC k-caching access pattern on MI355X.
//
// Same grid (NPROMA block -> workgroup, column -> lane), same field layout
// ([nblocks][klev][nproma] per field, 26 input planes + 24 output planes per
// level), same level loop -- but trivial arithmetic.  What this kernel achieves
// is the HBM ceiling the real kernel can hope for with the reference layout.
// Also: a plain streaming copy of the same byte count (the chip's achievable
// peak) and the same pattern with a "level-packed" layout (all fields of one
// level of one block contiguous) to see whether the layout costs bandwidth.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int NIN = 26, NOUT = 24;

struct Ptrs { const double* in[NIN]; double* out[NOUT]; };

// reference layout: field f at level k of block b: f[(b*klev + k)*nproma + jl]
template <int NI, int NO>
__global__ void __launch_bounds__(256) pattern_kernel(Ptrs p, int klev, int nproma) {
  const int b = blockIdx.x, jl = threadIdx.x;
  double acc = 0.0;
  for (int k = 0; k < klev; k++) {
    const size_t i = ((size_t)b * klev + k) * nproma + jl;
    double v[NI];
#pragma unroll
    for (int f = 0; f < NI; f++) v[f] = p.in[f][i];
    double s = acc;
#pragma unroll
    for (int f = 0; f < NI; f++) s += v[f];
#pragma unroll
    for (int f = 0; f < NO; f++) p.out[f][i] = s + f;
    acc = s * 1e-3;
  }
}

// level-packed layout: one chunk [field][nproma] per (block, level)
template <int NI, int NO>
__global__ void __launch_bounds__(256) packed_kernel(const double* in, double* out, int klev, int nproma) {
  const int b = blockIdx.x, jl = threadIdx.x;
  double acc = 0.0;
  for (int k = 0; k < klev; k++) {
    const size_t ci = (((size_t)b * klev + k) * NI) * nproma + jl;
    const size_t co = (((size_t)b * klev + k) * NO) * nproma + jl;
    double v[NI];
#pragma unroll
    for (int f = 0; f < NI; f++) v[f] = in[ci + (size_t)f * nproma];
    double s = acc;
#pragma unroll
    for (int f = 0; f < NI; f++) s += v[f];
#pragma unroll
    for (int f = 0; f < NO; f++) out[co + (size_t)f * nproma] = s + f;
    acc = s * 1e-3;
  }
}

__global__ void copy_kernel(const double4* __restrict__ in, double4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
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
  const int klev = 137;
  for (int nproma : {64, 128, 256}) {
    const int nblocks = ngptot / nproma;
    const size_t plane = (size_t)nblocks * klev * nproma;
    Ptrs p;
    std::vector<void*> allocs;
    for (int f = 0; f < NIN; f++) { void* q; CHK(hipMalloc(&q, plane * 8)); CHK(hipMemset(q, 0, plane * 8)); p.in[f] = (const double*)q; allocs.push_back(q); }
    for (int f = 0; f < NOUT; f++) { void* q; CHK(hipMalloc(&q, plane * 8)); p.out[f] = (double*)q; allocs.push_back(q); }
    const double bytes = (double)(NIN + NOUT) * plane * 8;
    float ms = time_it([&] { hipLaunchKernelGGL((pattern_kernel<NIN, NOUT>), dim3(nblocks), dim3(nproma), 0, 0, p, klev, nproma); }, 10);
    printf("{\"test\": \"reference_layout\", \"nproma\": %d, \"ms\": %.4f, \"GBs\": %.1f}\n", nproma, ms, bytes / ms / 1e6);
    void *pin, *pout;
    CHK(hipMalloc(&pin, plane * 8 * NIN)); CHK(hipMalloc(&pout, plane * 8 * NOUT));
    CHK(hipMemset(pin, 0, plane * 8 * NIN));
    ms = time_it([&] { hipLaunchKernelGGL((packed_kernel<NIN, NOUT>), dim3(nblocks), dim3(nproma), 0, 0, (const double*)pin, (double*)pout, klev, nproma); }, 10);
    printf("{\"test\": \"level_packed\", \"nproma\": %d, \"ms\": %.4f, \"GBs\": %.1f}\n", nproma, ms, bytes / ms / 1e6);
    if (nproma == 128) {
      const size_t n4 = plane * NIN / 4;
      ms = time_it([&] { hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, 0, (const double4*)pin, (double4*)pout, std::min(n4, plane * NOUT / 4)); }, 10);
      const double cb = 2.0 * 32.0 * std::min(n4, plane * NOUT / 4);
      printf("{\"test\": \"stream_copy\", \"bytes\": %.0f, \"ms\": %.4f, \"GBs\": %.1f}\n", cb, ms, cb / ms / 1e6);
    }
    CHK(hipFree(pin)); CHK(hipFree(pout));
    for (void* q : allocs) CHK(hipFree(q));
  }
  return 0;
}
