// membench4.hip -- HBM placement of the k-caching kernel's streams (diagnostic).
//
// The memory-only model of membench3 (26 input and 24 output planes per level,
// NPROMA 64 = one wave per workgroup, persistent grid at 2 waves per SIMD,
// blocks dequeued in order) with the field placement as the variable:
//   0  one hipMalloc per field (the state's default: scattered 2 MiB pages)
//   1  one arena, fields one after the other, field i at a 2 MiB boundary
//   2  one arena, fields interleaved per level: [block][level][field][64]
//      (a wave's 26 loads of one level are ONE contiguous 13 KB run, its 24
//      stores another)
// and the arena allocated with hipMalloc or hipExtMallocWithFlags(contiguous).
// Every configuration is allocated `reps` times (fresh memory each time) and
// timed (best of 5 launches after a warm-up) to show the spread.
//
//   ./membench4 <layout 0|1|2> <contiguous 0|1> [reps 3] [len 0] [ngptot 163840] [nt 1]
// build: hipcc --offload-arch=gfx950 -O3 tools/membench4.hip -o build/membench4
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

constexpr int NIN = 26, NOUT = 24;

struct Layout {
  const double* in[NIN];
  double* out[NOUT];
  long long bstride, kstride;   // elements between blocks / levels of one field
};

template <bool NT>
__global__ void __launch_bounds__(64) persistent(Layout p, int klev, int nblocks, unsigned* counter, int len) {
  extern __shared__ double pad[];
  __shared__ int s_item;
  const int jl = threadIdx.x;
  for (;;) {
    if (jl == 0) s_item = (int)atomicAdd(counter, 1u);
    __syncthreads();
    const int b = __builtin_amdgcn_readfirstlane(s_item);
    __syncthreads();
    if (b >= nblocks) break;
    double carry = 0.0;
    for (int kk = 0; kk < klev; kk++) {
      // the CLOUDSC kernel's addressing: uniform element index (SGPRs) + the
      // lane's 32-bit byte offset, i.e. global_load/store ... v_off, s[base]
      int k = kk;
      asm volatile("" : "+s"(k));
      unsigned lo = (unsigned)jl * 8u;
      asm volatile("" : "+v"(lo));
      const size_t u = (size_t)b * p.bstride + (size_t)k * p.kstride;
      double v[NIN];
#pragma unroll
      for (int f = 0; f < NIN; f++)
        v[f] = NT ? __builtin_nontemporal_load((const double*)((const char*)(p.in[f] + u) + lo))
                  : *(const double*)((const char*)(p.in[f] + u) + lo);
      double s = carry;
#pragma unroll
      for (int f = 0; f < NIN; f++) s += v[f];
#pragma unroll 8
      for (int n = 0; n < len; n++) s = __builtin_fma(s, 0.999999, v[n & 7]);
#pragma unroll
      for (int f = 0; f < NOUT; f++)
        if (NT) __builtin_nontemporal_store(s + f, (double*)((char*)(p.out[f] + u) + lo));
        else *(double*)((char*)(p.out[f] + u) + lo) = s + f;
      carry = s * 1e-3;
    }
  }
  if (jl == 1000) pad[0] = 0.0;
}

int main(int argc, char** argv) {
  const int layout = argc > 1 ? atoi(argv[1]) : 0;
  const int contig = argc > 2 ? atoi(argv[2]) : 0;
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  const int len = argc > 4 ? atoi(argv[4]) : 0;
  const int ngptot = argc > 5 ? atoi(argv[5]) : 163840;
  const int nt = argc > 6 ? atoi(argv[6]) : 1;   // non-temporal loads and stores (the kernel's policy)
  const int klev = 137, nblocks = ngptot / 64, wps = 2;
  const size_t plane = (size_t)nblocks * klev * 64;
  const size_t two_mb = (size_t)2 << 20;
  const size_t span = (plane * sizeof(double) + two_mb - 1) / two_mb * two_mb;
  unsigned* counter;
  CHK(hipMalloc(&counter, 4));
  const size_t lds = (160 * 1024) / (4 * wps) - 512;
  const int grid = 256 * 4 * wps;
  auto alloc = [&](size_t bytes) {
    void* d = nullptr;
    if (contig) CHK(hipExtMallocWithFlags(&d, bytes, hipDeviceMallocContiguous));
    else CHK(hipMalloc(&d, bytes));
    CHK(hipMemset(d, 0, bytes));
    return (double*)d;
  };
  for (int r = 0; r < reps; r++) {
    Layout p;
    std::vector<double*> bufs;
    if (layout == 0) {
      for (int f = 0; f < NIN + NOUT; f++) {
        double* d = alloc(plane * sizeof(double));
        bufs.push_back(d);
        if (f < NIN) p.in[f] = d; else p.out[f - NIN] = d;
      }
      p.bstride = (long long)klev * 64; p.kstride = 64;
    } else if (layout == 1) {
      double* a = alloc(span * (NIN + NOUT));
      bufs.push_back(a);
      for (int f = 0; f < NIN + NOUT; f++) {
        double* d = (double*)((char*)a + f * span);
        if (f < NIN) p.in[f] = d; else p.out[f - NIN] = d;
      }
      p.bstride = (long long)klev * 64; p.kstride = 64;
    } else {
      double* ai = alloc(plane * NIN * sizeof(double));
      double* ao = alloc(plane * NIN * sizeof(double));   // NIN planes per level: the store fields padded to the load stride
      bufs.push_back(ai); bufs.push_back(ao);
      for (int f = 0; f < NIN; f++) p.in[f] = ai + f * 64;
      for (int f = 0; f < NOUT; f++) p.out[f] = ao + f * 64;
      p.bstride = 0; p.kstride = 0;   // per-arena strides below
    }
    float best = 1e30f;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (int rep = 0; rep < 6; rep++) {
      CHK(hipMemset(counter, 0, 4));
      CHK(hipEventRecord(e0));
      if (layout == 2) {
        // inputs and outputs have different field counts: run with the input
        // arena's strides for loads and the output arena's for stores by
        // giving the kernel per-field bases that already include the field
        // offset and a common (block, level) stride in units of 64 doubles;
        // both arenas use NIN fields per level (outputs padded to NIN planes).
        Layout q = p;
        q.bstride = (long long)klev * NIN * 64; q.kstride = (long long)NIN * 64;
        if (nt) hipLaunchKernelGGL(persistent<true>, dim3(grid), dim3(64), lds, 0, q, klev, nblocks, counter, len);
        else hipLaunchKernelGGL(persistent<false>, dim3(grid), dim3(64), lds, 0, q, klev, nblocks, counter, len);
      } else {
        if (nt) hipLaunchKernelGGL(persistent<true>, dim3(grid), dim3(64), lds, 0, p, klev, nblocks, counter, len);
        else hipLaunchKernelGGL(persistent<false>, dim3(grid), dim3(64), lds, 0, p, klev, nblocks, counter, len);
      }
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;
    }
    const double bytes = (double)ngptot * klev * (NIN + NOUT) * 8.0;
    printf("{\"layout\": %d, \"contiguous\": %d, \"nt\": %d, \"replica\": %d, \"len\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n",
           layout, contig, nt, r, len, best, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
    for (double* d : bufs) CHK(hipFree(d));
  }
  CHK(hipFree(counter));
  return 0;
}
