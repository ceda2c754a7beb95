// cloudsc_hbm.hip -- the achievable-HBM measurement behind bench.py's
// roofline.achievable_peak (report achieved GB/s against the
// 8 TB/s spec AND against a STREAM-copy peak measured on the same box; the
// pool's boxes differ by 10+ % in this kernel, so the spec fraction alone does
// not normalise).
//
// A STREAM copy b[i] = a[i] over two device buffers, 16 B per lane per access,
// one tile per workgroup (each lane's loads of its tile in flight before its
// stores), cached or non-temporal; the figure is the best launch of any shape
// over three buffer pairs.  Bytes moved = 2 x buffer size per launch.
//
// Round 6 (the in-run figure read 5.9-6.27 TB/s where
// MI355X_MICROARCH.md quotes 6.29 TB/s): a sweep of shapes and buffer pairs
// (tools/stream_sweep.hip, profiles/r06/stream_sweep.jsonl) found the 16 KiB
// non-temporal tile the fastest shape by far (6.18-6.48 TB/s over three pairs
// on one box; persistent grid-stride forms with 2-16 loads in flight per lane
// at 16-64 waves per CU: 4.7-5.2 TB/s; 32 / 64 KiB tiles 4.4 / 5.6 TB/s), and
// the buffers' placement moving it by 5 %: so three pairs are measured (held
// together, so each gets pages of its own) and the best launch counts.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "cloudsc_amd.h"
#include "cloudsc_internal.h"

using namespace cloudsc_impl;

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// one workgroup per tile of 256 x U 16-B vectors: lane t copies t, t + 256, ...
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_tiles(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int q = 0; q < U; q++)
    if (base + q * 256 < n) v[q] = ld<NT>(a + base + q * 256);
#pragma unroll
  for (int q = 0; q < U; q++)
    if (base + q * 256 < n) st<NT>(b + base + q * 256, v[q]);
}

}  // namespace

extern "C" int cloudsc_hbm_copy_gbps(int device, long long bytes, int reps, double* gbps) {
  if (!gbps || bytes < (2 << 20) || reps <= 0) return CLOUDSC_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return CLOUDSC_ENODEV;
  HIPCHK(hipSetDevice(device));
  // three pairs of `bytes` / 2 each (the total footprint of one pair of `bytes`
  // times 1.5); each buffer stays far beyond the 256 MiB Infinity Cache
  constexpr int kPairs = 3;
  const size_t nvec = (size_t)bytes / 2 / sizeof(u32x4);
  void* buf[2 * kPairs] = {};
  int rc = CLOUDSC_OK;
  for (int i = 0; i < 2 * kPairs && rc == CLOUDSC_OK; i++)
    if (hipMalloc(&buf[i], nvec * sizeof(u32x4)) != hipSuccess) { (void)hipGetLastError(); rc = CLOUDSC_ENOMEM; }
  // the shapes tried; the achievable figure is the best launch of any of them
  struct Shape { void (*k)(const u32x4*, u32x4*, size_t); int vecs; };
  const Shape shapes[] = {{copy_tiles<4, true>, 1024}, {copy_tiles<2, true>, 512}, {copy_tiles<4, false>, 1024},
                          {copy_tiles<16, true>, 4096}};
  constexpr int ns = (int)(sizeof(shapes) / sizeof(shapes[0]));
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double best_ms = 0.0;
  hipError_t e = hipSuccess;
  if (rc == CLOUDSC_OK) {
    e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    for (int i = 0; i < 2 * kPairs && e == hipSuccess; i += 2)
      e = hipMemsetAsync(buf[i], 0x3c, nvec * sizeof(u32x4), st);
  }
  for (int pr = 0; pr < kPairs && rc == CLOUDSC_OK && e == hipSuccess; pr++) {
    const u32x4* a = (const u32x4*)buf[2 * pr];
    u32x4* b = (u32x4*)buf[2 * pr + 1];
    for (int r = -1; r < reps * ns && e == hipSuccess; r++) {
      const Shape& sh = shapes[(r < 0 ? 0 : r) % ns];   // r = -1: warm-up
      e = hipEventRecord(e0, st);
      if (e != hipSuccess) break;
      hipLaunchKernelGGL(sh.k, dim3((unsigned)((nvec + sh.vecs - 1) / sh.vecs)), dim3(256), 0, st, a, b, nvec);
      e = hipGetLastError();
      if (e == hipSuccess) e = hipEventRecord(e1, st);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      float ms = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
      if (e == hipSuccess && r >= 0 && (best_ms == 0.0 || ms < best_ms)) best_ms = ms;
    }
  }
  if (rc == CLOUDSC_OK && e != hipSuccess) rc = hip_fail(e, "hbm copy measurement");
  if (rc == CLOUDSC_OK) *gbps = 2.0 * (double)(nvec * sizeof(u32x4)) / (best_ms * 1e-3) / 1e9;
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  for (void* p : buf)
    if (p) (void)hipFree(p);
  return rc;
}

// The host<->device ceiling the host-buffer pipeline is held against (bench.py's
// pcie_inclusive): pinned host buffers of `bytes` each way, copied by the copy
// engines with one stream per direction (the fastest arrangement,
// tools/pcie_probe.hip: 97 GB/s both ways at once against 65-85 GB/s with 2-8
// streams per direction), in 64 MiB pieces; H2D alone, D2H alone, and both at
// once (total of the two directions); best of `reps` after one warm-up each.
extern "C" int cloudsc_pcie_gbps(int device, long long bytes, int reps, double* h2d, double* d2h, double* both) {
  if (!h2d || !d2h || !both || bytes < (1 << 20) || reps <= 0) return CLOUDSC_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return CLOUDSC_ENODEV;
  HIPCHK(hipSetDevice(device));
  const size_t nb = (size_t)bytes;
  char *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  hipStream_t s_in = nullptr, s_out = nullptr;
  hipError_t e = hipHostMalloc((void**)&h_in, nb, hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc((void**)&h_out, nb, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc((void**)&d_in, nb);
  if (e == hipSuccess) e = hipMalloc((void**)&d_out, nb);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMemset(d_out, 1, nb);
  if (e == hipSuccess) std::fill(h_in, h_in + nb, (char)2);
  const size_t piece = (size_t)64 << 20;
  double best[3] = {0, 0, 0};
  for (int dir = 1; dir <= 3 && e == hipSuccess; dir++) {
    for (int r = -1; r < reps && e == hipSuccess; r++) {
      e = hipDeviceSynchronize();
      const auto t0 = std::chrono::steady_clock::now();
      for (size_t off = 0; off < nb && e == hipSuccess; off += piece) {
        const size_t len = std::min(piece, nb - off);
        if (dir & 1) e = hipMemcpyAsync(d_in + off, h_in + off, len, hipMemcpyHostToDevice, s_in);
        if ((dir & 2) && e == hipSuccess) e = hipMemcpyAsync(h_out + off, d_out + off, len, hipMemcpyDeviceToHost, s_out);
      }
      if (e == hipSuccess) e = hipDeviceSynchronize();
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      const double gbs = (dir == 3 ? 2.0 : 1.0) * (double)nb / s / 1e9;
      if (r >= 0 && gbs > best[dir - 1]) best[dir - 1] = gbs;
    }
  }
  if (s_in) (void)hipStreamDestroy(s_in);
  if (s_out) (void)hipStreamDestroy(s_out);
  if (d_in) (void)hipFree(d_in);
  if (d_out) (void)hipFree(d_out);
  if (h_in) (void)hipHostFree(h_in);
  if (h_out) (void)hipHostFree(h_out);
  if (e != hipSuccess) return hip_fail(e, "pcie copy measurement");
  // the HIP runtime's engine choice serialises the two directions now and then
  // (profiles/r04/pipeline_engines.txt): the same copies on the engine pair the
  // pipelines use, and per figure the better of the two
  double eh = 0.0, ed = 0.0, eb = 0.0;
  if (pcie_engine_gbps(device, nb, reps, &eh, &ed, &eb) == CLOUDSC_OK) {
    best[0] = std::max(best[0], eh);
    best[1] = std::max(best[1], ed);
    best[2] = std::max(best[2], eb);
  }
  *h2d = best[0];
  *d2h = best[1];
  *both = best[2];
  return CLOUDSC_OK;
}

// ---------------------------------------------------------------------------
// Counter calibration (round 5): MI355X_MICROARCH.md
// calibrates rocprofv3's FETCH_SIZE (x2) and WRITE_SIZE (x1) only for 16-byte
// per-lane streaming accesses.  The CLOUDSC kernels load and store 8 bytes
// (fp64) or 4 bytes (fp32) per lane, non-temporal, one 512 / 256-byte row per
// wave instruction.  This streams a known byte count with exactly that access
// shape -- a read of `bytes` (mode 0) or a write of `bytes` (mode 1), `width`
// bytes per lane, consecutive lanes on consecutive elements, a grid striding
// over the buffer -- so a PMC pass over it gives the counters' factor for the
// kernels' own widths (tools/calib_counters.py).
namespace {
template <typename T, bool WRITE>
__global__ void __launch_bounds__(256) stream_probe(T* __restrict__ a, size_t n, unsigned* __restrict__ sink) {
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, step = (size_t)gridDim.x * blockDim.x;
  if constexpr (WRITE) {
    for (size_t i = i0; i < n; i += step) {
      T v;
      if constexpr (sizeof(T) == 16) v = T{(unsigned)i, 0u, 0u, 0u};
      else v = (T)i;
      __builtin_nontemporal_store(v, a + i);
    }
  } else {
    T acc{};
    for (size_t i = i0; i < n; i += step) acc += __builtin_nontemporal_load(a + i);
    bool hit;
    if constexpr (sizeof(T) == 16) hit = acc.x == 1u;
    else hit = acc == (T)1;
    if (hit) sink[0] = 1;   // keeps the loads; never true for the zero-filled buffer
  }
}
}  // namespace

extern "C" int cloudsc_debug_stream_probe(int device, int mode, int width, long long bytes, int reps, double* ms) {
  if (!ms || (mode != 0 && mode != 1) || (width != 4 && width != 8 && width != 16) || bytes < (1 << 20) ||
      bytes % 16 || reps <= 0)
    return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(device));
  void* a = nullptr;
  unsigned* sink = nullptr;
  HIPCHK(hipMalloc(&a, (size_t)bytes));
  hipError_t e = hipMalloc((void**)&sink, 64);
  if (e == hipSuccess) e = hipMemset(a, 0, (size_t)bytes);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  double best = 0.0;
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  for (int r = 0; r < reps && e == hipSuccess; r++) {
    e = hipEventRecord(e0, nullptr);
    const dim3 g(2048), b(256);
    const size_t n = (size_t)bytes / width;
    if (e == hipSuccess) {
      if (width == 4) {
        if (mode) hipLaunchKernelGGL((stream_probe<float, true>), g, b, 0, nullptr, (float*)a, n, sink);
        else hipLaunchKernelGGL((stream_probe<float, false>), g, b, 0, nullptr, (float*)a, n, sink);
      } else if (width == 8) {
        if (mode) hipLaunchKernelGGL((stream_probe<double, true>), g, b, 0, nullptr, (double*)a, n, sink);
        else hipLaunchKernelGGL((stream_probe<double, false>), g, b, 0, nullptr, (double*)a, n, sink);
      } else {
        if (mode) hipLaunchKernelGGL((stream_probe<u32x4v, true>), g, b, 0, nullptr, (u32x4v*)a, n, sink);
        else hipLaunchKernelGGL((stream_probe<u32x4v, false>), g, b, 0, nullptr, (u32x4v*)a, n, sink);
      }
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(e1, nullptr);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    if (e == hipSuccess && (best == 0.0 || t < best)) best = t;
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(sink);
  (void)hipFree(a);
  if (e != hipSuccess) return hip_fail(e, "stream probe");
  *ms = best;
  return CLOUDSC_OK;
}
