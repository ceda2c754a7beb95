// tools/pcie_probe.hip -- the host<->device transfer ceiling of this box, the
// bound of the host-buffer pipeline (cloudsc_host_pipeline_*):
// one direction alone and both at once, by two engines:
//   sdma  hipMemcpyAsync on pinned host memory (the copy engines), S streams per
//         direction, the buffer cut into chunks issued round-robin;
//   blit  a copy kernel reading / writing the pinned host memory directly over
//         PCIe (nontemporal 16-byte accesses), G workgroups per direction.
// Both-direction runs issue the two directions on separate streams at once.
// One JSON line per configuration, then the best of each kind.
//   hipcc -O3 --offload-arch=gfx950 tools/pcie_probe.hip -o build/pcie_probe
//   build/pcie_probe [GiB per direction]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
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

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) blit(v4u* __restrict__ dst, const v4u* __restrict__ src, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

struct Bufs {
  char *h_in, *h_out, *d_in, *d_out;
  size_t bytes;
};

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// dir: 1 = H2D only, 2 = D2H only, 3 = both
double run_sdma(const Bufs& b, int dir, int nstreams, size_t chunk, std::vector<hipStream_t>& st) {
  CK(hipDeviceSynchronize());
  const double t0 = now();
  const size_t nchunks = (b.bytes + chunk - 1) / chunk;
  for (size_t c = 0; c < nchunks; c++) {
    const size_t off = c * chunk, len = std::min(chunk, b.bytes - off);
    if (dir & 1) CK(hipMemcpyAsync(b.d_in + off, b.h_in + off, len, hipMemcpyHostToDevice, st[c % nstreams]));
    if (dir & 2)
      CK(hipMemcpyAsync(b.h_out + off, b.d_out + off, len, hipMemcpyDeviceToHost, st[nstreams + c % nstreams]));
  }
  CK(hipDeviceSynchronize());
  return now() - t0;
}

double run_blit(const Bufs& b, int dir, int grid, std::vector<hipStream_t>& st) {
  CK(hipDeviceSynchronize());
  const double t0 = now();
  const size_t n = b.bytes / sizeof(v4u);
  if (dir & 1) hipLaunchKernelGGL(blit, dim3(grid), dim3(256), 0, st[0], (v4u*)b.d_in, (const v4u*)b.h_in, n);
  if (dir & 2) hipLaunchKernelGGL(blit, dim3(grid), dim3(256), 0, st[1], (v4u*)b.h_out, (const v4u*)b.d_out, n);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return now() - t0;
}

// both directions at once, one by the copy engine and one by a blit kernel
// (h2d_blit: H2D blit + D2H sdma; else H2D sdma + D2H blit), 64 MiB copies
double run_mixed(const Bufs& b, bool h2d_blit, int grid, std::vector<hipStream_t>& st) {
  CK(hipDeviceSynchronize());
  const double t0 = now();
  const size_t n = b.bytes / sizeof(v4u), piece = (size_t)64 << 20;
  if (h2d_blit) {
    hipLaunchKernelGGL(blit, dim3(grid), dim3(256), 0, st[0], (v4u*)b.d_in, (const v4u*)b.h_in, n);
    for (size_t off = 0; off < b.bytes; off += piece)
      CK(hipMemcpyAsync(b.h_out + off, b.d_out + off, std::min(piece, b.bytes - off), hipMemcpyDeviceToHost, st[1]));
  } else {
    for (size_t off = 0; off < b.bytes; off += piece)
      CK(hipMemcpyAsync(b.d_in + off, b.h_in + off, std::min(piece, b.bytes - off), hipMemcpyHostToDevice, st[0]));
    hipLaunchKernelGGL(blit, dim3(grid), dim3(256), 0, st[1], (v4u*)b.h_out, (const v4u*)b.d_out, n);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return now() - t0;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 2.0;
  Bufs b;
  b.bytes = (size_t)(gib * (1u << 30));
  CK(hipHostMalloc((void**)&b.h_in, b.bytes, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&b.h_out, b.bytes, hipHostMallocDefault));
  CK(hipMalloc((void**)&b.d_in, b.bytes));
  CK(hipMalloc((void**)&b.d_out, b.bytes));
  CK(hipMemset(b.d_out, 1, b.bytes));
  for (size_t i = 0; i < b.bytes; i += 4096) b.h_in[i] = (char)i;
  std::vector<hipStream_t> st(16);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char* dname[] = {"", "h2d", "d2h", "both"};
  double best[2][4] = {};
  for (int dir = 1; dir <= 3; dir++) {
    for (int ns : {1, 2, 4, 8}) {
      for (size_t chunk : {(size_t)8 << 20, (size_t)64 << 20, b.bytes}) {
        if (chunk == b.bytes && ns > 1) continue;
        run_sdma(b, dir, ns, chunk, st);   // warm
        double t = 1e30;
        for (int r = 0; r < 3; r++) t = std::min(t, run_sdma(b, dir, ns, chunk, st));
        const double gbs = (dir == 3 ? 2.0 : 1.0) * b.bytes / t / 1e9;
        best[0][dir] = std::max(best[0][dir], gbs);
        std::printf("{\"engine\": \"sdma\", \"dir\": \"%s\", \"streams_per_dir\": %d, \"chunk_MiB\": %zu, \"GBs_total\": %.1f}\n",
                    dname[dir], ns, chunk >> 20, gbs);
        std::fflush(stdout);
      }
    }
    for (int grid : {64, 256, 1024}) {
      run_blit(b, dir, grid, st);
      double t = 1e30;
      for (int r = 0; r < 3; r++) t = std::min(t, run_blit(b, dir, grid, st));
      const double gbs = (dir == 3 ? 2.0 : 1.0) * b.bytes / t / 1e9;
      best[1][dir] = std::max(best[1][dir], gbs);
      std::printf("{\"engine\": \"blit\", \"dir\": \"%s\", \"workgroups_per_dir\": %d, \"GBs_total\": %.1f}\n", dname[dir],
                  grid, gbs);
      std::fflush(stdout);
    }
  }
  // repeatability of the both-direction forms: 10 runs each, every time printed
  for (int mode = 0; mode < 3; mode++) {
    std::printf("{\"repeat\": \"%s\", \"GBs_total\": [", mode == 0 ? "sdma+sdma" : mode == 1 ? "sdma_h2d+blit_d2h" : "blit_h2d+sdma_d2h");
    for (int r = 0; r < 10; r++) {
      const double t = mode == 0 ? run_sdma(b, 3, 1, (size_t)64 << 20, st) : run_mixed(b, mode == 2, 256, st);
      std::printf("%s%.1f", r ? ", " : "", 2.0 * b.bytes / t / 1e9);
    }
    std::printf("]}\n");
    std::fflush(stdout);
  }
  std::printf("{\"summary\": true, \"bytes_each_direction\": %zu, \"sdma_h2d\": %.1f, \"sdma_d2h\": %.1f, "
              "\"sdma_both_total\": %.1f, \"blit_h2d\": %.1f, \"blit_d2h\": %.1f, \"blit_both_total\": %.1f}\n",
              b.bytes, best[0][1], best[0][2], best[0][3], best[1][1], best[1][2], best[1][3]);
  return 0;
}
