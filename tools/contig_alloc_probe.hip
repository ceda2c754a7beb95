// tools/contig_alloc_probe.hip -- diagnostic, no CLOUDSC code: do device
// allocations made after hipDeviceMallocContiguous allocations were freed hold
// what is written to them?
//
// A "state" is the allocation pattern of one cloudsc_state_create at NGPTOT
// columns, NPROMA 64, KLEV 137 (28 input fields, 21 outputs, a KSEG workspace;
// level / half-level / species / surface sizes, element size 8 or 4): every
// field is allocated (hipMalloc, or hipExtMallocWithFlags(hipDeviceMallocContiguous)),
// filled the way the state fills it -- inputs through a temporary hipMalloc'd
// staging buffer (H2D copy from pageable memory, a copy kernel, hipFree of the
// temporary), outputs by hipMemsetAsync -- all on one non-blocking stream, then
// EVERY field is read back and checked (a field whose pages alias another's
// shows the other's pattern), then everything is freed.  The sequence of states
// is the one of profiles/r04/contiguous_alloc_hazard_repro.py --fp64-first:
// P = plain, C = contiguous, fp64 sizes then fp32 sizes.
//   hipcc -O2 --offload-arch=gfx950 tools/contig_alloc_probe.hip -o build/contig_alloc_probe
//   build/contig_alloc_probe [ngptot]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(2);                                                                                \
    }                                                                                              \
  } while (0)

__global__ void copy_words(unsigned* dst, const unsigned* src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static unsigned pattern(int field, size_t i, unsigned salt) { return (unsigned)(i * 2654435761u) ^ (field * 0x9e3779b9u) ^ salt; }

int main(int argc, char** argv) {
  const long ngptot = argc > 1 ? atol(argv[1]) : 3000;
  const int nproma = 64, klev = 137;
  const long nb = (ngptot + nproma - 1) / nproma;
  const char* seq = "PPPPPCPPCPP";           // the repro's layouts: arena layouts counted as plain
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  long long total_bad = 0;
  for (int es : {8, 4}) {
    // 23 level inputs (incl. aerosol-free set + plude), 1 half-level, 2 species, 2 surface;
    // 18 level/half outputs etc.: sizes in words of 4 bytes
    const size_t lev = nb * klev * nproma * es / 4, half = nb * (klev + 1) * nproma * es / 4;
    const size_t spec = 5 * lev, surf = nb * nproma * es / 4;
    std::vector<size_t> in_sz, out_sz;
    for (int i = 0; i < 19; i++) in_sz.push_back(lev);
    in_sz.push_back(half); in_sz.push_back(spec); in_sz.push_back(spec); in_sz.push_back(surf);
    in_sz.push_back(nb * nproma);   // ktype
    for (int i = 0; i < 5; i++) out_sz.push_back(lev);
    out_sz.push_back(spec); out_sz.push_back(surf);
    for (int i = 0; i < 14; i++) out_sz.push_back(half);
    const size_t ws = 64 + nb + nb * 19 * nproma * es / 4;
    for (int r = 0; seq[r]; r++) {
      const bool contig = seq[r] == 'C';
      const unsigned salt = 0x51ed270bu * (unsigned)(r + 17 * es);
      auto dalloc = [&](size_t words) {
        void* p = nullptr;
        if (contig) CK(hipExtMallocWithFlags(&p, words * 4, hipDeviceMallocContiguous));
        else CK(hipMalloc(&p, words * 4));
        return (unsigned*)p;
      };
      std::vector<unsigned*> in(in_sz.size()), out(out_sz.size());
      std::vector<unsigned> h;
      for (size_t f = 0; f < in_sz.size(); f++) {
        in[f] = dalloc(in_sz[f]);
        h.resize(in_sz[f]);
        for (size_t i = 0; i < h.size(); i++) h[i] = pattern((int)f, i, salt);
        unsigned* tmp = nullptr;
        CK(hipMalloc((void**)&tmp, in_sz[f] * 4));
        CK(hipMemcpyAsync(tmp, h.data(), in_sz[f] * 4, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(copy_words, dim3(1024), dim3(256), 0, st, in[f], tmp, in_sz[f]);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        CK(hipFree(tmp));
      }
      for (size_t f = 0; f < out_sz.size(); f++) {
        out[f] = dalloc(out_sz[f]);
        CK(hipMemsetAsync(out[f], 0xff, out_sz[f] * 4, st));
      }
      unsigned* w = dalloc(ws);
      CK(hipMemsetAsync(w, 0, ws * 4, st));
      CK(hipStreamSynchronize(st));
      long long bad = 0;
      for (size_t f = 0; f < in_sz.size(); f++) {
        h.resize(in_sz[f]);
        CK(hipMemcpy(h.data(), in[f], in_sz[f] * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h.size(); i++) bad += h[i] != pattern((int)f, i, salt);
      }
      for (size_t f = 0; f < out_sz.size(); f++) {
        h.resize(out_sz[f]);
        CK(hipMemcpy(h.data(), out[f], out_sz[f] * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h.size(); i++) bad += h[i] != 0xffffffffu;
      }
      std::printf("fp%d state %2d %s: %lld wrong words\n", 8 * es, r, contig ? "contiguous" : "plain     ", bad);
      std::fflush(stdout);
      total_bad += bad;
      for (unsigned* p : in) CK(hipFree(p));
      for (unsigned* p : out) CK(hipFree(p));
      CK(hipFree(w));
    }
  }
  std::printf("RESULT: %lld wrong words\n", total_bad);
  CK(hipStreamDestroy(st));
  return total_bad ? 1 : 0;
}
