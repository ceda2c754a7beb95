// tools/contig_alloc_probe.hip -- diagnostic, no CLOUDSC code: do device
// allocations made after hipDeviceMallocContiguous allocations were freed hold
// what is written to them?
//
// A "state" is the allocation pattern of one cloudsc_state_create at NGPTOT
// columns, NPROMA 64, KLEV 137 (28 input fields, 21 outputs, a KSEG workspace;
// level / half-level / species / surface sizes, element size 8 or 4): every
// field is allocated (hipMalloc, or hipExtMallocWithFlags(hipDeviceMallocContiguous)),
// filled the way the state fills it -- inputs from a small template (the
// 100-column reference state's size) copied into a temporary hipMalloc'd buffer
// from pageable memory and expanded by a kernel, the temporary freed; outputs by
// hipMemsetAsync -- all on one non-blocking stream, then
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
// the state's expansion: dst[e] = src[(e / period) * klon + (e % period) % klon] for a small
// template src of nrow x klon words (period = nproma columns; g % klon with no block offset
// is enough to place every word)
__global__ void expand_words(unsigned* dst, const unsigned* src, size_t n, int nproma, int klon, int nrow) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t row = (e / nproma) % nrow, col = (e / ((size_t)nproma * nrow) * nproma + e % nproma) % klon;
    dst[e] = src[row * klon + col];
  }
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
      // inputs as the state expands them: a small template (nrow x 100 columns,
      // 110-550 KB like the reference's 100-column state) copied in from pageable
      // memory to a temporary, expanded by a kernel, the temporary freed
      const int klon = 100;
      std::vector<std::vector<unsigned>> tmpl(in_sz.size());
      std::vector<int> nrow(in_sz.size());
      for (size_t f = 0; f < in_sz.size(); f++) {
        in[f] = dalloc(in_sz[f]);
        nrow[f] = (int)(in_sz[f] / ((size_t)nb * nproma));
        tmpl[f].resize((size_t)nrow[f] * klon);
        for (size_t i = 0; i < tmpl[f].size(); i++) tmpl[f][i] = pattern((int)f, i, salt);
        unsigned* tmp = nullptr;
        CK(hipMalloc((void**)&tmp, tmpl[f].size() * 4));
        CK(hipMemcpyAsync(tmp, tmpl[f].data(), tmpl[f].size() * 4, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(expand_words, dim3(1024), dim3(256), 0, st, in[f], tmp, in_sz[f], nproma, klon, nrow[f]);
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
        for (size_t e = 0; e < h.size(); e++) {
          const size_t row = (e / nproma) % nrow[f], col = (e / ((size_t)nproma * nrow[f]) * nproma + e % nproma) % klon;
          bad += h[e] != tmpl[f][row * klon + col];
        }
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
