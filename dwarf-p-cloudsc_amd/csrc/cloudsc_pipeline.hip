// cloudsc_pipeline.hip -- the host-buffer pipeline of include/cloudsc_amd.h
// (cloudsc_host_pipeline_*).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include <sys/mman.h>
#include <unistd.h>

#include "cloudsc_amd.h"
#include "cloudsc_internal.h"

using namespace cloudsc_impl;

// ---------------------------------------------------------------------------
// C ABI: host-buffer pipeline
// ---------------------------------------------------------------------------
// The reference GPU drivers copy every block-layout host array to the device,
// run, and copy the outputs back (cloudsc_driver.cu:344-456; the "field"
// variant of README.md:311-330 overlaps them).  Here the blocks are cut into
// chunks of `chunk_blocks` NPROMA blocks -- one contiguous range of every
// field, because the layout is block-major -- and chunk c uses device buffer
// slot c % nslots.  Three streams form the pipeline (round 4): one carries every
// host-to-device copy, one every kernel, one every device-to-host copy, ordered
// per slot by events -- the inputs of chunk c go in while chunk c-1 computes and
// chunk c-2's outputs come out.  One stream per direction is what the copy
// engines run fastest: 97 GB/s both directions together with one stream each,
// 65-85 GB/s with 2-8 streams per direction (tools/pcie_probe.hip,
// profiles/r04/pcie_probe.jsonl; round 3 ran H2D, kernel and D2H of a chunk on
// one of 4 streams: 74 GB/s).  The host arrays are pinned in place
// (hipHostRegister) once, at creation.
//
// Pinning is by whole pages, and arrays from a general-purpose allocator share
// pages (the end of one field and the start of the next).  Registering each
// array on its own then makes two registrations of one page; a copy of the
// second array can be resolved against the first registration and run off its
// end (a device page fault, seen in round 2 as "illegal memory access" in a
// chunked SCC pipeline after other pipelines had come and gone).  So the page
// ranges of all fields are merged first and every merged range is registered
// once: each array lies wholly inside exactly one registration.
// (The field table, kFieldTable, is in cloudsc_internal.h.)

// D2H of one chunk by a copy kernel instead of the copy engine (diagnostic
// mode 2 of cloudsc_debug_set_pipeline_copy): every output field's chunk range,
// device buffer -> pinned host memory through its device-visible address, in
// one launch.  16-byte accesses where both ends are 16-byte aligned, else 4 B.
constexpr int kMaxBlitSeg = 24;
struct BlitSegs {
  const char* src[kMaxBlitSeg];
  char* dst[kMaxBlitSeg];
  unsigned long long bytes[kMaxBlitSeg];
  int n;
};
__global__ void __launch_bounds__(256) d2h_blit_kernel(const BlitSegs s) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
  for (int q = 0; q < s.n; q++) {
    const char* src = s.src[q];
    char* dst = s.dst[q];
    const size_t nb = s.bytes[q];
    if ((((uintptr_t)src | (uintptr_t)dst | nb) & 15) == 0) {
      const u4* a = (const u4*)src;
      u4* b = (u4*)dst;
      for (size_t i = tid; i < nb / 16; i += nth) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
    } else {
      const unsigned* a = (const unsigned*)src;
      unsigned* b = (unsigned*)dst;
      for (size_t i = tid; i < nb / 4; i += nth) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
    }
  }
}
// how the pipeline moves data (cloudsc_debug_set_pipeline_copy): 1 (default)
// copy engines chosen explicitly through HSA, one per direction; 0 HIP streams
// (the runtime picks the engines); 2 HIP streams with the outputs written back
// by a copy kernel instead of a copy engine
enum PipeCopy { PC_HIP = 0, PC_ENGINES = 1, PC_HIP_BLIT = 2 };
std::atomic<int> g_pipe_copy{PC_ENGINES};

// ---------------------------------------------------------------------------
// Copy engines per direction (round 4).  Through hipMemcpyAsync the runtime
// picks an SDMA engine per stream from the engines free at the moment it asks
// (the recommended ones first: engine 0 for host->device, 1-2 for
// device->host on MI355X).  When the host->device stream asks while engine 0 is
// busy it lands on engine 1 -- the device->host stream's engine -- and the two
// directions run one after the other: steps of 177-343 ms instead of 104 for
// the same work, in runs of several steps (a copy trace shows zero overlap of
// the two directions in the slow steps; profiles/r04/pipeline_engines.txt).  So
// the pipeline issues its copies itself, with hsa_amd_memory_async_copy_on_engine,
// H2D and D2H each on its own engine chosen once at creation, and orders them
// with the kernels from the host: chunk c's inputs go in when the kernel of
// chunk c - nslots has finished with the slot, chunk c-1's outputs go out as
// soon as its kernel has finished, and chunk c's kernel starts once its inputs
// are in and chunk c - nslots's outputs are out.  The copies of one direction
// queue back to back on their engine, so the host's reaction time only adds
// at the ends of the pipeline.
struct HsaEngines {
  bool ok = false;
  hsa_agent_t cpu{}, gpu{};
  hsa_amd_sdma_engine_id_t h2d{}, d2h{};
  uint32_t rec_in = 0, rec_out = 0;    // the runtime's recommended engine masks per direction
  double overlap = 0.0;                // both-at-once time / the slower direction alone (1 = full overlap)
  int pairs_tried = 0;
};

struct AgentSearch {
  uint32_t bdfid, domain;
  hsa_agent_t cpu{}, gpu{};
  bool have_cpu = false, have_gpu = false;
};

hsa_status_t agent_cb(hsa_agent_t a, void* data) {
  auto* q = (AgentSearch*)data;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !q->have_cpu) { q->cpu = a; q->have_cpu = true; }
  if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
        bdf == q->bdfid && dom == q->domain) {
      q->gpu = a;
      q->have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

// the lowest engine of `mask` other than `not_this` (0 when none)
uint32_t pick_engine(uint32_t mask, uint32_t not_this) {
  for (uint32_t b = 1; b && b <= mask; b <<= 1)
    if ((mask & b) && b != not_this) return b;
  return 0;
}

HsaEngines find_engines(int device) {
  HsaEngines e;
  static std::once_flag once;
  static bool hsa_up = false;
  std::call_once(once, [] { hsa_up = hsa_init() == HSA_STATUS_SUCCESS; });   // HIP's runtime: a reference
  if (!hsa_up) return e;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return e;
  AgentSearch q;
  q.bdfid = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
  q.domain = (uint32_t)prop.pciDomainID;
  if (hsa_iterate_agents(agent_cb, &q) != HSA_STATUS_SUCCESS || !q.have_cpu || !q.have_gpu) return e;
  uint32_t rec_in = 0, rec_out = 0;
  if (hsa_amd_memory_get_preferred_copy_engine(q.gpu, q.cpu, &rec_in) != HSA_STATUS_SUCCESS) rec_in = 0;
  if (hsa_amd_memory_get_preferred_copy_engine(q.cpu, q.gpu, &rec_out) != HSA_STATUS_SUCCESS) rec_out = 0;
  uint32_t in = pick_engine(rec_in ? rec_in : 0x1, 0);
  uint32_t out = pick_engine(rec_out ? rec_out : 0x6, in);
  if (!out) out = pick_engine(0xffff, in);
  if (!in || !out) return e;
  e.rec_in = rec_in; e.rec_out = rec_out;
  e.cpu = q.cpu; e.gpu = q.gpu;
  e.h2d = (hsa_amd_sdma_engine_id_t)in;
  e.d2h = (hsa_amd_sdma_engine_id_t)out;
  e.ok = true;
  return e;
}

// Engine pair check at creation.  One diagnostic run of the engine path ran
// every step with the two directions serialised (174 ms instead of 103 ms per
// step, the same engine ids; profiles/r04/pipeline_steps_r04.jsonl), so the
// pair is measured before it is used: 256 MiB H2D alone, D2H alone, then both
// at once; overlap = both / the slower alone (1.0 when the directions run
// fully concurrently, 2.0 when serialised).  Pairs from the recommended masks
// first, then the other engines; the first pair below 1.3 is taken, else the
// best one seen (at most kMaxPairs).
constexpr int kMaxPairs = 6;
double time_pair(const HsaEngines& e, hsa_amd_sdma_engine_id_t ein, hsa_amd_sdma_engine_id_t eout, char* h_in,
                 char* h_out, char* d_in, char* d_out, size_t nb, hsa_signal_t sg, int dirs) {
  const size_t piece = (size_t)64 << 20;
  int n = 0;
  for (size_t off = 0; off < nb; off += piece) n += ((dirs & 1) ? 1 : 0) + ((dirs & 2) ? 1 : 0);
  hsa_signal_store_screlease(sg, n);
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t off = 0; off < nb; off += piece) {
    const size_t len = std::min(piece, nb - off);
    if ((dirs & 1) && hsa_amd_memory_async_copy_on_engine(d_in + off, e.gpu, h_in + off, e.cpu, len, 0, nullptr, sg,
                                                          ein, true) != HSA_STATUS_SUCCESS) {
      hsa_signal_subtract_screlease(sg, 1);
      return -1.0;
    }
    if ((dirs & 2) && hsa_amd_memory_async_copy_on_engine(h_out + off, e.cpu, d_out + off, e.gpu, len, 0, nullptr, sg,
                                                          eout, true) != HSA_STATUS_SUCCESS) {
      hsa_signal_subtract_screlease(sg, 1);
      return -1.0;
    }
  }
  if (hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) != 0) return -1.0;
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void check_engines(HsaEngines& e) {
  const size_t nb = (size_t)256 << 20;
  char *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  hsa_signal_t sg{};
  bool have_sg = false;
  if (hipHostMalloc((void**)&h_in, nb, hipHostMallocDefault) == hipSuccess &&
      hipHostMalloc((void**)&h_out, nb, hipHostMallocDefault) == hipSuccess &&
      hipMalloc((void**)&d_in, nb) == hipSuccess && hipMalloc((void**)&d_out, nb) == hipSuccess &&
      hipMemset(d_out, 1, nb) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
      hsa_signal_create(0, 0, nullptr, &sg) == HSA_STATUS_SUCCESS) {
    have_sg = true;
    std::memset(h_in, 2, nb);
    // candidate pairs: recommended engines first, then every other engine bit
    std::vector<std::pair<uint32_t, uint32_t>> pairs;
    const uint32_t rin = e.rec_in ? e.rec_in : 0x1, rout = e.rec_out ? e.rec_out : 0x6;
    pairs.push_back({(uint32_t)e.h2d, (uint32_t)e.d2h});
    for (uint32_t a = 1; a && a <= 0x8000; a <<= 1)
      for (uint32_t b = 1; b && b <= 0x8000; b <<= 1) {
        if (a == b) continue;
        const int rank = ((rin & a) ? 0 : 1) + ((rout & b) ? 0 : 1);
        if (rank == 0 && !(a == (uint32_t)e.h2d && b == (uint32_t)e.d2h)) pairs.push_back({a, b});
      }
    for (uint32_t b = 1; b && b <= 0x8000; b <<= 1)
      if (b != (uint32_t)e.h2d && !(rout & b)) pairs.push_back({(uint32_t)e.h2d, b});
    double best = 1e30;
    std::pair<uint32_t, uint32_t> pick{(uint32_t)e.h2d, (uint32_t)e.d2h};
    for (size_t i = 0; i < pairs.size() && e.pairs_tried < kMaxPairs; i++) {
      const auto ein = (hsa_amd_sdma_engine_id_t)pairs[i].first, eout = (hsa_amd_sdma_engine_id_t)pairs[i].second;
      if (time_pair(e, ein, eout, h_in, h_out, d_in, d_out, nb, sg, 3) < 0.0) continue;   // warm-up / unusable pair
      const double ti = time_pair(e, ein, eout, h_in, h_out, d_in, d_out, nb, sg, 1);
      const double to = time_pair(e, ein, eout, h_in, h_out, d_in, d_out, nb, sg, 2);
      const double tb = time_pair(e, ein, eout, h_in, h_out, d_in, d_out, nb, sg, 3);
      e.pairs_tried++;
      if (ti <= 0.0 || to <= 0.0 || tb <= 0.0) continue;
      const double r = tb / std::max(ti, to);
      if (r < best) { best = r; pick = pairs[i]; }
      if (r < 1.3) break;
    }
    if (best < 1e30) {
      e.h2d = (hsa_amd_sdma_engine_id_t)pick.first;
      e.d2h = (hsa_amd_sdma_engine_id_t)pick.second;
      e.overlap = best;
    }
  }
  if (have_sg) hsa_signal_destroy(sg);
  if (d_in) (void)hipFree(d_in);
  if (d_out) (void)hipFree(d_out);
  if (h_in) (void)hipHostFree(h_in);
  if (h_out) (void)hipHostFree(h_out);
  (void)hipGetLastError();
}

// The copy ceiling on the engine pair the pipelines use (cloudsc_pcie_gbps
// takes the better of this and its HIP-stream figures): H2D alone, D2H alone
// and both at once of `nb` bytes each way, best of `reps`; 0 when the engines
// are not available.
int cloudsc_impl::pcie_engine_gbps(int device, size_t nb, int reps, double* h2d, double* d2h, double* both) {
  *h2d = *d2h = *both = 0.0;
  HsaEngines e = find_engines(device);
  if (!e.ok) return CLOUDSC_OK;
  check_engines(e);
  char *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  hsa_signal_t sg{};
  bool have_sg = false;
  int rc = CLOUDSC_OK;
  if (hipHostMalloc((void**)&h_in, nb, hipHostMallocDefault) == hipSuccess &&
      hipHostMalloc((void**)&h_out, nb, hipHostMallocDefault) == hipSuccess &&
      hipMalloc((void**)&d_in, nb) == hipSuccess && hipMalloc((void**)&d_out, nb) == hipSuccess &&
      hipMemset(d_out, 1, nb) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
      hsa_signal_create(0, 0, nullptr, &sg) == HSA_STATUS_SUCCESS) {
    have_sg = true;
    std::memset(h_in, 2, nb);
    double* out[3] = {h2d, d2h, both};
    for (int dirs = 1; dirs <= 3; dirs++)
      for (int r = -1; r < reps; r++) {
        const double ms = time_pair(e, e.h2d, e.d2h, h_in, h_out, d_in, d_out, nb, sg, dirs);
        if (ms <= 0.0) { rc = CLOUDSC_EHIP; break; }
        const double gbs = (dirs == 3 ? 2.0 : 1.0) * (double)nb / (ms * 1e-3) / 1e9;
        if (r >= 0 && gbs > *out[dirs - 1]) *out[dirs - 1] = gbs;
      }
  } else {
    rc = CLOUDSC_ENOMEM;
  }
  if (have_sg) hsa_signal_destroy(sg);
  if (d_in) (void)hipFree(d_in);
  if (d_out) (void)hipFree(d_out);
  if (h_in) (void)hipHostFree(h_in);
  if (h_out) (void)hipHostFree(h_out);
  (void)hipGetLastError();
  return rc;
}

struct cloudsc_host_pipeline {
  int device, precision, ngptot, nproma, klev, nblocks, chunk_blocks, nstreams;   // nstreams: device slots
  size_t es;
  cloudsc_fields_t host;
  std::vector<void*> pinned;
  struct Slot {
    cloudsc_fields_t dev{};
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    int scratch_variant = 0;
    hipEvent_t in_done = nullptr, k_done = nullptr, out_done = nullptr;   // the slot's last chunk, per stage
  };
  std::vector<Slot> slots;
  hipStream_t st_in = nullptr, st_k = nullptr, st_out = nullptr;
  void* host_dev[kNumFields] = {};   // agent (device-visible) addresses of the pinned host arrays
  HsaEngines eng;                    // copy engines per direction (PC_ENGINES)
  std::vector<hsa_signal_t> sig_in, sig_out;   // per slot: its chunk's copies still running
  std::vector<void*> allocs;
  ParamSet params;          // snapshot of the device's default set at creation
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace {

size_t field_bytes(const cloudsc_host_pipeline* p, int i, int nblocks) {
  const FieldDesc& d = kFieldTable[i];
  return (size_t)nblocks * per_block_elems(d.kind, p->nproma, p->klev) * (d.is_int ? sizeof(int) : p->es);
}

// [ptr, ptr+bytes) is host memory the device can reach as ONE mapping: both ends
// resolve to pinned host memory at device addresses exactly bytes-1 apart
bool pinned_as_one(const void* ptr, size_t bytes) {
  hipPointerAttribute_t a, b;
  if (hipPointerGetAttributes(&a, ptr) != hipSuccess ||
      hipPointerGetAttributes(&b, (const char*)ptr + bytes - 1) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost && b.type == hipMemoryTypeHost && a.devicePointer && b.devicePointer &&
         (const char*)b.devicePointer - (const char*)a.devicePointer == (ptrdiff_t)(bytes - 1);
}

// Pin the caller's arrays in place: the page ranges of all fields merged into
// disjoint ranges, each registered once (see the note at the top).  A range the
// caller has pinned already (hipHostMalloc, or its own hipHostRegister) is used
// as it is if every field in it is covered by one mapping; otherwise the
// pipeline refuses the arrays rather than risk a partial mapping.
int pin_host_fields(cloudsc_host_pipeline* p, void* const* hf) {
  const long sys_pg = sysconf(_SC_PAGESIZE);
  const uintptr_t pg = sys_pg > 0 ? (uintptr_t)sys_pg : 4096;
  struct Span { uintptr_t lo, hi; };
  std::vector<Span> spans;
  for (int i = 0; i < kNumFields; i++) {
    if (!hf[i]) continue;
    const uintptr_t a = (uintptr_t)hf[i], e = a + field_bytes(p, i, p->nblocks);
    spans.push_back({a & ~(pg - 1), (e + pg - 1) & ~(pg - 1)});
  }
  std::sort(spans.begin(), spans.end(), [](const Span& x, const Span& y) { return x.lo < y.lo; });
  std::vector<Span> merged;
  for (const Span& s : spans) {
    if (!merged.empty() && s.lo <= merged.back().hi) merged.back().hi = std::max(merged.back().hi, s.hi);
    else merged.push_back(s);
  }
  for (const Span& s : merged) {
    const hipError_t e = hipHostRegister((void*)s.lo, s.hi - s.lo, hipHostRegisterDefault);
    if (e == hipSuccess) { p->pinned.push_back((void*)s.lo); continue; }
    (void)hipGetLastError();
    // memory pinned by the caller: hipHostRegister reports it as already
    // registered, or (hipHostMalloc memory, ROCm 7) as an invalid argument
    bool all_pinned = true, any_pinned = false;
    for (int i = 0; i < kNumFields; i++) {
      const uintptr_t a = (uintptr_t)hf[i];
      if (!hf[i] || a < s.lo || a >= s.hi) continue;
      const bool one = pinned_as_one(hf[i], field_bytes(p, i, p->nblocks));
      all_pinned = all_pinned && one;
      any_pinned = any_pinned || one;
    }
    if (all_pinned) continue;
    if (e != hipErrorHostMemoryAlreadyRegistered && !any_pinned) return hip_fail(e, "hipHostRegister");
    set_error_text("host pipeline: an array lies partly in memory pinned by the caller; pin all or none");
    return CLOUDSC_EINVAL;
  }
  return CLOUDSC_OK;
}

// one step with every copy on the engines of p->eng (HsaEngines above); the
// host orders copies and kernels
int run_on_engines(cloudsc_host_pipeline* p, int variant, int vk, double* ms) {
  const int nchunks = (p->nblocks + p->chunk_blocks - 1) / p->chunk_blocks;
  const int nslots = (int)p->slots.size();
  const void* const* hf = (const void* const*)&p->host;
  HIPCHK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  // the copies of chunk c in one direction, counted down on the slot's signal.
  // H2D is issued in two parts: part 0 sets the count for every H2D copy of
  // the chunk and issues the pure inputs, part 1 issues the INOUT field
  // (plude), which the slot's previous D2H still reads (the caller
  // waits for that D2H between the two parts).  D2H is one part.
  auto issue = [&](int c, bool in, int part) -> int {
    auto& s = p->slots[c % nslots];
    hsa_signal_t sg = in ? p->sig_in[c % nslots] : p->sig_out[c % nslots];
    const int b0 = c * p->chunk_blocks;
    const int nb = (b0 + p->chunk_blocks <= p->nblocks) ? p->chunk_blocks : p->nblocks - b0;
    void* const* df = (void* const*)&s.dev;
    auto selected = [&](int dir, int pt) {
      if (!in) return dir == FD_OUT || dir == FD_INOUT;
      return dir != FD_OUT && (pt < 0 || (pt == 0) == (dir != FD_INOUT));
    };
    int n = 0;                 // copies of this call not yet issued
    for (int i = 0; i < kNumFields; i++)
      if (hf[i] && selected(kFieldTable[i].dir, part)) n++;
    int later = 0;             // part 1's copies, counted by part 0
    if (part <= 0) {
      int total = 0;
      for (int i = 0; i < kNumFields; i++)
        if (hf[i] && selected(kFieldTable[i].dir, -1)) total++;
      later = total - n;
      hsa_signal_store_screlease(sg, total);
    }
    for (int i = 0; i < kNumFields; i++) {
      const FieldDesc& d = kFieldTable[i];
      if (!hf[i] || !selected(d.dir, part)) continue;
      const size_t per = per_block_elems(d.kind, p->nproma, p->klev) * (d.is_int ? sizeof(int) : p->es);
      char* h = (char*)p->host_dev[i] + (size_t)b0 * per;
      const hsa_status_t st =
          in ? hsa_amd_memory_async_copy_on_engine(df[i], p->eng.gpu, h, p->eng.cpu, (size_t)nb * per, 0, nullptr, sg,
                                                   p->eng.h2d, true)
             : hsa_amd_memory_async_copy_on_engine(h, p->eng.cpu, df[i], p->eng.gpu, (size_t)nb * per, 0, nullptr, sg,
                                                   p->eng.d2h, true);
      if (st != HSA_STATUS_SUCCESS) {
        hsa_signal_subtract_screlease(sg, n + later);   // the copies not issued (the issued ones still count down)
        set_error_text("host pipeline: hsa_amd_memory_async_copy_on_engine failed");
        return CLOUDSC_EHIP;
      }
      n--;
    }
    return CLOUDSC_OK;
  };
  // 0 when every copy counted on sg is done; < 0 when one failed
  auto wait = [](hsa_signal_t sg) {
    return hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) == 0
               ? CLOUDSC_OK : CLOUDSC_EHIP;
  };
  int rc = CLOUDSC_OK;
  int out_issued = -1;                     // the last chunk whose D2H is issued
  // a chunk's outputs (and plude), once its kernel is done
  auto drain = [&](int c) -> int {
    if (hipEventSynchronize(p->slots[c % nslots].k_done) != hipSuccess) return CLOUDSC_EHIP;
    out_issued = c;
    return issue(c, false, 0);
  };
  for (int c = 0; c < nchunks && rc == CLOUDSC_OK; c++) {
    auto& s = p->slots[c % nslots];
    const bool reuse = c >= nslots;        // the slot held chunk c - nslots
    // inputs: after the slot's previous kernel has read its inputs
    if (reuse && hipEventSynchronize(s.k_done) != hipSuccess) { rc = CLOUDSC_EHIP; break; }
    if ((rc = issue(c, true, 0))) break;
    // plude: after the slot's previous D2H has read it back (with one slot
    // that D2H is the previous chunk's, not issued yet)
    if (reuse) {
      if (out_issued < c - nslots) rc = drain(c - nslots);
      if (!rc) rc = wait(p->sig_out[c % nslots]);
      if (rc) {
        // part 1 is never issued: take its copies off the count part 0 set,
        // or the final wait below would never see the signal reach zero
        int n1 = 0;
        for (int i = 0; i < kNumFields; i++)
          if (hf[i] && kFieldTable[i].dir == FD_INOUT) n1++;
        hsa_signal_subtract_screlease(p->sig_in[c % nslots], n1);
        break;
      }
    }
    if ((rc = issue(c, true, 1))) break;
    // the previous chunk's outputs, as soon as its kernel is done
    if (c >= 1 && out_issued < c - 1 && (rc = drain(c - 1))) break;
    // kernel: after its inputs are in and the slot's previous outputs are out
    if ((rc = wait(p->sig_in[c % nslots]))) break;
    const int b0 = c * p->chunk_blocks;
    const int nb = (b0 + p->chunk_blocks <= p->nblocks) ? p->chunk_blocks : p->nblocks - b0;
    const long long col0 = (long long)b0 * p->nproma;
    const int ncols = (int)((col0 + (long long)nb * p->nproma <= p->ngptot) ? (long long)nb * p->nproma
                                                                            : p->ngptot - col0);
    if ((rc = gpu_run_impl(p->device, p->st_k, p->precision, variant, ncols, p->nproma, p->klev, &s.dev, s.scratch,
                           nullptr, &p->params)))
      break;
    if (hipEventRecord(s.k_done, p->st_k) != hipSuccess) { rc = CLOUDSC_EHIP; break; }
  }
  if (rc == CLOUDSC_OK && out_issued < nchunks - 1) rc = drain(nchunks - 1);
  // every copy issued, finished (also after a failure: the slots are reused)
  for (auto* v : {&p->sig_in, &p->sig_out})
    for (hsa_signal_t sg : *v) {
      const int r = wait(sg);
      if (r && !rc) rc = r;
    }
  if (hipStreamSynchronize(p->st_k) != hipSuccess && !rc) rc = CLOUDSC_EHIP;
  const auto t1 = std::chrono::steady_clock::now();
  if (rc) return rc;
  if (vk == CLOUDSC_VARIANT_KSEG)
    for (auto& s : p->slots) {
      const int r = kseg_check(p->device, p->st_k, s.scratch);
      if (r && !rc) rc = r;
    }
  if (rc) return rc;
  if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  return CLOUDSC_OK;
}

// one step's copies without the kernels, on the same engines, host arrays and
// device slots: every input chunk H2D and every output chunk D2H, each
// direction queued back to back on its engine (a slot's signals are reused
// once its previous copies are done).  The bound the pipeline is held against:
// the same bytes over the same path.  The outputs copied back are the slots'
// contents, not results.
int copies_only_on_engines(cloudsc_host_pipeline* p, double* ms) {
  const int nchunks = (p->nblocks + p->chunk_blocks - 1) / p->chunk_blocks;
  const int nslots = (int)p->slots.size();
  const void* const* hf = (const void* const*)&p->host;
  HIPCHK(hipDeviceSynchronize());
  auto wait = [](hsa_signal_t sg) {
    return hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) == 0
               ? CLOUDSC_OK : CLOUDSC_EHIP;
  };
  const auto t0 = std::chrono::steady_clock::now();
  int rc = CLOUDSC_OK;
  for (int c = 0; c < nchunks && rc == CLOUDSC_OK; c++) {
    auto& s = p->slots[c % nslots];
    if (c >= nslots && ((rc = wait(p->sig_in[c % nslots])) || (rc = wait(p->sig_out[c % nslots])))) break;
    const int b0 = c * p->chunk_blocks;
    const int nb = (b0 + p->chunk_blocks <= p->nblocks) ? p->chunk_blocks : p->nblocks - b0;
    void* const* df = (void* const*)&s.dev;
    for (int in = 1; in >= 0 && rc == CLOUDSC_OK; in--) {
      hsa_signal_t sg = in ? p->sig_in[c % nslots] : p->sig_out[c % nslots];
      int n = 0;
      for (int i = 0; i < kNumFields; i++) {
        const int dir = kFieldTable[i].dir;
        if (hf[i] && (in ? dir != FD_OUT : (dir == FD_OUT || dir == FD_INOUT))) n++;
      }
      hsa_signal_store_screlease(sg, n);
      for (int i = 0; i < kNumFields; i++) {
        const FieldDesc& d = kFieldTable[i];
        if (!hf[i] || !(in ? d.dir != FD_OUT : (d.dir == FD_OUT || d.dir == FD_INOUT))) continue;
        const size_t per = per_block_elems(d.kind, p->nproma, p->klev) * (d.is_int ? sizeof(int) : p->es);
        char* h = (char*)p->host_dev[i] + (size_t)b0 * per;
        const hsa_status_t st =
            in ? hsa_amd_memory_async_copy_on_engine(df[i], p->eng.gpu, h, p->eng.cpu, (size_t)nb * per, 0, nullptr,
                                                     sg, p->eng.h2d, true)
               : hsa_amd_memory_async_copy_on_engine(h, p->eng.cpu, df[i], p->eng.gpu, (size_t)nb * per, 0, nullptr,
                                                     sg, p->eng.d2h, true);
        if (st != HSA_STATUS_SUCCESS) {
          hsa_signal_subtract_screlease(sg, n);
          set_error_text("host pipeline: hsa_amd_memory_async_copy_on_engine failed");
          rc = CLOUDSC_EHIP;
          break;
        }
        n--;
      }
    }
  }
  for (auto* v : {&p->sig_in, &p->sig_out})
    for (hsa_signal_t sg : *v) {
      const int r = wait(sg);
      if (r && !rc) rc = r;
    }
  const auto t1 = std::chrono::steady_clock::now();
  if (rc) return rc;
  if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  return CLOUDSC_OK;
}

}  // namespace

extern "C" {

int cloudsc_host_pipeline_destroy(cloudsc_host_pipeline_t* p);

int cloudsc_host_pipeline_create(cloudsc_host_pipeline_t** out, int device, int precision, int ngptot, int nproma,
                                 int klev, int chunk_blocks, int nstreams, const cloudsc_fields_t* host) {
  if (!out || !host || chunk_blocks <= 0 || nstreams <= 0 || nstreams > 16) return CLOUDSC_EINVAL;
  *out = nullptr;
  int rc = validate_run_args(device, precision, CLOUDSC_VARIANT_KCACHE, ngptot, nproma, klev);
  if (rc) return rc;
  if (!fields_complete(host)) return CLOUDSC_EINVAL;
  cloudsc_host_pipeline* p = new cloudsc_host_pipeline();
  p->device = device; p->precision = precision; p->ngptot = ngptot; p->nproma = nproma; p->klev = klev;
  p->nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  p->chunk_blocks = chunk_blocks < p->nblocks ? chunk_blocks : p->nblocks;
  p->nstreams = nstreams;
  p->es = precision == CLOUDSC_FP64 ? sizeof(double) : sizeof(float);
  p->host = *host;
  auto fail = [&](int r) { cloudsc_host_pipeline_destroy(p); return r; };
  if (hipSetDevice(device) != hipSuccess) return fail(CLOUDSC_ENODEV);
  // the pipeline runs with the parameters current at creation, whatever a
  // later cloudsc_gpu_init does to the device's default set
  if ((rc = param_set_copy(&p->params, device_default_params(device)))) return fail(rc);
  void* const* hf = (void* const*)&p->host;
  if ((rc = pin_host_fields(p, hf))) return fail(rc);
  for (int i = 0; i < kNumFields; i++) {   // device-visible addresses of the pinned arrays (D2H blit mode)
    if (!hf[i]) continue;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, hf[i], 0) == hipSuccess) p->host_dev[i] = d;
    else (void)hipGetLastError();
  }
  for (hipStream_t* q : {&p->st_in, &p->st_k, &p->st_out})
    if (hipStreamCreateWithFlags(q, hipStreamNonBlocking) != hipSuccess) return fail(CLOUDSC_EHIP);
  // more slots than chunks would never be used
  const int nchunks = (p->nblocks + p->chunk_blocks - 1) / p->chunk_blocks;
  p->slots.resize(nstreams < nchunks ? nstreams : nchunks);
  for (auto& s : p->slots) {
    for (hipEvent_t* e : {&s.in_done, &s.k_done, &s.out_done})
      if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return fail(CLOUDSC_EHIP);
    void** df = (void**)&s.dev;
    for (int i = 0; i < kNumFields; i++) {
      if (!hf[i]) continue;
      const FieldDesc& d = kFieldTable[i];
      const size_t bytes =
          (size_t)p->chunk_blocks * per_block_elems(d.kind, nproma, klev) * (d.is_int ? sizeof(int) : p->es);
      void* q = nullptr;
      if (hipMalloc(&q, bytes) != hipSuccess) { hip_fail(hipErrorOutOfMemory, "hipMalloc"); return fail(CLOUDSC_ENOMEM); }
      p->allocs.push_back(q);
      df[i] = q;
    }
  }
  if (hipEventCreate(&p->ev0) != hipSuccess || hipEventCreate(&p->ev1) != hipSuccess) return fail(CLOUDSC_EHIP);
  // copy engines per direction: every array needs its agent address
  bool all_dev = true;
  for (int i = 0; i < kNumFields; i++) all_dev = all_dev && (!hf[i] || p->host_dev[i]);
  if (all_dev) p->eng = find_engines(device);
  if (p->eng.ok) check_engines(p->eng);
  if (p->eng.ok) {
    for (auto* v : {&p->sig_in, &p->sig_out})
      for (size_t k = 0; k < p->slots.size(); k++) {
        hsa_signal_t sg;
        if (hsa_signal_create(0, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) { p->eng.ok = false; break; }
        v->push_back(sg);
      }
  }
  *out = p;
  return CLOUDSC_OK;
}

int cloudsc_host_pipeline_run(cloudsc_host_pipeline_t* p, int variant, double* ms) {
  if (!p) return CLOUDSC_EINVAL;
  int rc = validate_run_args(p->device, p->precision, variant, p->ngptot, p->nproma, p->klev);
  if (rc) return rc;
  HIPCHK(hipSetDevice(p->device));
  const int vk = variant_kind(variant);   // without the option bits
  const int nchunks = (p->nblocks + p->chunk_blocks - 1) / p->chunk_blocks;
  const int nslots = (int)p->slots.size();
  // workspaces for the chunk size (SCC / KSEG), allocated on first use
  for (auto& s : p->slots) {
    if (vk == CLOUDSC_VARIANT_KCACHE || vk == CLOUDSC_VARIANT_SCC_PRIVATE || s.scratch_variant == vk) continue;
    const long long nb = cloudsc_gpu_scratch_bytes(p->precision, vk, p->chunk_blocks * p->nproma, p->nproma,
                                                   p->klev);
    if (nb <= 0) return CLOUDSC_EINVAL;
    if ((size_t)nb > s.scratch_bytes) {
      void* q = nullptr;
      if (hipMalloc(&q, (size_t)nb) != hipSuccess) return CLOUDSC_ENOMEM;
      p->allocs.push_back(q);
      // control words of a fresh KSEG workspace (recycled memory may hold a
      // matching tag and a stale hand-off error count), zeroed on the stream
      // that launches the kernels, so the order is the stream's
      if (hipMemsetAsync(q, 0, 256, p->st_k) != hipSuccess) return CLOUDSC_EHIP;
      s.scratch = q;
      s.scratch_bytes = (size_t)nb;
    }
    s.scratch_variant = vk;
  }
  if (p->eng.ok && g_pipe_copy.load(std::memory_order_relaxed) == PC_ENGINES)
    return run_on_engines(p, variant, vk, ms);
  const void* const* hf = (const void* const*)&p->host;
  // the three streams start after ev0 (recorded on the null stream) and ev1 waits for all of them
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipEventRecord(p->ev0, nullptr));
  for (hipStream_t q : {p->st_in, p->st_k, p->st_out}) HIPCHK(hipStreamWaitEvent(q, p->ev0, 0));
  for (int c = 0; c < nchunks && rc == CLOUDSC_OK; c++) {
    auto& s = p->slots[c % nslots];
    const bool reuse = c >= nslots;        // the slot held chunk c - nslots
    const int b0 = c * p->chunk_blocks;
    const int nb = (b0 + p->chunk_blocks <= p->nblocks) ? p->chunk_blocks : p->nblocks - b0;
    const long long col0 = (long long)b0 * p->nproma;
    const int ncols = (int)((col0 + (long long)nb * p->nproma <= p->ngptot) ? (long long)nb * p->nproma
                                                                            : p->ngptot - col0);
    void* const* df = (void* const*)&s.dev;
    // inputs: after the slot's previous kernel has read its inputs; plude
    // (INOUT) last, after the slot's previous D2H has read it back
    if (reuse) HIPCHK(hipStreamWaitEvent(p->st_in, s.k_done, 0));
    for (int part = 0; part < 2; part++) {
      if (part == 1 && reuse) HIPCHK(hipStreamWaitEvent(p->st_in, s.out_done, 0));
      for (int i = 0; i < kNumFields; i++) {
        const FieldDesc& d = kFieldTable[i];
        if (!hf[i] || d.dir == FD_OUT || (part == 0) != (d.dir != FD_INOUT)) continue;
        const size_t eb = d.is_int ? sizeof(int) : p->es;
        const size_t per = per_block_elems(d.kind, p->nproma, p->klev) * eb;
        HIPCHK(hipMemcpyAsync(df[i], (const char*)hf[i] + (size_t)b0 * per, (size_t)nb * per, hipMemcpyHostToDevice,
                              p->st_in));
      }
    }
    HIPCHK(hipEventRecord(s.in_done, p->st_in));
    // kernel: after its inputs are in and the slot's previous outputs are out
    HIPCHK(hipStreamWaitEvent(p->st_k, s.in_done, 0));
    if (reuse) HIPCHK(hipStreamWaitEvent(p->st_k, s.out_done, 0));
    rc = gpu_run_impl(p->device, p->st_k, p->precision, variant, ncols, p->nproma, p->klev, &s.dev, s.scratch,
                      nullptr, &p->params);
    if (rc) break;
    HIPCHK(hipEventRecord(s.k_done, p->st_k));
    // outputs (and plude): after the kernel
    HIPCHK(hipStreamWaitEvent(p->st_out, s.k_done, 0));
    BlitSegs bs{};
    const bool blit = g_pipe_copy.load(std::memory_order_relaxed) == PC_HIP_BLIT;
    for (int i = 0; i < kNumFields; i++) {
      const FieldDesc& d = kFieldTable[i];
      if (!hf[i] || !(d.dir == FD_OUT || d.dir == FD_INOUT)) continue;
      const size_t per = per_block_elems(d.kind, p->nproma, p->klev) * p->es;
      if (blit && p->host_dev[i] && bs.n < kMaxBlitSeg) {
        bs.src[bs.n] = (const char*)df[i];
        bs.dst[bs.n] = (char*)p->host_dev[i] + (size_t)b0 * per;
        bs.bytes[bs.n] = (unsigned long long)((size_t)nb * per);
        bs.n++;
        continue;
      }
      HIPCHK(hipMemcpyAsync((char*)hf[i] + (size_t)b0 * per, df[i], (size_t)nb * per, hipMemcpyDeviceToHost,
                            p->st_out));
    }
    if (bs.n) {
      hipLaunchKernelGGL(d2h_blit_kernel, dim3(256), dim3(256), 0, p->st_out, bs);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(s.out_done, p->st_out));
  }
  for (hipStream_t q : {p->st_in, p->st_k, p->st_out}) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e, q));
    HIPCHK(hipStreamWaitEvent(nullptr, e, 0));
    (void)hipEventDestroy(e);
  }
  HIPCHK(hipEventRecord(p->ev1, nullptr));
  HIPCHK(hipEventSynchronize(p->ev1));
  if (rc) return rc;
  // KSEG: a timed-out segment hand-off in any chunk invalidates the step (the
  // error word of a slot's workspace accumulates over its chunks; every slot's
  // word is read and cleared, also after the first failure)
  if (vk == CLOUDSC_VARIANT_KSEG)
    for (auto& s : p->slots) {
      const int r = kseg_check(p->device, p->st_k, s.scratch);
      if (r && !rc) rc = r;
    }
  if (rc) return rc;
  float t = 0.f;
  HIPCHK(hipEventElapsedTime(&t, p->ev0, p->ev1));
  if (ms) *ms = t;
  return CLOUDSC_OK;
}

int cloudsc_host_pipeline_destroy(cloudsc_host_pipeline_t* p) {
  if (!p) return CLOUDSC_EINVAL;
  (void)hipSetDevice(p->device);
  for (hipStream_t q : {p->st_in, p->st_k, p->st_out})
    if (q) { (void)hipStreamSynchronize(q); (void)hipStreamDestroy(q); }
  for (auto& s : p->slots)
    for (hipEvent_t e : {s.in_done, s.k_done, s.out_done})
      if (e) (void)hipEventDestroy(e);
  for (void* q : p->allocs) (void)hipFree(q);
  for (auto* v : {&p->sig_in, &p->sig_out})
    for (hsa_signal_t sg : *v) {
      // a failed step may leave copies running: let them finish before the memory goes
      hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
      (void)hsa_signal_destroy(sg);
    }
  for (void* h : p->pinned) (void)hipHostUnregister(h);
  param_set_free(&p->params);
  if (p->ev0) (void)hipEventDestroy(p->ev0);
  if (p->ev1) (void)hipEventDestroy(p->ev1);
  delete p;
  return CLOUDSC_OK;
}

int cloudsc_debug_host_pipeline_mapping(const cloudsc_host_pipeline_t* p, int* n_arrays, int* n_not_one_mapping) {
  if (!p || !n_arrays || !n_not_one_mapping) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(p->device));
  const void* const* hf = (const void* const*)&p->host;
  int n = 0, bad = 0;
  for (int i = 0; i < kNumFields; i++) {
    if (!hf[i]) continue;
    n++;
    if (!pinned_as_one(hf[i], field_bytes(p, i, p->nblocks))) bad++;
  }
  *n_arrays = n;
  *n_not_one_mapping = bad;
  return CLOUDSC_OK;
}

int cloudsc_debug_set_pipeline_copy(int mode) {
  if (mode < 0) mode = PC_ENGINES;
  if (mode > PC_HIP_BLIT) return CLOUDSC_EINVAL;
  g_pipe_copy.store(mode, std::memory_order_relaxed);
  return CLOUDSC_OK;
}

int cloudsc_debug_host_pipeline_copy(const cloudsc_host_pipeline_t* p, int* mode, int* h2d_engine, int* d2h_engine) {
  if (!p) return CLOUDSC_EINVAL;
  if (mode) *mode = p->eng.ok ? PC_ENGINES : PC_HIP;
  if (h2d_engine) *h2d_engine = p->eng.ok ? (int)p->eng.h2d : 0;
  if (d2h_engine) *d2h_engine = p->eng.ok ? (int)p->eng.d2h : 0;
  return CLOUDSC_OK;
}

int cloudsc_host_pipeline_copy_bound(cloudsc_host_pipeline_t* p, double* ms) {
  if (!p || !ms) return CLOUDSC_EINVAL;
  if (!p->eng.ok) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(p->device));
  return copies_only_on_engines(p, ms);
}

int cloudsc_debug_host_pipeline_engine_check(const cloudsc_host_pipeline_t* p, double* overlap, int* pairs_tried) {
  if (!p) return CLOUDSC_EINVAL;
  if (overlap) *overlap = p->eng.ok ? p->eng.overlap : 0.0;
  if (pairs_tried) *pairs_tried = p->eng.ok ? p->eng.pairs_tried : 0;
  return CLOUDSC_OK;
}

int cloudsc_debug_host_pinned(const void* ptr, long long bytes) {
  if (!ptr || bytes <= 0) return 0;
  return pinned_as_one(ptr, (size_t)bytes) ? 1 : 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// C ABI: one synchronous step on host arrays from any host thread
// (cloudsc_host_run).  This is what a per-block caller such as the reference
// C dwarf's OpenMP loop needs (cloudsc_driver.c:183-217 calls cloudsc_c() on
// one NPROMA block at a time, from every thread): no creation call, no pinned
// registration of the caller's arrays.  Each calling thread owns a context per
// device -- its stream, a pinned staging buffer and a device buffer laid out
// alike (grown to the largest call so far), a KSEG workspace and a private
// parameter set, re-uploaded only when the parameters change -- so concurrent
// callers never share state or race on a parameter block.
//
// Transfers: the active lanes of every input are packed on the host into the
// staging buffer and go to the device in ONE copy; the outputs come back in one
// copy and are unpacked.  Only lanes < ngptot of the caller's arrays are read
// or written (a caller whose arrays start at column kidia-1 of a klon-wide
// block, cloudsc_c_dropin.c, is never read or written past their end).
// ---------------------------------------------------------------------------
namespace {

struct HostRunCtx {
  hipStream_t st = nullptr;
  hipEvent_t ev[4] = {};    // profiling: before H2D, after H2D, after the kernel, after D2H
  long long calls = 0;      // calls on this context (the one that created it is profiled apart)
  char* stage = nullptr;    // pinned host
  char* dbuf = nullptr;     // device, same layout
  size_t cap = 0;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  ParamSet params;
  cloudsc_params_t cur{};
  bool have_params = false;
};
// Device memory is not released at thread exit (the runtime may be gone by
// then); cloudsc_host_run_release frees the calling thread's contexts.
thread_local HostRunCtx* t_host_ctx[kMaxDevices] = {};

// cloudsc_host_run_profile: per-call cost sums over all threads
std::atomic<bool> g_hr_prof{false};
std::mutex g_hr_prof_mu;
cloudsc_host_run_profile_t g_hr_sum{};
using HrClock = std::chrono::steady_clock;
double ms_since(HrClock::time_point t0, HrClock::time_point t1) {
  return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

// copy the active lanes between a caller's field and its packed image: the full
// blocks before the last one as one run, then `bsize` lanes of each row of the
// last block
void pack_active(char* img, const char* fld, size_t per, size_t full, size_t row, size_t lanes, bool to_img) {
  if (full) {
    if (to_img) std::memcpy(img, fld, full);
    else std::memcpy((char*)fld, img, full);
  }
  for (size_t off = full; off < full + per; off += row) {
    if (to_img) std::memcpy(img + off, fld + off, lanes);
    else std::memcpy((char*)fld + off, img + off, lanes);
  }
}

// Fault in the pages of a caller's output field that pack_active(.., false)
// will write, while the device works.  A caller's freshly allocated output
// arrays (the reference driver's) are untouched pages, and faulting them in
// during the unpack made it 2-5x slower than the copy itself
// (profiles/r06/host_run_cost.jsonl); here that cost overlaps the device's
// H2D + kernel + D2H.  madvise(MADV_POPULATE_WRITE) (Linux >= 5.14) populates
// the pages writable without accessing their contents, so it may cover whole
// pages around the active lanes; where it is refused, one byte per page of
// the active lanes (and only of them) takes an atomic add of zero -- a single
// write fault, the byte unchanged (a plain read-then-write would fault twice:
// the zero page first, then the copy on write).
void prefault_range(const char* b, size_t n) {
  constexpr size_t kPage = 4096;
  if (!n) return;
  const uintptr_t lo = (uintptr_t)b & ~(uintptr_t)(kPage - 1);
  const uintptr_t hi = ((uintptr_t)b + n + kPage - 1) & ~(uintptr_t)(kPage - 1);
#ifdef MADV_POPULATE_WRITE
  if (madvise((void*)lo, hi - lo, MADV_POPULATE_WRITE) == 0) return;
#else
  if (madvise((void*)lo, hi - lo, 23 /* MADV_POPULATE_WRITE */) == 0) return;
#endif
  for (size_t o = 0; o < n;) {
    __atomic_fetch_add((char*)b + o, (char)0, __ATOMIC_RELAXED);
    o += kPage - (((uintptr_t)(b + o)) & (kPage - 1));   // the next page's first byte
  }
}
void prefault_active(const char* fld, size_t per, size_t full, size_t row, size_t lanes) {
  if (full) prefault_range(fld, full);
  if (lanes == row) {                  // the last block's rows are whole: one range
    prefault_range(fld + full, per);
    return;
  }
  for (size_t off = full; off < full + per; off += row) prefault_range(fld + off, lanes);
}

}  // namespace

extern "C" int cloudsc_host_run(int device, int precision, int variant, int ngptot, int nproma, int klev,
                                const cloudsc_params_t* params, const cloudsc_fields_t* host) {
  const bool prof = g_hr_prof.load(std::memory_order_relaxed);
  const HrClock::time_point t_start = prof ? HrClock::now() : HrClock::time_point{};
  HrClock::time_point t_packed{}, t_enq{}, t_synced{};
  int rc = validate_run_args(device, precision, variant, ngptot, nproma, klev);
  if (rc) return rc;
  if (!params || !host || !fields_complete(host)) return CLOUDSC_EINVAL;
  if ((rc = check_params(params))) return rc;
  const bool aer = params->laericesed || params->laericeauto;
  if (aer && (!host->pre_ice || !host->picrit_aer || !host->pnice)) return CLOUDSC_EINVAL;
  const HrClock::time_point t_a0 = prof ? HrClock::now() : HrClock::time_point{};
  double alloc_ms = 0.0, scratch_ms = 0.0;
  HIPCHK(hipSetDevice(device));
  HostRunCtx*& ctx = t_host_ctx[device];
  if (!ctx) {
    ctx = new HostRunCtx();
    if (hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking) != hipSuccess) {
      delete ctx;
      ctx = nullptr;
      return CLOUDSC_EHIP;
    }
  }
  if (!ctx->have_params || std::memcmp(&ctx->cur, params, sizeof(*params)) != 0) {
    if ((rc = param_set_upload(&ctx->params, device, params))) return rc;
    ctx->cur = *params;
    ctx->have_params = true;
  }
  if (prof) alloc_ms += ms_since(t_a0, HrClock::now());
  const bool first_call = ctx->calls++ == 0;   // this call created the context (profiled apart)
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  const int bsize = ngptot - (nblocks - 1) * nproma;   // active lanes of the last block
  const size_t es = precision == CLOUDSC_FP64 ? sizeof(double) : sizeof(float);
  const void* const* hf = (const void* const*)host;
  // image layout: the inputs (and plude) first, then the outputs; 256-byte aligned fields
  size_t off[kNumFields] = {}, bytes[kNumFields] = {};
  size_t in_end = 0, total = 0;
  for (int pass = 0; pass < 2; pass++)
    for (int i = 0; i < kNumFields; i++) {
      const FieldDesc& d = kFieldTable[i];
      if (!hf[i] || (pass == 0) != (d.dir != FD_OUT)) continue;
      bytes[i] = (size_t)nblocks * per_block_elems(d.kind, nproma, klev) * (d.is_int ? sizeof(int) : es);
      off[i] = total;
      total += (bytes[i] + 255) & ~(size_t)255;
      if (pass == 0) in_end = total;
    }
  if (total > ctx->cap) {
    const HrClock::time_point t_g0 = prof ? HrClock::now() : HrClock::time_point{};
    if (ctx->stage) (void)hipHostFree(ctx->stage);
    if (ctx->dbuf) (void)hipFree(ctx->dbuf);
    ctx->stage = ctx->dbuf = nullptr;
    ctx->cap = 0;
    hipError_t e = hipHostMalloc((void**)&ctx->stage, total, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->dbuf, total);
    if (e != hipSuccess) {
      if (ctx->stage) (void)hipHostFree(ctx->stage);
      ctx->stage = nullptr;
      hip_fail(e, "host_run buffers");
      return CLOUDSC_ENOMEM;
    }
    ctx->cap = total;
    if (prof) alloc_ms += ms_since(t_g0, HrClock::now());
  }
  if (prof && !ctx->ev[0])
    for (auto& e : ctx->ev) HIPCHK(hipEventCreate(&e));
  HrClock::time_point t_setup = prof ? HrClock::now() : HrClock::time_point{};
  cloudsc_fields_t dev{};
  void** df = (void**)&dev;
  for (int i = 0; i < kNumFields; i++) {
    if (!hf[i]) continue;
    const FieldDesc& d = kFieldTable[i];
    const size_t eb = d.is_int ? sizeof(int) : es;
    const size_t per = per_block_elems(d.kind, nproma, klev) * eb;
    df[i] = ctx->dbuf + off[i];
    if (d.dir != FD_OUT)
      pack_active(ctx->stage + off[i], (const char*)hf[i], per, (size_t)(nblocks - 1) * per, (size_t)nproma * eb,
                  (size_t)bsize * eb, true);
  }
  if (prof) {
    t_packed = HrClock::now();
    HIPCHK(hipEventRecord(ctx->ev[0], ctx->st));
  }
  HIPCHK(hipMemcpyAsync(ctx->dbuf, ctx->stage, in_end, hipMemcpyHostToDevice, ctx->st));
  if (prof) HIPCHK(hipEventRecord(ctx->ev[1], ctx->st));
  const int vk = variant_kind(variant);
  if (vk == CLOUDSC_VARIANT_SCC || vk == CLOUDSC_VARIANT_KSEG) {
    const long long nb = cloudsc_gpu_scratch_bytes(precision, vk, ngptot, nproma, klev);
    if (nb <= 0) return CLOUDSC_EINVAL;
    if ((size_t)nb > ctx->scratch_bytes) {
      const HrClock::time_point t_s0 = prof ? HrClock::now() : HrClock::time_point{};
      if (ctx->scratch) (void)hipFree(ctx->scratch);
      ctx->scratch = nullptr;
      ctx->scratch_bytes = 0;
      const hipError_t e = hipMalloc(&ctx->scratch, (size_t)nb);
      if (e != hipSuccess) { ctx->scratch = nullptr; hip_fail(e, "hipMalloc"); return CLOUDSC_ENOMEM; }
      ctx->scratch_bytes = (size_t)nb;
      HIPCHK(hipMemsetAsync(ctx->scratch, 0, 256, ctx->st));   // control words (recycled memory)
      if (prof) {
        scratch_ms = ms_since(t_s0, HrClock::now());
        alloc_ms += scratch_ms;
      }
    }
  }
  rc = gpu_run_impl(device, ctx->st, precision, variant, ngptot, nproma, klev, &dev, ctx->scratch, nullptr,
                    &ctx->params);
  if (rc) {
    (void)hipStreamSynchronize(ctx->st);
    return rc;
  }
  if (prof) HIPCHK(hipEventRecord(ctx->ev[2], ctx->st));
  // plude (INOUT) sits in the input region: bring back from it to the end
  const int iplude = (int)(offsetof(cloudsc_fields_t, plude) / sizeof(void*));
  HIPCHK(hipMemcpyAsync(ctx->stage + off[iplude], ctx->dbuf + off[iplude], total - off[iplude],
                        hipMemcpyDeviceToHost, ctx->st));
  if (prof) {
    HIPCHK(hipEventRecord(ctx->ev[3], ctx->st));
    t_enq = HrClock::now();
  }
  // while the device works: fault in the caller's output pages the unpack will write
  for (int i = 0; i < kNumFields; i++) {
    const FieldDesc& d = kFieldTable[i];
    if (!hf[i] || !(d.dir == FD_OUT || d.dir == FD_INOUT)) continue;
    const size_t per = per_block_elems(d.kind, nproma, klev) * es;
    prefault_active((const char*)hf[i], per, (size_t)(nblocks - 1) * per, (size_t)nproma * es, (size_t)bsize * es);
  }
  HIPCHK(hipStreamSynchronize(ctx->st));
  if (prof) t_synced = HrClock::now();
  if (vk == CLOUDSC_VARIANT_KSEG && (rc = kseg_check(device, ctx->st, ctx->scratch))) return rc;
  for (int i = 0; i < kNumFields; i++) {
    const FieldDesc& d = kFieldTable[i];
    if (!hf[i] || !(d.dir == FD_OUT || d.dir == FD_INOUT)) continue;
    const size_t per = per_block_elems(d.kind, nproma, klev) * es;
    pack_active(ctx->stage + off[i], (const char*)hf[i], per, (size_t)(nblocks - 1) * per, (size_t)nproma * es,
                (size_t)bsize * es, false);
  }
  if (prof) {
    const HrClock::time_point t_end = HrClock::now();
    float dev_ms[3] = {0.f, 0.f, 0.f};
    for (int q = 0; q < 3; q++) HIPCHK(hipEventElapsedTime(&dev_ms[q], ctx->ev[q], ctx->ev[q + 1]));
    std::lock_guard<std::mutex> lk(g_hr_prof_mu);
    if (first_call) {   // the context's creation (and the runtime's start-up): apart
      g_hr_sum.first_calls++;
      g_hr_sum.first_calls_ms += ms_since(t_start, t_end);
      return CLOUDSC_OK;
    }
    g_hr_sum.calls++;
    g_hr_sum.alloc_ms += alloc_ms;
    g_hr_sum.setup_ms += ms_since(t_start, t_setup) - (alloc_ms - scratch_ms);
    g_hr_sum.pack_ms += ms_since(t_setup, t_packed);
    g_hr_sum.enqueue_ms += ms_since(t_packed, t_enq) - scratch_ms;
    g_hr_sum.h2d_ms += dev_ms[0];
    g_hr_sum.kernel_ms += dev_ms[1];
    g_hr_sum.d2h_ms += dev_ms[2];
    g_hr_sum.wait_ms += ms_since(t_enq, t_synced);
    g_hr_sum.unpack_ms += ms_since(t_synced, t_end);
    g_hr_sum.total_ms += ms_since(t_start, t_end);
    g_hr_sum.max_call_ms = std::max(g_hr_sum.max_call_ms, ms_since(t_start, t_end));
  }
  return CLOUDSC_OK;
}

extern "C" int cloudsc_host_run_profile(int mode, cloudsc_host_run_profile_t* out) {
  if (mode < -1 || mode > 1) return CLOUDSC_EINVAL;
  std::lock_guard<std::mutex> lk(g_hr_prof_mu);
  if (mode == 1) {
    g_hr_sum = cloudsc_host_run_profile_t{};
    g_hr_prof.store(true);
  } else {
    if (out) *out = g_hr_sum;
    if (mode == -1) g_hr_prof.store(false);
  }
  return CLOUDSC_OK;
}

extern "C" int cloudsc_host_run_release(void) {
  for (int d = 0; d < kMaxDevices; d++) {
    HostRunCtx* ctx = t_host_ctx[d];
    if (!ctx) continue;
    (void)hipSetDevice(d);
    if (ctx->st) { (void)hipStreamSynchronize(ctx->st); (void)hipStreamDestroy(ctx->st); }
    for (auto& e : ctx->ev)
      if (e) (void)hipEventDestroy(e);
    if (ctx->stage) (void)hipHostFree(ctx->stage);
    if (ctx->dbuf) (void)hipFree(ctx->dbuf);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    param_set_free(&ctx->params);
    delete ctx;
    t_host_ctx[d] = nullptr;
  }
  return CLOUDSC_OK;
}
