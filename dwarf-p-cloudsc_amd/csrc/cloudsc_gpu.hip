// cloudsc_gpu.hip -- libcloudsc_amd.so: the C ABI of include/cloudsc_amd.h on
// top of the hand-written CDNA4 kernels.
//
//   * parameters -> a device-memory block per parameter set (fp64 + fp32
//     mirrors, host-folded), passed to every launch by pointer and read with
//     scalar loads through the constant address space.  Each device has a
//     default set (cloudsc_gpu_init); every state and host pipeline owns its
//     own, so two states with different parameters never see each other's.
//     This replaces the TECLDP device struct passed by pointer + the 28
//     by-value scalars of src/cloudsc_cuda/cloudsc/cloudsc_driver.cu:312,383,411-416.
//   * cloudsc_gpu_run: one launch, NPROMA block -> workgroup, column -> lane
//     (KCACHE, SCC) or a persistent work queue of (level segment, 64-column
//     sub-block) items (KSEG).
//
// No CPU fallback: every GPU entry point fails with a CLOUDSC_E* code if HIP or
// the device is unavailable.  (cloudsc_cpu_run, cloudsc_cpu.cpp, is a separate,
// explicitly selected host variant, never substituted for a GPU run.)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "cloudsc_amd.h"
#include "cloudsc_dev.h"
#include "cloudsc_internal.h"
#include "cloudsc_kcache.h"
#include "cloudsc_params.h"
#include "cloudsc_scc.h"

using namespace cloudsc;
using namespace cloudsc_impl;

// ---------------------------------------------------------------------------
// error text (per calling thread)
// ---------------------------------------------------------------------------
namespace cloudsc_impl {
thread_local char g_hip_err[256] = "";
int hip_fail(hipError_t e, const char* what) {
  snprintf(g_hip_err, sizeof(g_hip_err), "%s: %s", what, hipGetErrorString(e));
  return CLOUDSC_EHIP;
}
void set_error_text(const char* text) { snprintf(g_hip_err, sizeof(g_hip_err), "%s", text); }
}  // namespace cloudsc_impl

// ---------------------------------------------------------------------------
// parameter sets
// ---------------------------------------------------------------------------
namespace {

// device layout of one parameter set: the fp64 mirror, then the fp32 one
constexpr size_t kSpOffset = (sizeof(DevParams<double>) + 255) & ~(size_t)255;
constexpr size_t kParamBlockBytes = kSpOffset + sizeof(DevParams<float>);

// the per-device default parameter sets (cloudsc_gpu_init)
std::mutex g_default_mu;
ParamSet g_default[kMaxDevices];

}  // namespace

namespace cloudsc_impl {

int check_params(const cloudsc_params_t* p) {
  if (!p) return CLOUDSC_EINVAL;
  if (p->ncldtop < 2) return CLOUDSC_EINVAL;        // the physics reads level jk-1 (za, ztp1)
  if (p->nssopt < 0 || p->nssopt > 3) return CLOUDSC_EINVAL;
  if (!(p->ptsphy > 0.0)) return CLOUDSC_EINVAL;
  return CLOUDSC_OK;
}

int param_set_upload(ParamSet* ps, int device, const cloudsc_params_t* p) {
  int rc = check_params(p);
  if (rc) return rc;
  HIPCHK(hipSetDevice(device));
  if (!ps->dev) {
    hipError_t e = hipMalloc(&ps->dev, kParamBlockBytes);
    if (e != hipSuccess) { ps->dev = nullptr; hip_fail(e, "hipMalloc(params)"); return CLOUDSC_ENOMEM; }
  }
  std::vector<char> blk(kParamBlockBytes, 0);
  const DevParams<double> dp = fold_params<double>(*p);
  const DevParams<float> sp = fold_params<float>(*p);
  std::memcpy(blk.data(), &dp, sizeof(dp));
  std::memcpy(blk.data() + kSpOffset, &sp, sizeof(sp));
  // hipMemcpy from pageable memory may return before the bytes have reached the
  // device, and the launches that read them run on non-blocking streams, which
  // do not wait for the null stream: a state created right after another one's
  // destruction read part of a stale parameter block in its first launch.
  // Copy on the null stream and wait for it.
#ifdef CLOUDSC_DEBUG_UNORDERED_PARAM_UPLOAD
  // diagnostic build only: the round-3 upload, unordered with the launches
  // (profiles/r04/contiguous_alloc_hazard.txt re-introduces it on purpose)
  HIPCHK(hipMemcpy(ps->dev, blk.data(), kParamBlockBytes, hipMemcpyHostToDevice));
#else
  HIPCHK(hipMemcpyAsync(ps->dev, blk.data(), kParamBlockBytes, hipMemcpyHostToDevice, nullptr));
  HIPCHK(hipStreamSynchronize(nullptr));
#endif
  ps->device = device;
  ps->aer = p->laericesed || p->laericeauto;
  ps->ncldtop = p->ncldtop;
  return CLOUDSC_OK;
}

int param_set_copy(ParamSet* dst, const ParamSet* src) {
  if (!src || !src->dev) return CLOUDSC_ENOINIT;
  HIPCHK(hipSetDevice(src->device));
  if (!dst->dev) {
    hipError_t e = hipMalloc(&dst->dev, kParamBlockBytes);
    if (e != hipSuccess) { dst->dev = nullptr; hip_fail(e, "hipMalloc(params)"); return CLOUDSC_ENOMEM; }
  }
  HIPCHK(hipMemcpyAsync(dst->dev, src->dev, kParamBlockBytes, hipMemcpyDeviceToDevice, nullptr));
  HIPCHK(hipStreamSynchronize(nullptr));   // D2D hipMemcpy does not wait either (param_set_upload)
  dst->device = src->device;
  dst->aer = src->aer;
  dst->ncldtop = src->ncldtop;
  return CLOUDSC_OK;
}

void param_set_free(ParamSet* ps) {
  if (ps && ps->dev) {
    (void)hipSetDevice(ps->device);
    (void)hipFree(ps->dev);
    ps->dev = nullptr;
  }
}

const ParamSet* device_default_params(int device) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lk(g_default_mu);
  return g_default[device].dev ? &g_default[device] : nullptr;
}

bool fields_complete(const cloudsc_fields_t* f) {
  const void* req[] = {f->pt, f->pq, f->tendency_tmp_t, f->tendency_tmp_q, f->tendency_tmp_a,
                       f->tendency_tmp_cld, f->pvfl, f->pvfi, f->phrsw, f->phrlw, f->pvervel, f->pap,
                       f->paph, f->plsm, f->ktype, f->plu, f->psnde, f->pmfu, f->pmfd, f->pa, f->pclv,
                       f->psupsat, f->plude, f->tendency_loc_t, f->tendency_loc_q, f->tendency_loc_a,
                       f->tendency_loc_cld, f->pcovptot, f->prainfrac_toprfz, f->pfsqlf, f->pfsqif,
                       f->pfcqnng, f->pfcqlng, f->pfsqrf, f->pfsqsf, f->pfcqrng, f->pfcqsng,
                       f->pfsqltur, f->pfsqitur, f->pfplsl, f->pfplsn, f->pfhpsl, f->pfhpsn};
  for (const void* q : req)
    if (!q) return false;
  return true;
}

}  // namespace cloudsc_impl

namespace {

template <typename real>
KArgs<real> make_args(const cloudsc_fields_t* f, int ngptot, int nproma, int klev, const ParamSet& ps) {
  KArgs<real> a;
  a.pt = (const real*)f->pt; a.pq = (const real*)f->pq;
  a.ttt = (const real*)f->tendency_tmp_t; a.ttq = (const real*)f->tendency_tmp_q;
  a.tta = (const real*)f->tendency_tmp_a; a.ttcld = (const real*)f->tendency_tmp_cld;
  a.pvfl = (const real*)f->pvfl; a.pvfi = (const real*)f->pvfi;
  a.phrsw = (const real*)f->phrsw; a.phrlw = (const real*)f->phrlw; a.pvervel = (const real*)f->pvervel;
  a.pap = (const real*)f->pap; a.paph = (const real*)f->paph; a.plsm = (const real*)f->plsm;
  a.ktype = f->ktype;
  a.plu = (const real*)f->plu; a.psnde = (const real*)f->psnde; a.pmfu = (const real*)f->pmfu;
  a.pmfd = (const real*)f->pmfd; a.pa = (const real*)f->pa; a.pclv = (const real*)f->pclv;
  a.psupsat = (const real*)f->psupsat; a.picrit_aer = (const real*)f->picrit_aer;
  a.pre_ice = (const real*)f->pre_ice; a.pnice = (const real*)f->pnice;
  a.plude = (real*)f->plude; a.plude_in = (const real*)f->plude; a.tlt = (real*)f->tendency_loc_t; a.tlq = (real*)f->tendency_loc_q;
  a.tla = (real*)f->tendency_loc_a; a.tlcld = (real*)f->tendency_loc_cld;
  a.pcovptot = (real*)f->pcovptot; a.prainfrac = (real*)f->prainfrac_toprfz;
  a.pfsqlf = (real*)f->pfsqlf; a.pfsqif = (real*)f->pfsqif; a.pfcqnng = (real*)f->pfcqnng;
  a.pfcqlng = (real*)f->pfcqlng; a.pfsqrf = (real*)f->pfsqrf; a.pfsqsf = (real*)f->pfsqsf;
  a.pfcqrng = (real*)f->pfcqrng; a.pfcqsng = (real*)f->pfcqsng; a.pfsqltur = (real*)f->pfsqltur;
  a.pfsqitur = (real*)f->pfsqitur; a.pfplsl = (real*)f->pfplsl; a.pfplsn = (real*)f->pfplsn;
  a.pfhpsl = (real*)f->pfhpsl; a.pfhpsn = (real*)f->pfhpsn;
  a.par = (const DevParams<real>*)((const char*)ps.dev + (sizeof(real) == 8 ? 0 : kSpOffset));
  a.ngptot = ngptot; a.nproma = nproma; a.klev = klev;
  return a;
}

// the launch's parameter block, as a constant-address-space pointer (scalar
// loads), typed with the kernel's choice of single-precision exp/pow forms
template <typename real, bool FAST>
__device__ __forceinline__ cptr<DevParamsT<real, FAST>> params_of(cptr<KArgs<real>> ka) {
  return (cptr<DevParamsT<real, FAST>>)((const KArgs<real>*)ka)->par;
}

}  // namespace

// Kernel entry points.  The KArgs struct is the first explicit kernel argument,
// i.e. it sits at offset 0 of the kernarg segment; the bodies read it (and the
// parameter block it points at) through constant-address-space pointers.
// FAST: fp32 exp/pow in their float-internal device forms (the CLOUDSC_FP32
// default); false: the reference CPU build's algorithms (always for fp64).
template <typename real, int WAVES, int PF, bool AER, bool LDSC, bool FAST = false>
__global__ void __launch_bounds__(256, WAVES) kcache_entry(const KArgs<real> a) {
  (void)a;
  libm_tables_to_lds<real>();
  const cptr<KArgs<real>> ka = (cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr();
  cloudsc_kcache_body<real, PF, AER, LDSC>(ka, params_of<real, FAST>(ka));
}
template <typename real, int WAVES, int PF, bool AER, bool LDSC, bool FAST = false>
__global__ void __launch_bounds__(256, WAVES) kseg_entry(const KArgs<real> a, const PersistArgs<real> pa) {
  (void)a;
  libm_tables_to_lds<real>();
  const cptr<KArgs<real>> ka = (cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr();
  cloudsc_kcache_persistent_body<real, PF, AER, LDSC>(ka, params_of<real, FAST>(ka), pa);
}
template <typename real, bool AER, bool FAST = false>
__global__ void __launch_bounds__(256) scc_entry(const KArgs<real> a, const SccScratch<real> s) {
  (void)a;
  libm_tables_to_lds<real>();
  const cptr<KArgs<real>> ka = (cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr();
  cloudsc_scc_body<real, AER>(ka, s, params_of<real, FAST>(ka));
}
template <typename real, bool AER, bool FAST = false>
__global__ void __launch_bounds__(256) scc_private_entry(const KArgs<real> a) {
  (void)a;
  libm_tables_to_lds<real>();
  const cptr<KArgs<real>> ka = (cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr();
  cloudsc_scc_private_body<real, AER>(ka, params_of<real, FAST>(ka));
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
namespace {

// Kernel configuration: occupancy target (waves per SIMD, via __launch_bounds__)
// x load schedule (PF) x where the carried state lives (LDSC).  The product
// library instantiates only the measured defaults:
//   fp64: 2 waves/SIMD, carried state and neighbour planes in registers, the
//         next level's first-consumed inputs issued in the middle of the level
//         (cfg 23, PF 3; round 3: 0.8 % faster than cfg 20 on two boxes,
//         profiles/r03/sweep_pf3_fp64.jsonl; cfg 20 was 1.8 % faster than the
//         LDS-carry cfg 122, profiles/r01/sweep_kseg_cfgs_nt.jsonl);
//   fp32: 2 waves/SIMD with the register prefetch of level k+1 (cfg 21) -- 1.8-3.5 %
//         faster than round 1's 3-wave cfg 31 on the same box (profiles/r02/fp32_cfg_sweep.jsonl;
//         cfg 31 was 2-3 % faster than the 4-wave LDS-carry cfg 140, sweep_fp32_cfgs_libm.jsonl).
// The diagnostic build (-DCLOUDSC_DEBUG_KNOBS, `make variant`) instantiates the
// whole table and reads CLOUDSC_KCACHE_CFG / CLOUDSC_KSEG_* from the environment
// (tools/sweep.py); the product library never reads the environment.
template <typename real> struct DefaultCfg;
template <> struct DefaultCfg<double> { static constexpr int code = 23, waves = 2, pf = 3; };
#ifndef CLOUDSC_FP32_PF   // experiment builds: the fp32 load schedule (make variant VFLAGS=-DCLOUDSC_FP32_PF=3)
#define CLOUDSC_FP32_PF 1
#endif
template <> struct DefaultCfg<float> {
  static constexpr int code = 20 + CLOUDSC_FP32_PF, waves = 2, pf = CLOUDSC_FP32_PF;
};

#ifdef CLOUDSC_DEBUG_KNOBS
// code: [1]<waves><pf> -- leading 1 = carried state in LDS
#define CLOUDSC_FOR_EACH_CFG(X) \
  X(10, 1, 0, false) X(11, 1, 1, false) X(20, 2, 0, false) X(21, 2, 1, false) X(30, 3, 0, false) \
  X(31, 3, 1, false) X(40, 4, 0, false) X(41, 4, 1, false) X(120, 2, 0, true) X(121, 2, 1, true) X(23, 2, 3, false) X(24, 2, 4, false) X(33, 3, 3, false) \
  X(122, 2, 2, true) X(130, 3, 0, true) X(132, 3, 2, true) X(22, 2, 2, false) X(131, 3, 1, true) X(140, 4, 0, true) \
  X(123, 2, 3, true) X(133, 3, 3, true)
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
#endif

// One physics-kernel launch.  With `ev`, the dispatch packet itself records the
// start and stop timestamps (hipExtLaunchKernelGGL), so timing a step adds no
// event packets between consecutive kernels.
template <typename... Args>
void launch_physics(void (*kern)(Args...), dim3 grid, dim3 block, size_t lds, hipStream_t st, const LaunchEvents* ev,
                    Args... args) {
  if (ev) hipExtLaunchKernelGGL(kern, grid, block, (std::uint32_t)lds, st, ev->start, ev->stop, 0u, args...);
  else hipLaunchKernelGGL(kern, grid, block, lds, st, args...);
}

template <typename real, bool AER, bool FAST>
int launch_kcache(hipStream_t st, const KArgs<real>& a, int nblocks, int nproma, const LaunchEvents* ev) {
#ifdef CLOUDSC_DEBUG_KNOBS
  switch (env_int("CLOUDSC_KCACHE_CFG", DefaultCfg<real>::code)) {
#define X(code, w, pf, ldsc)                                                                                 \
  case code:                                                                                                 \
    launch_physics(kcache_entry<real, w, pf, AER, ldsc, FAST>, dim3(nblocks), dim3(nproma),                 \
                   ldsc ? carry_lds_bytes<real>(nproma) : 0, st, ev, a);                                     \
    return CLOUDSC_OK;
    CLOUDSC_FOR_EACH_CFG(X)
#undef X
    default: return CLOUDSC_EINVAL;
  }
#else
  launch_physics(kcache_entry<real, DefaultCfg<real>::waves, DefaultCfg<real>::pf, AER, false, FAST>, dim3(nblocks),
                 dim3(nproma), 0, st, ev, a);
  return CLOUDSC_OK;
#endif
}

// ---- persistent segmented variant ----
// Every item is one wave: a block of NPROMA > 64 columns is run as
// ceil(NPROMA/64) 64-column sub-blocks (the block layout is unchanged: sub-block
// h is columns h*64.. of each plane of the block), so every NPROMA runs with the
// one-wave schedule that measures fastest (profiles/r01/nproma_sweep_*).
int kseg_nsub(int nproma) { return (nproma + 63) / 64; }
int kseg_wg(int nproma) { return nproma < 64 ? nproma : 64; }
// workspace: [err, tag, clock sums..][stripe counters, one per 128 B][flags: nblocks*nsub][carry state]
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
constexpr size_t kKsegCtrOffset = 256;                                   // bytes
constexpr size_t kKsegFlagOffset = kKsegCtrOffset + kKsegStripes * kKsegCtrStride * sizeof(unsigned);
static_assert(kKsegFlagOffset == 1280, "KSEG control layout");
static_assert(sizeof(KsegEpoch::base) / sizeof(unsigned) == kKsegStripes, "one epoch base per stripe");
size_t kseg_ctl_bytes(int nblocks, int nproma) {
  return align256(kKsegFlagOffset + (size_t)nblocks * kseg_nsub(nproma) * sizeof(unsigned));
}
template <typename real>
size_t kseg_scratch_bytes(int nblocks, int nproma) {
  return kseg_ctl_bytes(nblocks, nproma) + (size_t)nblocks * kCarryN * nproma * sizeof(real);
}

// Segmentation, measured (profiles/r01/kseg_nseg_sweep*.jsonl,
// kseg_bounds_sweep_*.jsonl), for one-wave items (2048 slots): 2 segments, the
// second one smaller ("guided": the items dequeued last are short, so the tail
// is short; lower levels also cost more per level) -- the split at NCLDTOP +
// a share of the physics levels: 60 % in rounds 1-2 (1.768 ms against 1.788 at
// 62 %, profiles/r01/kseg_bounds_sweep_nt.jsonl); re-tuned in round 3 for the
// current kernels, interleaved on three boxes (profiles/r03/kseg_split_sweep.txt):
// fp32 50 % (-2.5 / -2.6 / -1.0 % against 60), fp64 55 % (-1.9 / -0.8 / +0.8 /
// -1.6 % on four boxes); 3 or 4 guided segments are 2.6-12 % slower.  Each hand-off
// costs 19 values out and in plus an L1 invalidate, so fewer segments win once
// the tail is short.
constexpr int kKsegNseg = 2;
#ifdef CLOUDSC_KSEG_SPLIT_PCT   // experiment builds override both (make variant VFLAGS=-DCLOUDSC_KSEG_SPLIT_PCT=..)
template <typename real> constexpr int kKsegSplitPct = CLOUDSC_KSEG_SPLIT_PCT;
#else
template <typename real> constexpr int kKsegSplitPct = sizeof(real) == 8 ? 55 : 50;
#endif

void kseg_bounds(int nseg, int klev, int ncldtop, int split_pct, int* lev) {
  const int top = ncldtop - 1 < klev ? (ncldtop - 1 > 0 ? ncldtop - 1 : 0) : klev;
  const int phys = klev - top;
  lev[0] = 0;
  if (nseg == 2) {
    lev[1] = top + (int)(((long long)split_pct * phys + 50) / 100);
    if (lev[1] <= 0) lev[1] = 1;
    if (lev[1] >= klev) lev[1] = klev - 1;
  } else {
    for (int sgm = 1; sgm < nseg; sgm++) lev[sgm] = top + (int)(((long long)phys * sgm + nseg / 2) / nseg);
  }
  lev[nseg] = klev;
}

// dequeue stripes of a grid (cloudsc_kcache.h): one per XCD, never more than workgroups
int kseg_nstripes(int grid) { return grid < kKsegStripes ? (grid > 0 ? grid : 1) : kKsegStripes; }

// consumer spin bound of a KSEG hand-off (cloudsc_debug_set_kseg_spin_limit)
std::atomic<unsigned> g_kseg_spin_limit{1u << 24};
// schedule overrides for the tests of the hand-off (cloudsc_debug_set_kseg_schedule); 0 = default
std::atomic<int> g_kseg_nseg{0}, g_kseg_grid{0};

}  // namespace

// KSEG workspace words: [1] timed-out hand-offs (sticky: accumulated over
// launches until cloudsc_gpu_check reads and clears it), [2] a tag marking [1]
// as initialised, [32..35] two 64-bit clock sums (PersistArgs::clk, accumulated
// like [1]), [64 + 32 s] the dequeue counter of stripe s, [320..] per-sub-block
// flags.  This
// kernel zeroes the counter and the flags before every launch of the low-level
// entry points, and before the first launch on a state's workspace (later
// launches of the state continue the counter and the flag stamps, KsegEpoch);
// the first launch on a workspace (tag absent) also zeroes the error word.
constexpr unsigned kKsegTag = 0xC105D5C1u;
constexpr size_t kKsegClkOffset = 128;   // bytes: words [32..35]
__global__ void __launch_bounds__(256) kseg_prepare_kernel(unsigned* ws, int nflags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && ws[2] != kKsegTag) { ws[1] = 0u; ws[2] = kKsegTag; ws[32] = ws[33] = ws[34] = ws[35] = 0u; }
  if (i < kKsegStripes) ws[kKsegCtrOffset / 4 + i * kKsegCtrStride] = 0u;
  for (int j = i; j < nflags; j += gridDim.x * blockDim.x) ws[kKsegFlagOffset / 4 + j] = 0u;
}

namespace {

template <typename real, int WAVES, int PF, bool AER, bool LDSC, bool FAST>
int launch_kseg_cfg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems,
                    int* grid_out, const LaunchEvents* ev) {
  const int nseg = pa.nseg;
  auto kern = kseg_entry<real, WAVES, PF, AER, LDSC, FAST>;
  const int wg = kseg_wg(nproma);
  const size_t lds = LDSC ? carry_lds_bytes<real>(wg) : 0;
  // Waves per SIMD: as many as fit, but no more than whole rounds of the work
  // units (one column's 64-column sub-block) per SIMD: 2560 units on 1024 SIMDs
  // take 2 waves each; a third resident wave (fp32 fits 3) would only find a
  // next-segment item and spin until its predecessor finishes (fp32 KSEG 1.12 ms
  // at 2 waves/SIMD against 1.23 ms at 3, profiles/r02/kseg_grid_sweep.jsonl).
  // An over-estimate of residency only delays the extra workgroups: progress
  // never depends on it, items are dequeued in order.
  // Cached per workgroup size; threads driving different devices may race here, hence atomics.
  static std::atomic<int> cache[65];
  int per_cu = cache[wg].load(std::memory_order_relaxed);
  if (!per_cu) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, wg, lds) != hipSuccess || n <= 0) n = 1;
    per_cu = n;
    cache[wg].store(n, std::memory_order_relaxed);
  }
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    ncu = 256;
  constexpr int kSimdsPerCu = 4;                       // CDNA4 compute unit
  const int simds = kSimdsPerCu * ncu;
  const int units = nitems / (nseg > 0 ? nseg : 1);   // 64-column sub-blocks
  const int per_simd = per_cu / kSimdsPerCu > 0 ? per_cu / kSimdsPerCu : 1;
  int w = units / simds;
  if (w < 1) w = 1;
  if (w > per_simd) w = per_simd;
  int grid = per_cu < kSimdsPerCu ? per_cu * ncu : w * simds;
  if (const int g = g_kseg_grid.load(std::memory_order_relaxed)) grid = g;
#ifdef CLOUDSC_DEBUG_KNOBS
  grid = env_int("CLOUDSC_KSEG_GRID", 0) > 0 ? env_int("CLOUDSC_KSEG_GRID", 0) : grid;
#endif
  if (grid > nitems) grid = nitems;
  PersistArgs<real> pg = pa;
  pg.nstripes = kseg_nstripes(grid);
  launch_physics(kern, dim3(grid), dim3(wg), lds, st, ev, a, pg);
  *grid_out = grid;
  return CLOUDSC_OK;
}

template <typename real, bool AER, bool FAST>
int launch_kseg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems,
                int* grid_out, const LaunchEvents* ev) {
#ifdef CLOUDSC_DEBUG_KNOBS
  switch (env_int("CLOUDSC_KCACHE_CFG", DefaultCfg<real>::code)) {
#define X(code, w, pf, ldsc) \
  case code: return launch_kseg_cfg<real, w, pf, AER, ldsc, FAST>(st, a, pa, nproma, nitems, grid_out, ev);
    CLOUDSC_FOR_EACH_CFG(X)
#undef X
    default: return CLOUDSC_EINVAL;
  }
#else
  return launch_kseg_cfg<real, DefaultCfg<real>::waves, DefaultCfg<real>::pf, AER, false, FAST>(st, a, pa, nproma, nitems,
                                                                                        grid_out, ev);
#endif
}

// Experiment builds (make variant VFLAGS=-DCLOUDSC_ONLY_KSEG=8 ...) instantiate
// only the KSEG kernel of one element size without aerosols -- one kernel to
// compile instead of twelve, for the per-phase ablation builds of
// tools/ablation.sh; every other combination returns CLOUDSC_EINVAL.
#ifdef CLOUDSC_ONLY_KSEG
#define CLOUDSC_KEEP_KERNEL(real_, kseg_, aer_) (sizeof(real_) == CLOUDSC_ONLY_KSEG && (kseg_) && !(aer_))
#else
#define CLOUDSC_KEEP_KERNEL(real_, kseg_, aer_) true
#endif

template <typename real, bool FAST>
int launch_v(hipStream_t st, int variant, const cloudsc_fields_t* f, int ngptot, int nproma, int klev,
             void* scratch, const void* plude_in, const ParamSet& ps, KsegEpoch* ep, const LaunchEvents* ev) {
#ifdef CLOUDSC_ONLY_KSEG
  if (variant != CLOUDSC_VARIANT_KSEG || ps.aer || sizeof(real) != CLOUDSC_ONLY_KSEG) return CLOUDSC_EINVAL;
#endif
  KArgs<real> a = make_args<real>(f, ngptot, nproma, klev, ps);
  if (plude_in) a.plude_in = (const real*)plude_in;
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  const bool aer = ps.aer;
  if (aer && (!f->pre_ice || !f->picrit_aer || !f->pnice)) return CLOUDSC_EINVAL;
  int rc = CLOUDSC_OK;
  if (variant == CLOUDSC_VARIANT_KCACHE) {
    if constexpr (CLOUDSC_KEEP_KERNEL(real, false, false))
      rc = aer ? launch_kcache<real, true, FAST>(st, a, nblocks, nproma, ev)
               : launch_kcache<real, false, FAST>(st, a, nblocks, nproma, ev);
  } else if (variant == CLOUDSC_VARIANT_KSEG) {
    if (!scratch) return CLOUDSC_EINVAL;
    PersistArgs<real> pa;
    pa.ctr = (unsigned*)((char*)scratch + kKsegCtrOffset);
    pa.err = (unsigned*)scratch + 1;
    pa.clk = (unsigned long long*)((char*)scratch + kKsegClkOffset);
    pa.flags = (unsigned*)((char*)scratch + kKsegFlagOffset);
    pa.state = (real*)((char*)scratch + kseg_ctl_bytes(nblocks, nproma));
    pa.nsub = kseg_nsub(nproma);
    pa.spin_limit = g_kseg_spin_limit.load(std::memory_order_relaxed);
    // item order (segment, block, sub-block); (segment, sub-block, block) measured
    // the same within noise at NPROMA 128, 2 % slower at 256 (profiles/r01/kseg_subblock_order.jsonl)
    pa.sb_major = 0;
    pa.nseg = kKsegNseg;
    if (const int n = g_kseg_nseg.load(std::memory_order_relaxed)) pa.nseg = n > kMaxSeg ? kMaxSeg : n;
#ifdef CLOUDSC_DEBUG_KNOBS
    pa.sb_major = env_int("CLOUDSC_KSEG_SBMAJOR", 0) != 0;
    pa.nseg = env_int("CLOUDSC_KSEG_NSEG", kKsegNseg);
    pa.nseg = pa.nseg < 1 ? 1 : (pa.nseg > kMaxSeg ? kMaxSeg : pa.nseg);
#endif
    if (pa.nseg > klev) pa.nseg = klev;
    pa.nblocks = nblocks;
    for (int q = 0; q <= kMaxSeg; q++) pa.lev[q] = klev;
    kseg_bounds(pa.nseg, klev, ps.ncldtop, kKsegSplitPct<real>, pa.lev);
#ifdef CLOUDSC_DEBUG_KNOBS
    if (const char* e = getenv("CLOUDSC_KSEG_BOUNDS")) {   // explicit interior boundaries
      int n = 1, v = 0;
      const char* q = e;
      while (*q && n < kMaxSeg) {
        v = (int)strtol(q, (char**)&q, 10);
        if (v <= pa.lev[n - 1] || v >= klev) break;
        pa.lev[n++] = v;
        if (*q == ',') q++;
      }
      pa.nseg = n;
      pa.lev[n] = klev;
    }
#endif
    pa.nitems = pa.nseg * nblocks * pa.nsub;
    const bool zero_ws = !(ep && ep->ready);
    if (zero_ws) {
      const int nflags = nblocks * pa.nsub;
      const int g = (nflags + 255) / 256 < 64 ? (nflags + 255) / 256 : 64;
      hipLaunchKernelGGL(kseg_prepare_kernel, dim3(g > 0 ? g : 1), dim3(256), 0, st, (unsigned*)scratch, nflags);
      if (ep) ep->ready = false;
    }
    for (int q = 0; q < kKsegStripes; q++) pa.base[q] = zero_ws ? 0u : ep->base[q];
    pa.stamp = zero_ws ? 0u : ep->stamp;
    int grid = 0;
    if constexpr (CLOUDSC_KEEP_KERNEL(real, true, true))
      rc = aer ? launch_kseg<real, true, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev)
               : launch_kseg<real, false, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev);
    else if constexpr (CLOUDSC_KEEP_KERNEL(real, true, false))
      rc = launch_kseg<real, false, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev);
    if (rc) return rc;
    HIPCHK(hipGetLastError());
    if (ep) {   // the next launch on this workspace continues where this one ends
      // stripe q took its items plus one past-the-end ticket per workgroup of it
      const int S = kseg_nstripes(grid);
      for (int q = 0; q < kKsegStripes; q++) {
        const unsigned nbs = q < S ? (unsigned)((nblocks - q + S - 1) / S) : 0u;
        const unsigned wgs = q < S ? (unsigned)((grid - q + S - 1) / S) : 0u;
        ep->base[q] = pa.base[q] + (unsigned)pa.nseg * nbs * (unsigned)pa.nsub + wgs;
      }
      ep->stamp = pa.stamp + (unsigned)(kMaxSeg + 1);
      ep->ready = true;
    }
  } else if (variant == CLOUDSC_VARIANT_SCC_PRIVATE) {
    if (klev > kPrivKlev) return CLOUDSC_EINVAL;    // the private arrays are sized at compile time
    if constexpr (CLOUDSC_KEEP_KERNEL(real, false, false)) {
      if (aer) launch_physics(scc_private_entry<real, true, FAST>, dim3(nblocks), dim3(nproma), 0, st, ev, a);
      else launch_physics(scc_private_entry<real, false, FAST>, dim3(nblocks), dim3(nproma), 0, st, ev, a);
    }
  } else {
    if (!scratch) return CLOUDSC_EINVAL;
    if constexpr (CLOUDSC_KEEP_KERNEL(real, false, false)) {
      SccScratch<real> s = scc_scratch_carve<real>((char*)scratch, nblocks, nproma, klev);
      if (aer) launch_physics(scc_entry<real, true, FAST>, dim3(nblocks), dim3(nproma), 0, st, ev, a, s);
      else launch_physics(scc_entry<real, false, FAST>, dim3(nblocks), dim3(nproma), 0, st, ev, a, s);
    }
  }
  if (rc) return rc;
  HIPCHK(hipGetLastError());
  return CLOUDSC_OK;
}

// fp32 runs the float-internal exp/pow unless the caller asks for the
// reference CPU build's forms (CLOUDSC_FP32_EXACT_LIBM); fp64 has only those
template <typename real>
int launch(hipStream_t st, int variant, bool exact_libm, const cloudsc_fields_t* f, int ngptot, int nproma,
           int klev, void* scratch, const void* plude_in, const ParamSet& ps, KsegEpoch* ep, const LaunchEvents* ev) {
  if constexpr (std::is_same<real, float>::value) {
    if (!exact_libm) return launch_v<real, true>(st, variant, f, ngptot, nproma, klev, scratch, plude_in, ps, ep, ev);
  }
  (void)exact_libm;
  return launch_v<real, false>(st, variant, f, ngptot, nproma, klev, scratch, plude_in, ps, ep, ev);
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI: low level
// ---------------------------------------------------------------------------
extern "C" {

int cloudsc_gpu_device_count(int* count) {
  if (!count) return CLOUDSC_EINVAL;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) { *count = 0; return hip_fail(e, "hipGetDeviceCount"); }
  *count = n;
  return CLOUDSC_OK;
}

int cloudsc_gpu_init(int device, const cloudsc_params_t* params) {
  int rc = check_params(params);
  if (rc) return rc;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n || device >= kMaxDevices)
    return CLOUDSC_ENODEV;
  HIPCHK(hipSetDevice(device));
  // The default set is overwritten in place: wait for every launch on the
  // device that may still read it (states and pipelines have their own sets).
  HIPCHK(hipDeviceSynchronize());
  std::lock_guard<std::mutex> lk(g_default_mu);
  return param_set_upload(&g_default[device], device, params);
}

long long cloudsc_gpu_scratch_bytes(int precision, int variant, int ngptot, int nproma, int klev) {
  if (ngptot <= 0 || nproma <= 0 || klev < 2) return -1;
  variant = variant_kind(variant);
  if (variant == CLOUDSC_VARIANT_KCACHE || variant == CLOUDSC_VARIANT_SCC_PRIVATE) return 0;
  if (precision != CLOUDSC_FP64 && precision != CLOUDSC_FP32) return -1;
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  if (variant == CLOUDSC_VARIANT_KSEG)
    return precision == CLOUDSC_FP64 ? kseg_scratch_bytes<double>(nblocks, nproma)
                                     : kseg_scratch_bytes<float>(nblocks, nproma);
  if (variant != CLOUDSC_VARIANT_SCC) return -1;
  return precision == CLOUDSC_FP64 ? scc_scratch_bytes<double>(nblocks, nproma, klev)
                                   : scc_scratch_bytes<float>(nblocks, nproma, klev);
}

}  // extern "C"

namespace cloudsc_impl {
int validate_run_args(int device, int precision, int variant, int ngptot, int nproma, int klev) {
  if (variant & ~(0xff | CLOUDSC_FP32_EXACT_LIBM)) return CLOUDSC_EINVAL;
  variant = variant_kind(variant);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CLOUDSC_ENODEV;
  if (device < 0 || device >= n || device >= kMaxDevices) return CLOUDSC_ENODEV;
  if (precision != CLOUDSC_FP64 && precision != CLOUDSC_FP32) return CLOUDSC_EINVAL;
  if (variant != CLOUDSC_VARIANT_KCACHE && variant != CLOUDSC_VARIANT_SCC && variant != CLOUDSC_VARIANT_KSEG &&
      variant != CLOUDSC_VARIANT_SCC_PRIVATE)
    return CLOUDSC_EINVAL;
  // KCACHE and SCC run one workgroup of nproma threads per block; KSEG runs
  // 64-column sub-blocks of any block width
  const int max_nproma = variant == CLOUDSC_VARIANT_KSEG ? (1 << 24) : 256;
  if (ngptot <= 0 || nproma <= 0 || nproma > max_nproma || klev < 2) return CLOUDSC_EINVAL;
  return CLOUDSC_OK;
}

// plude_in: NULL = in place (the reference INOUT semantics); otherwise the
// values of plude are read from there and the results written to f->plude.
// ps: the parameter set of the launch (NULL = the device's default set).
int gpu_run_impl(int device, void* stream, int precision, int variant, int ngptot, int nproma, int klev,
                 const cloudsc_fields_t* f, void* scratch, const void* plude_in, const ParamSet* ps,
                 KsegEpoch* ep, const LaunchEvents* lev) {
  const bool exact_libm = (variant & CLOUDSC_FP32_EXACT_LIBM) != 0;
  variant = variant_kind(variant);
  int rc = validate_run_args(device, precision, variant, ngptot, nproma, klev);
  if (rc) return rc;
  if (!ps) ps = device_default_params(device);
  if (!ps || !ps->dev) return CLOUDSC_ENOINIT;
  if (ps->device != device) return CLOUDSC_EINVAL;
  if (!f || !fields_complete(f)) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  return precision == CLOUDSC_FP64
             ? launch<double>(st, variant, exact_libm, f, ngptot, nproma, klev, scratch, plude_in, *ps, ep, lev)
             : launch<float>(st, variant, exact_libm, f, ngptot, nproma, klev, scratch, plude_in, *ps, ep, lev);
}

int kseg_clock(int device, void* stream, void* scratch, bool reset, double* ghz, double* seconds) {
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  unsigned long long w[2] = {0, 0};
  HIPCHK(hipMemcpy(w, (char*)scratch + kKsegClkOffset, sizeof(w), hipMemcpyDeviceToHost));
  int khz = 0;
  HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
  if (ghz) *ghz = w[1] && khz > 0 ? (double)w[0] / (double)w[1] * (double)khz * 1e-6 : 0.0;
  if (seconds) *seconds = khz > 0 ? (double)w[1] / ((double)khz * 1e3) : 0.0;
  if (reset) {
    HIPCHK(hipMemsetAsync((char*)scratch + kKsegClkOffset, 0, sizeof(w), (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  }
  return CLOUDSC_OK;
}

int kseg_check(int device, void* stream, void* scratch) {
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  unsigned w[3] = {0, 0, 0};
  HIPCHK(hipMemcpy(w, scratch, sizeof(w), hipMemcpyDeviceToHost));
  const unsigned err = w[2] == kKsegTag ? w[1] : 0u;   // no tag: no KSEG launch on this workspace yet
  if (err) {
    // on the launches' stream, and waited for: the next launch must not race it
    HIPCHK(hipMemsetAsync((unsigned*)scratch + 1, 0, sizeof(unsigned), (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    char msg[96];
    std::snprintf(msg, sizeof(msg), "KSEG: %u segment hand-offs timed out", err);
    set_error_text(msg);
    return CLOUDSC_EHANDOFF;
  }
  return CLOUDSC_OK;
}
}  // namespace cloudsc_impl

extern "C" {

int cloudsc_gpu_run(int device, void* stream, int precision, int variant, int ngptot, int nproma,
                    int klev, const cloudsc_fields_t* f, void* scratch) {
  return gpu_run_impl(device, stream, precision, variant, ngptot, nproma, klev, f, scratch, nullptr, nullptr);
}

int cloudsc_gpu_check(int device, void* stream, int variant, void* scratch) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return CLOUDSC_ENODEV;
  if (variant_kind(variant) != CLOUDSC_VARIANT_KSEG) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return CLOUDSC_OK;
  }
  if (!scratch) return CLOUDSC_EINVAL;
  return kseg_check(device, stream, scratch);
}

int cloudsc_debug_set_kseg_schedule(int nseg, int grid) {
  if (nseg < 0 || grid < 0) return CLOUDSC_EINVAL;
  g_kseg_nseg.store(nseg, std::memory_order_relaxed);
  g_kseg_grid.store(grid, std::memory_order_relaxed);
  return CLOUDSC_OK;
}

int cloudsc_debug_set_kseg_spin_limit(long long limit) {
  if (limit < 0) limit = 1LL << 24;
  g_kseg_spin_limit.store(limit > 0xffffffffLL ? 0xffffffffu : (unsigned)limit, std::memory_order_relaxed);
  return CLOUDSC_OK;
}

const char* cloudsc_strerror(int code) {
  switch (code) {
    case CLOUDSC_OK: return "success";
    case CLOUDSC_EINVAL: return "invalid argument";
    case CLOUDSC_ENODEV: return "no such HIP device";
    case CLOUDSC_EHIP: return "HIP runtime error";
    case CLOUDSC_ENOINIT: return "cloudsc_gpu_init not called for this device";
    case CLOUDSC_ENOMEM: return "out of memory";
    case CLOUDSC_EIO: return "I/O error";
    case CLOUDSC_EHANDOFF: return "KSEG segment hand-off timed out (outputs invalid)";
    default: return "unknown error";
  }
}

const char* cloudsc_last_hip_error(void) { return g_hip_err; }

#ifdef CLOUDSC_KSEG_TRACE
// diagnostic build only (tools/kseg_trace.py): per item {start, end, workgroup, xcc<<16|hw_id}
int cloudsc_kseg_trace(unsigned long long* host, int nitems) {
  if (nitems > kTraceMax) nitems = kTraceMax;
  HIPCHK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_kseg_trace), sizeof(unsigned long long) * 4 * nitems));
  return CLOUDSC_OK;
}
#endif

// Diagnostic: the single-precision exp/pow forms of the kernels on the device,
// element-wise (tests/test_gpu_parity.py measures their ulp distance).
__global__ void __launch_bounds__(256) fp32_libm_kernel(int which, const float* x, const float* y, float* out,
                                                        long long n) {
  libm_tables_to_lds<float>();
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r;
  switch (which) {
    case 0: r = cl_expf_fast(x[i]); break;
    case 1: r = cl_powf_fast(x[i], y[i]); break;
    case 2: r = cl_exp_impl(x[i]); break;
    case 3: r = cl_powr(x[i], y[i]); break;
    case 4: r = cl_divf_fast(x[i], y[i]); break;     // the fast kernels' x / y
    default: r = cl_div(x[i], y[i]); break;          // the exact kernels' x / y
  }
  out[i] = r;
}

int cloudsc_debug_fp32_libm(int device, int which, const float* x, const float* y, float* out, long long n) {
  if (which < 0 || which > 5 || !x || !out || n <= 0 || ((which & 1 || which >= 4) && !y)) return CLOUDSC_EINVAL;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return CLOUDSC_ENODEV;
  HIPCHK(hipSetDevice(device));
  float *dx = nullptr, *dy = nullptr, *dout = nullptr;
  const size_t bytes = (size_t)n * sizeof(float);
  hipError_t e = hipMalloc(&dx, bytes);
  if (e == hipSuccess) e = hipMalloc(&dy, bytes);
  if (e == hipSuccess) e = hipMalloc(&dout, bytes);
  if (e == hipSuccess) e = hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dy, y ? y : x, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(fp32_libm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, which, dx, dy,
                       dout, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(dx); (void)hipFree(dy); (void)hipFree(dout);
  if (e != hipSuccess) return hip_fail(e, "fp32 libm diagnostic");
  return CLOUDSC_OK;
}

long long cloudsc_abi_sizeof(int which) {
  switch (which) {
    case 0: return sizeof(cloudsc_params_t);
    case 1: return sizeof(cloudsc_fields_t);
    case 2: return sizeof(cloudsc_template_t);
    case 3: return sizeof(cloudsc_reference_t);
    case 4: return sizeof(cloudsc_stats_t);
    default: return -1;
  }
}

}  // extern "C"
