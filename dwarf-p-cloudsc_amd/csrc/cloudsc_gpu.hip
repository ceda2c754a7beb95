// cloudsc_gpu.hip -- libcloudsc_amd.so: the C ABI of include/cloudsc_amd.h on
// top of the hand-written CDNA4 kernels.
//
//   * parameters -> __constant__ mirrors (fp64 + fp32), one copy per device
//     (replaces the TECLDP device struct + 28 by-value scalars of
//     src/cloudsc_cuda/cloudsc/cloudsc_driver.cu:383,412-416)
//   * cloudsc_gpu_run: one launch, NPROMA block -> workgroup, column -> lane
//   * cloudsc_state_*: device-side expansion from the KLON-column template
//     (g % klon of the GLOBAL column, so shards are bit-identical to an
//     unsharded run), per-step timing with HIP events on the state's stream,
//     and device-side validation statistics against the KLON-column reference.
//
// No CPU fallback: every entry point fails with a CLOUDSC_E* code if HIP or
// the device is unavailable.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cloudsc_amd.h"
#include "cloudsc_dev.h"
#include "cloudsc_internal.h"
#include "cloudsc_kcache.h"
#include "cloudsc_scc.h"

using namespace cloudsc;
using namespace cloudsc_impl;

// ---------------------------------------------------------------------------
// __constant__ parameter mirrors
// ---------------------------------------------------------------------------
#ifdef CLOUDSC_NOINLINE_POW
__device__ __attribute__((noinline)) double cloudsc::cl_pow_ool(double x, double y) { return pow(x, y); }
__device__ __attribute__((noinline)) float cloudsc::cl_pow_ool(float x, float y) { return pow(x, y); }
#endif
__constant__ DevParams<double> g_params_dp;
__constant__ DevParams<float> g_params_sp;

namespace cloudsc_impl {
thread_local char g_hip_err[256] = "";
int hip_fail(hipError_t e, const char* what) {
  snprintf(g_hip_err, sizeof(g_hip_err), "%s: %s", what, hipGetErrorString(e));
  return CLOUDSC_EHIP;
}
void set_error_text(const char* text) { snprintf(g_hip_err, sizeof(g_hip_err), "%s", text); }
}  // namespace cloudsc_impl

namespace {

bool g_inited[kMaxDevices] = {false};
bool g_aer[kMaxDevices] = {false};      // LAERICESED || LAERICEAUTO of the device's parameters
int g_ncldtop[kMaxDevices] = {0};       // NCLDTOP of the device's parameters (KSEG segment bounds)

template <typename real>
DevParams<real> fold_params(const cloudsc_params_t& p) {
  DevParams<real> d;
  std::memset(&d, 0, sizeof(d));
#define CP(n) d.n = (real)p.n
  CP(ptsphy); CP(rg); CP(rd); CP(retv); CP(rlvtt); CP(rlstt); CP(rtt); CP(rv);
  CP(r2es); CP(r3les); CP(r3ies); CP(r4les); CP(r4ies); CP(r5les); CP(r5ies); CP(r5alvcp); CP(r5alscp);
  CP(ralvdcp); CP(ralsdcp); CP(ralfdcp); CP(rtwat); CP(rtice); CP(rtwat_rtice_r); CP(rkoop1); CP(rkoop2);
  CP(ramid); CP(rprecrhmax); CP(rtaumel); CP(ramin); CP(rlmin); CP(rlcritsnow); CP(rsnowlin2);
  CP(riceinit); CP(rvice); CP(rvrain); CP(rvsnow); CP(rthomo); CP(rcovpmin); CP(rnice); CP(rcldtopcf);
  CP(rdepliqrefrate); CP(rdepliqrefdepth); CP(rvrfactor); CP(rclcrit_sea); CP(rclcrit_land);
  CP(rcl_kkaac); CP(rcl_kkbac); CP(rcl_kkaau); CP(rcl_kkbauq); CP(rcl_kkbaun); CP(rcl_kk_cloud_num_sea);
  CP(rcl_kk_cloud_num_land); CP(rcl_const1s); CP(rcl_const7s); CP(rcl_const8s); CP(rdensref);
  CP(rcl_cdenom1); CP(rcl_cdenom2); CP(rcl_cdenom3); CP(rcl_const1r); CP(rcl_const2r); CP(rcl_const3r);
  CP(rcl_const4r); CP(rcl_fac1); CP(rcl_fac2); CP(rcl_const5r); CP(rcl_const6r); CP(rcl_fzrab);
#undef CP
  // Host folding in the working precision: the same single IEEE operation the
  // reference evaluates per point (x86-64 host float/double arithmetic is IEEE).
  const real ptsphy = (real)p.ptsphy, rg = (real)p.rg, rd = (real)p.rd, rcpd = (real)p.rcpd;
  volatile real one = (real)1.0;   // keep the compiler from re-associating
  d.zqtmst = one / ptsphy;
  d.zrdcp = rd / rcpd;
  d.zrg_r = one / rg;
  d.zrldcp = one / ((real)p.ralsdcp - (real)p.ralvdcp);
  d.zinv_tsrg = one / (ptsphy * rg);
  d.half_rg = (real)0.5 * rg;
  d.zldifdt0 = (real)p.rcldiff * ptsphy;
  d.zldifdt_conv = (real)p.rcldiff_convi * d.zldifdt0;
  d.zfaci_koop = ptsphy / (real)p.rkooptau;
  d.zzco_snow = ptsphy * (real)p.rsnowlin1;
  d.rv_rd = (real)p.rv / rd;
  d.rg_rpecons = rg * (real)p.rpecons;
  d.one_m_ramin = one - (real)p.ramin;
  d.nssopt = p.nssopt;
  d.ncldtop = p.ncldtop;
  d.laericesed = p.laericesed;
  d.laericeauto = p.laericeauto;
  return d;
}

int check_params(const cloudsc_params_t* p) {
  if (!p) return CLOUDSC_EINVAL;
  if (p->ncldtop < 2) return CLOUDSC_EINVAL;        // the physics reads level jk-1 (za, ztp1)
  if (p->nssopt < 0 || p->nssopt > 3) return CLOUDSC_EINVAL;
  if (!(p->ptsphy > 0.0)) return CLOUDSC_EINVAL;
  return CLOUDSC_OK;
}

template <typename real>
KArgs<real> make_args(const cloudsc_fields_t* f, int ngptot, int nproma, int klev) {
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
  a.ngptot = ngptot; a.nproma = nproma; a.klev = klev;
  return a;
}


// the __constant__ mirror of a precision, as a constant-address-space pointer
template <typename real> __device__ __forceinline__ cptr<DevParams<real>> dev_params();
template <> __device__ __forceinline__ cptr<DevParams<double>> dev_params<double>() {
  return (cptr<DevParams<double>>)&g_params_dp;
}
template <> __device__ __forceinline__ cptr<DevParams<float>> dev_params<float>() {
  return (cptr<DevParams<float>>)&g_params_sp;
}

}  // namespace

namespace cloudsc_impl {
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

// Kernel entry points.  The KArgs struct is the first explicit kernel argument,
// i.e. it sits at offset 0 of the kernarg segment; the bodies read it (and the
// parameter block) through constant-address-space pointers.
template <typename real, int WAVES, int PF, bool AER, bool LDSC>
__global__ void __launch_bounds__(256, WAVES) kcache_entry(const KArgs<real> a) {
  (void)a;
  libm_tables_to_lds<real>();
  cloudsc_kcache_body<real, PF, AER, LDSC>((cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr(),
                                           dev_params<real>());
}
template <typename real, int WAVES, int PF, bool AER, bool LDSC>
__global__ void __launch_bounds__(256, WAVES) kseg_entry(const KArgs<real> a, const PersistArgs<real> pa) {
  (void)a;
  libm_tables_to_lds<real>();
  cloudsc_kcache_persistent_body<real, PF, AER, LDSC>((cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr(),
                                                      dev_params<real>(), pa);
}
template <typename real, bool AER>
__global__ void __launch_bounds__(256) scc_entry(const KArgs<real> a, const SccScratch<real> s) {
  (void)a;
  libm_tables_to_lds<real>();
  cloudsc_scc_body<real, AER>((cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr(), s, dev_params<real>());
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
namespace {

template <typename real> int kcache_default_cfg();
template <> int kcache_default_cfg<double>() { return 20; }    // 2 waves/SIMD, carried state in registers
// fp32 KCACHE: 3 waves/SIMD with the register prefetch of level k+1; with the
// double-internal expf/powf it is 2-3 % faster than the 4-wave LDS-carry cfg 140
// (profiles/r01/sweep_fp32_cfgs_libm.jsonl)
template <> int kcache_default_cfg<float>() { return 31; }
template <typename real> int kseg_default_cfg();
// fp64 KSEG: 2 waves/SIMD, carried state and neighbour planes in registers
// (cfg 20).  With the streaming I/O it is 1.8 % faster than the LDS-carry cfg
// 122 (profiles/r01/sweep_kseg_cfgs_nt.jsonl), which had been 5-7 % faster
// before it (sweep_kseg_ldsc_libm.jsonl).
template <> int kseg_default_cfg<double>() { return 20; }
template <> int kseg_default_cfg<float>() { return 31; }      // 3 waves/SIMD, register prefetch


// kernel configuration code: [1]<waves><pf> -- leading 1 = carried state in LDS
#define CLOUDSC_FOR_EACH_CFG(X) \
  X(10, 1, 0, false) X(11, 1, 1, false) X(20, 2, 0, false) X(21, 2, 1, false) X(30, 3, 0, false) \
  X(31, 3, 1, false) X(40, 4, 0, false) X(41, 4, 1, false) X(120, 2, 0, true) X(121, 2, 1, true) X(122, 2, 2, true) X(130, 3, 0, true) X(132, 3, 2, true) X(22, 2, 2, false) \
  X(131, 3, 1, true) X(140, 4, 0, true)

template <typename real, bool AER>
int launch_kcache(hipStream_t st, const KArgs<real>& a, int nblocks, int nproma, int cfg) {
  switch (cfg) {
#define X(code, w, pf, ldsc)                                                                                 \
  case code:                                                                                                 \
    hipLaunchKernelGGL((kcache_entry<real, w, pf, AER, ldsc>), dim3(nblocks), dim3(nproma),                  \
                       ldsc ? carry_lds_bytes<real>(nproma) : 0, st, a);                                     \
    break;
    CLOUDSC_FOR_EACH_CFG(X)
#undef X
    default: return CLOUDSC_EINVAL;
  }
  return CLOUDSC_OK;
}

// ---- persistent segmented variant ----
// Every item is one wave: a block of NPROMA > 64 columns is run as
// ceil(NPROMA/64) 64-column sub-blocks (the block layout is unchanged: sub-block
// h is columns h*64.. of each plane of the block), so every NPROMA runs with the
// one-wave schedule that measures fastest (profiles/r01/nproma_sweep_*).
int kseg_nsub(int nproma) { return (nproma + 63) / 64; }
int kseg_wg(int nproma) { return nproma < 64 ? nproma : 64; }
// workspace: [counter, err, pad..][flags: nblocks*nsub][carry state], 256-byte aligned parts
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
size_t kseg_ctl_bytes(int nblocks, int nproma) {
  return align256(256 + (size_t)nblocks * kseg_nsub(nproma) * sizeof(unsigned));
}
template <typename real>
size_t kseg_scratch_bytes(int nblocks, int nproma) {
  return kseg_ctl_bytes(nblocks, nproma) + (size_t)nblocks * kCarryN * nproma * sizeof(real);
}

// Segmentation, measured (profiles/r01/kseg_nseg_sweep*.jsonl,
// kseg_bounds_sweep_*.jsonl), for one-wave items (2048 slots): 2 segments, the
// second one smaller ("guided": the items dequeued last are short, so the tail
// is short; lower levels also cost more per level) -- the split at NCLDTOP +
// 60 % of the physics levels (re-tuned with the streaming I/O: 1.768 ms against
// 1.788 at 62 %, profiles/r01/kseg_bounds_sweep_nt.jsonl); each hand-off costs 19 values out and in plus an
// L1 invalidate, so fewer segments win once the tail is short.  (Multi-wave
// workgroups, the earlier NPROMA > 64 form, wanted 8 even segments.)
int kseg_nseg(int nproma) {
  (void)nproma;
  int n = 2;
  if (const char* e = getenv("CLOUDSC_KSEG_NSEG")) n = atoi(e);
  return n < 1 ? 1 : (n > kMaxSeg ? kMaxSeg : n);
}

void kseg_bounds(int nseg, int klev, int ncldtop, int nproma, int* lev) {
  const int top = ncldtop - 1 < klev ? (ncldtop - 1 > 0 ? ncldtop - 1 : 0) : klev;
  const int phys = klev - top;
  lev[0] = 0;
  (void)nproma;
  if (nseg == 2) {
    lev[1] = top + (int)((60LL * phys + 50) / 100);
    if (lev[1] <= 0) lev[1] = 1;
    if (lev[1] >= klev) lev[1] = klev - 1;
  } else {
    for (int sgm = 1; sgm < nseg; sgm++) lev[sgm] = top + (int)(((long long)phys * sgm + nseg / 2) / nseg);
  }
  lev[nseg] = klev;
}

template <typename real, int WAVES, int PF, bool AER, bool LDSC>
int launch_kseg_cfg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems) {
  auto kern = kseg_entry<real, WAVES, PF, AER, LDSC>;
  const int wg = kseg_wg(nproma);
  const size_t lds = LDSC ? carry_lds_bytes<real>(wg) : 0;
  // one workgroup per resident slot (an over-estimate only delays the extra
  // workgroups: progress never depends on residency, items are dequeued in order).
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
  int grid = per_cu * ncu;
  if (const char* e = getenv("CLOUDSC_KSEG_GRID")) grid = atoi(e) > 0 ? atoi(e) : grid;
  if (grid > nitems) grid = nitems;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), lds, st, a, pa);
  return CLOUDSC_OK;
}

template <typename real, bool AER>
int launch_kseg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems,
                int cfg) {
  switch (cfg) {
#define X(code, w, pf, ldsc) \
  case code: return launch_kseg_cfg<real, w, pf, AER, ldsc>(st, a, pa, nproma, nitems);
    CLOUDSC_FOR_EACH_CFG(X)
#undef X
    default: return CLOUDSC_EINVAL;
  }
}

template <typename real>
int launch(int device, hipStream_t st, int variant, const cloudsc_fields_t* f, int ngptot, int nproma, int klev,
           void* scratch, const void* plude_in) {
  KArgs<real> a = make_args<real>(f, ngptot, nproma, klev);
  if (plude_in) a.plude_in = (const real*)plude_in;
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  const bool aer = g_aer[device];
  if (aer && (!f->pre_ice || !f->picrit_aer || !f->pnice)) return CLOUDSC_EINVAL;
  int rc = CLOUDSC_OK;
  if (variant == CLOUDSC_VARIANT_KCACHE) {
    // kernel configuration (occupancy target x load schedule); the default is
    // the measured best, CLOUDSC_KCACHE_CFG=<waves><pf> overrides it for experiments
    int cfg = kcache_default_cfg<real>();
    if (const char* e = getenv("CLOUDSC_KCACHE_CFG")) cfg = atoi(e);
    rc = aer ? launch_kcache<real, true>(st, a, nblocks, nproma, cfg)
             : launch_kcache<real, false>(st, a, nblocks, nproma, cfg);
  } else if (variant == CLOUDSC_VARIANT_KSEG) {
    if (!scratch) return CLOUDSC_EINVAL;
    int cfg = kseg_default_cfg<real>();
    if (const char* e = getenv("CLOUDSC_KCACHE_CFG")) cfg = atoi(e);
    const int ncldtop = g_ncldtop[device];
    PersistArgs<real> pa;
    pa.counter = (unsigned*)scratch;
    pa.err = (unsigned*)scratch + 1;
    pa.flags = (unsigned*)((char*)scratch + 256);
    pa.state = (real*)((char*)scratch + kseg_ctl_bytes(nblocks, nproma));
    pa.nsub = kseg_nsub(nproma);
    // item order (segment, block, sub-block); CLOUDSC_KSEG_SBMAJOR=1 runs
    // (segment, sub-block, block) instead -- the same within noise at NPROMA 128,
    // 2 % slower at 256 (profiles/r01/kseg_subblock_order.jsonl)
    pa.sb_major = 0;
    if (const char* e = getenv("CLOUDSC_KSEG_SBMAJOR")) pa.sb_major = atoi(e) != 0;
    pa.nseg = kseg_nseg(nproma);
    if (pa.nseg > klev) pa.nseg = klev;
    pa.nblocks = nblocks;
    pa.nitems = pa.nseg * nblocks * pa.nsub;
    for (int q = 0; q <= kMaxSeg; q++) pa.lev[q] = klev;
    kseg_bounds(pa.nseg, klev, ncldtop, nproma, pa.lev);
    if (const char* e = getenv("CLOUDSC_KSEG_BOUNDS")) {   // experiments: explicit interior boundaries
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
      pa.nitems = pa.nseg * nblocks * pa.nsub;
    }
    HIPCHK(hipMemsetAsync(scratch, 0, kseg_ctl_bytes(nblocks, nproma), st));
    rc = aer ? launch_kseg<real, true>(st, a, pa, nproma, pa.nitems, cfg)
             : launch_kseg<real, false>(st, a, pa, nproma, pa.nitems, cfg);
  } else {
    if (!scratch) return CLOUDSC_EINVAL;
    SccScratch<real> s = scc_scratch_carve<real>((char*)scratch, nblocks, nproma, klev);
    if (aer) hipLaunchKernelGGL((scc_entry<real, true>), dim3(nblocks), dim3(nproma), 0, st, a, s);
    else hipLaunchKernelGGL((scc_entry<real, false>), dim3(nblocks), dim3(nproma), 0, st, a, s);
  }
  if (rc) return rc;
  HIPCHK(hipGetLastError());
  return CLOUDSC_OK;
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
  const DevParams<double> dp = fold_params<double>(*params);
  const DevParams<float> sp = fold_params<float>(*params);
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_params_dp), &dp, sizeof(dp)));
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_params_sp), &sp, sizeof(sp)));
  HIPCHK(hipDeviceSynchronize());
  g_aer[device] = params->laericesed || params->laericeauto;
  g_ncldtop[device] = params->ncldtop;
  g_inited[device] = true;
  return CLOUDSC_OK;
}

long long cloudsc_gpu_scratch_bytes(int precision, int variant, int ngptot, int nproma, int klev) {
  if (variant == CLOUDSC_VARIANT_KCACHE) return 0;
  if (ngptot <= 0 || nproma <= 0 || klev < 2) return -1;
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
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CLOUDSC_ENODEV;
  if (device < 0 || device >= n || device >= kMaxDevices) return CLOUDSC_ENODEV;
  if (precision != CLOUDSC_FP64 && precision != CLOUDSC_FP32) return CLOUDSC_EINVAL;
  if (variant != CLOUDSC_VARIANT_KCACHE && variant != CLOUDSC_VARIANT_SCC && variant != CLOUDSC_VARIANT_KSEG)
    return CLOUDSC_EINVAL;
  // KCACHE and SCC run one workgroup of nproma threads per block; KSEG runs
  // 64-column sub-blocks of any block width
  const int max_nproma = variant == CLOUDSC_VARIANT_KSEG ? (1 << 24) : 256;
  if (ngptot <= 0 || nproma <= 0 || nproma > max_nproma || klev < 2) return CLOUDSC_EINVAL;
  if (!g_inited[device]) return CLOUDSC_ENOINIT;
  return CLOUDSC_OK;
}

// plude_in: NULL = in place (the reference INOUT semantics); otherwise the
// values of plude are read from there and the results written to f->plude
int gpu_run_impl(int device, void* stream, int precision, int variant, int ngptot, int nproma, int klev,
                 const cloudsc_fields_t* f, void* scratch, const void* plude_in) {
  int rc = validate_run_args(device, precision, variant, ngptot, nproma, klev);
  if (rc) return rc;
  if (!f || !fields_complete(f)) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  return precision == CLOUDSC_FP64 ? launch<double>(device, st, variant, f, ngptot, nproma, klev, scratch, plude_in)
                                   : launch<float>(device, st, variant, f, ngptot, nproma, klev, scratch, plude_in);
}
}  // namespace cloudsc_impl

extern "C" {

int cloudsc_gpu_run(int device, void* stream, int precision, int variant, int ngptot, int nproma,
                    int klev, const cloudsc_fields_t* f, void* scratch) {
  return gpu_run_impl(device, stream, precision, variant, ngptot, nproma, klev, f, scratch, nullptr);
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

