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
#include "cloudsc_kcache.h"
#include "cloudsc_scc.h"

using namespace cloudsc;

// ---------------------------------------------------------------------------
// __constant__ parameter mirrors
// ---------------------------------------------------------------------------
#ifdef CLOUDSC_NOINLINE_POW
__device__ __attribute__((noinline)) double cloudsc::cl_pow_ool(double x, double y) { return pow(x, y); }
__device__ __attribute__((noinline)) float cloudsc::cl_pow_ool(float x, float y) { return pow(x, y); }
#endif
__constant__ DevParams<double> g_params_dp;
__constant__ DevParams<float> g_params_sp;

namespace {

thread_local char g_hip_err[256] = "";
constexpr int kMaxDevices = 64;
bool g_inited[kMaxDevices] = {false};
bool g_aer[kMaxDevices] = {false};      // LAERICESED || LAERICEAUTO of the device's parameters
int g_ncldtop[kMaxDevices] = {0};       // NCLDTOP of the device's parameters (KSEG segment bounds)

int hip_fail(hipError_t e, const char* what) {
  snprintf(g_hip_err, sizeof(g_hip_err), "%s: %s", what, hipGetErrorString(e));
  return CLOUDSC_EHIP;
}
#define HIPCHK(call)                                  \
  do {                                                \
    hipError_t e_ = (call);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #call); \
  } while (0)

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

// the __constant__ mirror of a precision, as a constant-address-space pointer
template <typename real> __device__ __forceinline__ cptr<DevParams<real>> dev_params();
template <> __device__ __forceinline__ cptr<DevParams<double>> dev_params<double>() {
  return (cptr<DevParams<double>>)&g_params_dp;
}
template <> __device__ __forceinline__ cptr<DevParams<float>> dev_params<float>() {
  return (cptr<DevParams<float>>)&g_params_sp;
}

}  // namespace

// Kernel entry points.  The KArgs struct is the first explicit kernel argument,
// i.e. it sits at offset 0 of the kernarg segment; the bodies read it (and the
// parameter block) through constant-address-space pointers.
template <typename real, int WAVES, int PF, bool AER, bool LDSC>
__global__ void __launch_bounds__(256, WAVES) kcache_entry(const KArgs<real> a) {
  (void)a;
  cloudsc_kcache_body<real, PF, AER, LDSC>((cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr(),
                                           dev_params<real>());
}
template <typename real, int WAVES, int PF, bool AER, bool LDSC>
__global__ void __launch_bounds__(256, WAVES) kseg_entry(const KArgs<real> a, const PersistArgs<real> pa) {
  (void)a;
  cloudsc_kcache_persistent_body<real, PF, AER, LDSC>((cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr(),
                                                      dev_params<real>(), pa);
}
template <typename real, bool AER>
__global__ void __launch_bounds__(256) scc_entry(const KArgs<real> a, const SccScratch<real> s) {
  (void)a;
  cloudsc_scc_body<real, AER>((cptr<KArgs<real>>)__builtin_amdgcn_kernarg_segment_ptr(), s, dev_params<real>());
}

// ---------------------------------------------------------------------------
// plumbing kernels: expansion and validation statistics
// ---------------------------------------------------------------------------
// dst[b][L][i] = src[L][(col_offset + b*nproma + i) % klon], L < nlev
template <typename T, typename S>
__global__ void expand_kernel(T* __restrict__ dst, const S* __restrict__ src, int nlev, int klon,
                              int nproma, long long col_offset, long long nblocks) {
  const long long b = blockIdx.y;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nlev * nproma; e += gridDim.x * blockDim.x) {
    const int L = e / nproma, i = e - L * nproma;
    const long long g = col_offset + b * nproma + i;
    dst[(size_t)b * nlev * nproma + e] = (T)src[(size_t)L * klon + (size_t)(g % klon)];
  }
  (void)nblocks;
}

// One workgroup per NPROMA block: min/max of the field, max|d|, sum|d|, sum|ref|
// over the active lanes of that block (validate_mod.F90:136-146, with fabs).
template <typename real>
__global__ void __launch_bounds__(256) stats_kernel(const real* __restrict__ fld, const double* __restrict__ ref,
                                                    int nlev, int klon, int nproma, long long ngptot,
                                                    long long col_offset, double* __restrict__ part) {
  const long long b = blockIdx.x;
  const long long bsize = (ngptot - b * nproma) < nproma ? (ngptot - b * nproma) : nproma;
  double mn = __DBL_MAX__, mx = -__DBL_MAX__, me = 0.0, es = 0.0, rs = 0.0;
  for (int e = threadIdx.x; e < nlev * nproma; e += blockDim.x) {
    const int L = e / nproma, i = e - L * nproma;
    if (i >= bsize) continue;
    const long long g = col_offset + b * nproma + i;
    const double v = (double)fld[(size_t)b * nlev * nproma + e];
    const double r = ref[(size_t)L * klon + (size_t)(g % klon)];
    const double d = fabs(v - r);
    mn = fmin(mn, v); mx = fmax(mx, v); me = fmax(me, d); es += d; rs += fabs(r);
  }
  __shared__ double s[5][256];
  s[0][threadIdx.x] = mn; s[1][threadIdx.x] = mx; s[2][threadIdx.x] = me; s[3][threadIdx.x] = es; s[4][threadIdx.x] = rs;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const int t = threadIdx.x;
      s[0][t] = fmin(s[0][t], s[0][t + w]); s[1][t] = fmax(s[1][t], s[1][t + w]);
      s[2][t] = fmax(s[2][t], s[2][t + w]); s[3][t] += s[3][t + w]; s[4][t] += s[4][t + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int q = 0; q < 5; q++) part[b * 5 + q] = s[q][0];
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
namespace {

template <typename real> int kcache_default_cfg();
template <> int kcache_default_cfg<double>() { return 20; }    // 2 waves/SIMD, carried state in registers
template <> int kcache_default_cfg<float>() { return 140; }   // 4 waves/SIMD, carried state in LDS
template <typename real> int kseg_default_cfg();
template <> int kseg_default_cfg<double>() { return 20; }
template <> int kseg_default_cfg<float>() { return 31; }      // 3 waves/SIMD, register prefetch

int validate_run_args(int device, int precision, int variant, int ngptot, int nproma, int klev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CLOUDSC_ENODEV;
  if (device < 0 || device >= n || device >= kMaxDevices) return CLOUDSC_ENODEV;
  if (precision != CLOUDSC_FP64 && precision != CLOUDSC_FP32) return CLOUDSC_EINVAL;
  if (variant != CLOUDSC_VARIANT_KCACHE && variant != CLOUDSC_VARIANT_SCC && variant != CLOUDSC_VARIANT_KSEG)
    return CLOUDSC_EINVAL;
  if (ngptot <= 0 || nproma <= 0 || nproma > 256 || klev < 2) return CLOUDSC_EINVAL;
  if (!g_inited[device]) return CLOUDSC_ENOINIT;
  return CLOUDSC_OK;
}

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
// workspace: [counter, err, pad..][flags: nblocks][carry state], 256-byte aligned parts
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
size_t kseg_ctl_bytes(int nblocks) { return align256(256 + (size_t)nblocks * sizeof(unsigned)); }
template <typename real>
size_t kseg_scratch_bytes(int nblocks, int nproma) {
  return kseg_ctl_bytes(nblocks) + (size_t)nblocks * kCarryN * nproma * sizeof(real);
}

// Segmentation, measured (profiles/r01/kseg_nseg_sweep*.jsonl,
// kseg_bounds_sweep_*.jsonl):
//  - NPROMA > 64 (multi-wave workgroups, 1024 slots for 1280+ blocks): 8 even
//    segments of the physics levels;
//  - NPROMA <= 64 (one wave per workgroup, 2048 slots): 2 segments, the
//    second one smaller ("guided": the items dequeued last are short, so the
//    tail is short; lower levels also cost more per level) -- the split at
//    NCLDTOP + 62 % of the physics levels; each hand-off costs 19 values out
//    and in plus an L1 invalidate, so fewer segments win once the tail is short.
int kseg_nseg(int nproma) {
  int n = nproma > 64 ? 8 : 2;
  if (const char* e = getenv("CLOUDSC_KSEG_NSEG")) n = atoi(e);
  return n < 1 ? 1 : (n > kMaxSeg ? kMaxSeg : n);
}

void kseg_bounds(int nseg, int klev, int ncldtop, int nproma, int* lev) {
  const int top = ncldtop - 1 < klev ? (ncldtop - 1 > 0 ? ncldtop - 1 : 0) : klev;
  const int phys = klev - top;
  lev[0] = 0;
  if (nseg == 2 && nproma <= 64) {
    lev[1] = top + (int)((62LL * phys + 50) / 100);
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
  const size_t lds = LDSC ? carry_lds_bytes<real>(nproma) : 0;
  // one workgroup per resident slot (an over-estimate only delays the extra
  // workgroups: progress never depends on residency, items are dequeued in order).
  // Cached per NPROMA; threads driving different devices may race here, hence atomics.
  static std::atomic<int> cache[257];
  int per_cu = cache[nproma].load(std::memory_order_relaxed);
  if (!per_cu) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, nproma, lds) != hipSuccess || n <= 0) n = 1;
    per_cu = n;
    cache[nproma].store(n, std::memory_order_relaxed);
  }
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    ncu = 256;
  int grid = per_cu * ncu;
  if (const char* e = getenv("CLOUDSC_KSEG_GRID")) grid = atoi(e) > 0 ? atoi(e) : grid;
  if (grid > nitems) grid = nitems;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(nproma), lds, st, a, pa);
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
    pa.state = (real*)((char*)scratch + kseg_ctl_bytes(nblocks));
    pa.nseg = kseg_nseg(nproma);
    if (pa.nseg > klev) pa.nseg = klev;
    pa.nblocks = nblocks;
    pa.nitems = pa.nseg * nblocks;
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
      pa.nitems = pa.nseg * nblocks;
    }
    HIPCHK(hipMemsetAsync(scratch, 0, kseg_ctl_bytes(nblocks), st));
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

namespace {
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
}  // namespace

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

// ---------------------------------------------------------------------------
// C ABI: device-resident dwarf state
// ---------------------------------------------------------------------------
struct cloudsc_gpu_state {
  int device, precision, ngptot, nproma, klev, klon, nblocks;
  long long col_offset;
  size_t es;                      // element size
  hipStream_t stream;
  hipEvent_t ev0, ev1;
  cloudsc_fields_t f;             // device pointers
  void* plude_pristine;
  void* scratch;                  // SCC temporaries
  void* kseg_ws;                  // KSEG counter, flags and carried state
  std::vector<void*> allocs;
};

namespace {

size_t field_elems(const cloudsc_gpu_state* s, int kind /*0 2d,1 2dh,2 3d,3 1d*/) {
  const size_t nb = s->nblocks, np = s->nproma, kl = s->klev;
  switch (kind) {
    case 0: return nb * kl * np;
    case 1: return nb * (kl + 1) * np;
    case 2: return nb * 5 * kl * np;
    default: return nb * np;
  }
}
// validated field table: pointer slot and shape kind, in cloudsc_field_id order
void* const* valid_slot(const cloudsc_gpu_state* s, int id, int* kind) {
  const cloudsc_fields_t& f = s->f;
  static const int kinds[CLOUDSC_NVALID] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 2};
  void* const* slots[CLOUDSC_NVALID] = {
      &f.plude, &f.pcovptot, &f.prainfrac_toprfz, &f.pfsqlf, &f.pfsqif, &f.pfcqlng, &f.pfcqnng,
      &f.pfsqrf, &f.pfsqsf, &f.pfcqrng, &f.pfcqsng, &f.pfsqltur, &f.pfsqitur, &f.pfplsl, &f.pfplsn,
      &f.pfhpsl, &f.pfhpsn, &f.tendency_loc_a, &f.tendency_loc_q, &f.tendency_loc_t, &f.tendency_loc_cld};
  *kind = kinds[id];
  return slots[id];
}

int dalloc(cloudsc_gpu_state* s, void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) { hip_fail(e, "hipMalloc"); return CLOUDSC_ENOMEM; }
  s->allocs.push_back(*p);
  return CLOUDSC_OK;
}

// upload one template array and expand it into the block-layout device field
int expand_into(cloudsc_gpu_state* s, void* dst, const void* host_src, int nlev, bool is_int) {
  const size_t src_bytes = (size_t)nlev * s->klon * (is_int ? sizeof(int) : sizeof(double));
  void* d_src = nullptr;
  HIPCHK(hipMalloc(&d_src, src_bytes));
  hipError_t e = hipMemcpyAsync(d_src, host_src, src_bytes, hipMemcpyHostToDevice, s->stream);
  if (e == hipSuccess) {
    const int per = nlev * s->nproma;
    dim3 grid((per + 255) / 256, s->nblocks);
    if (is_int)
      hipLaunchKernelGGL((expand_kernel<int, int>), grid, dim3(256), 0, s->stream, (int*)dst, (const int*)d_src,
                         nlev, s->klon, s->nproma, s->col_offset, (long long)s->nblocks);
    else if (s->precision == CLOUDSC_FP64)
      hipLaunchKernelGGL((expand_kernel<double, double>), grid, dim3(256), 0, s->stream, (double*)dst,
                         (const double*)d_src, nlev, s->klon, s->nproma, s->col_offset, (long long)s->nblocks);
    else
      hipLaunchKernelGGL((expand_kernel<float, double>), grid, dim3(256), 0, s->stream, (float*)dst,
                         (const double*)d_src, nlev, s->klon, s->nproma, s->col_offset, (long long)s->nblocks);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  }
  (void)hipFree(d_src);
  if (e != hipSuccess) return hip_fail(e, "expand");
  return CLOUDSC_OK;
}

}  // namespace

extern "C" {

int cloudsc_state_create(cloudsc_gpu_state_t** out, int device, int precision, int ngptot, int nproma,
                         long long col_offset, const cloudsc_template_t* t, const cloudsc_params_t* params) {
  if (!out || !t || !params || col_offset < 0) return CLOUDSC_EINVAL;
  *out = nullptr;
  int rc = cloudsc_gpu_init(device, params);
  if (rc) return rc;
  rc = validate_run_args(device, precision, CLOUDSC_VARIANT_KCACHE, ngptot, nproma, t->klev);
  if (rc) return rc;
  if (t->klon <= 0) return CLOUDSC_EINVAL;
  const void* req[] = {t->pt, t->pq, t->tendency_tmp_t, t->tendency_tmp_q, t->tendency_tmp_a,
                       t->tendency_tmp_cld, t->pvfl, t->pvfi, t->phrsw, t->phrlw, t->pvervel, t->pap,
                       t->paph, t->plsm, t->ktype, t->plu, t->plude, t->psnde, t->pmfu, t->pmfd, t->pa,
                       t->pclv, t->psupsat};
  for (const void* q : req)
    if (!q) return CLOUDSC_EINVAL;
  if (params->laericesed && !t->pre_ice) return CLOUDSC_EINVAL;
  if (params->laericeauto && (!t->picrit_aer || !t->pnice)) return CLOUDSC_EINVAL;

  cloudsc_gpu_state* s = new cloudsc_gpu_state();
  s->device = device; s->precision = precision; s->ngptot = ngptot; s->nproma = nproma;
  s->klev = t->klev; s->klon = t->klon; s->col_offset = col_offset;
  s->nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  s->es = precision == CLOUDSC_FP64 ? sizeof(double) : sizeof(float);
  std::memset(&s->f, 0, sizeof(s->f));
  auto fail = [&](int r) { cloudsc_state_destroy(s); return r; };
  if (hipSetDevice(device) != hipSuccess) return fail(CLOUDSC_ENODEV);
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return fail(CLOUDSC_EHIP);
  if (hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess) return fail(CLOUDSC_EHIP);

  const size_t n2 = field_elems(s, 0) * s->es, n2h = field_elems(s, 1) * s->es;
  const size_t n3 = field_elems(s, 2) * s->es, n1 = field_elems(s, 3) * s->es;
  const int kl = s->klev;
  struct In { const void** dst; const void* src; int nlev; size_t bytes; bool is_int; };
  cloudsc_fields_t& f = s->f;
  void* plude_dev = nullptr;
  In ins[] = {
      {&f.pt, t->pt, kl, n2, false}, {&f.pq, t->pq, kl, n2, false},
      {&f.tendency_tmp_t, t->tendency_tmp_t, kl, n2, false}, {&f.tendency_tmp_q, t->tendency_tmp_q, kl, n2, false},
      {&f.tendency_tmp_a, t->tendency_tmp_a, kl, n2, false}, {&f.tendency_tmp_cld, t->tendency_tmp_cld, 5 * kl, n3, false},
      {&f.pvfl, t->pvfl, kl, n2, false}, {&f.pvfi, t->pvfi, kl, n2, false}, {&f.phrsw, t->phrsw, kl, n2, false},
      {&f.phrlw, t->phrlw, kl, n2, false}, {&f.pvervel, t->pvervel, kl, n2, false}, {&f.pap, t->pap, kl, n2, false},
      {&f.paph, t->paph, kl + 1, n2h, false}, {&f.plsm, t->plsm, 1, n1, false},
      {(const void**)&f.ktype, t->ktype, 1, (size_t)s->nblocks * nproma * sizeof(int), true},
      {&f.plu, t->plu, kl, n2, false}, {&f.psnde, t->psnde, kl, n2, false}, {&f.pmfu, t->pmfu, kl, n2, false},
      {&f.pmfd, t->pmfd, kl, n2, false}, {&f.pa, t->pa, kl, n2, false}, {&f.pclv, t->pclv, 5 * kl, n3, false},
      {&f.psupsat, t->psupsat, kl, n2, false},
      {&f.plcrit_aer, t->plcrit_aer, kl, n2, false}, {&f.picrit_aer, t->picrit_aer, kl, n2, false},
      {&f.pre_ice, t->pre_ice, kl, n2, false}, {&f.pccn, t->pccn, kl, n2, false}, {&f.pnice, t->pnice, kl, n2, false},
      {(const void**)&plude_dev, t->plude, kl, n2, false},
  };
  for (In& in : ins) {
    if (!in.src) continue;
    void* p = nullptr;
    if ((rc = dalloc(s, &p, in.bytes))) return fail(rc);
    if ((rc = expand_into(s, p, in.src, in.nlev, in.is_int))) return fail(rc);
    *in.dst = p;
  }
  s->plude_pristine = plude_dev;
  struct Out { void** dst; size_t bytes; };
  Out outs[] = {{&f.plude, n2}, {&f.tendency_loc_t, n2}, {&f.tendency_loc_q, n2}, {&f.tendency_loc_a, n2},
                {&f.tendency_loc_cld, n3}, {&f.pcovptot, n2}, {&f.prainfrac_toprfz, n1},
                {&f.pfsqlf, n2h}, {&f.pfsqif, n2h}, {&f.pfcqnng, n2h}, {&f.pfcqlng, n2h}, {&f.pfsqrf, n2h},
                {&f.pfsqsf, n2h}, {&f.pfcqrng, n2h}, {&f.pfcqsng, n2h}, {&f.pfsqltur, n2h}, {&f.pfsqitur, n2h},
                {&f.pfplsl, n2h}, {&f.pfplsn, n2h}, {&f.pfhpsl, n2h}, {&f.pfhpsn, n2h}};
  for (Out& o : outs) {
    if ((rc = dalloc(s, o.dst, o.bytes))) return fail(rc);
    if (hipMemsetAsync(*o.dst, 0xff, o.bytes, s->stream) != hipSuccess) return fail(CLOUDSC_EHIP);  // NaN
  }
  if (hipMemcpyAsync(f.plude, s->plude_pristine, n2, hipMemcpyDeviceToDevice, s->stream) != hipSuccess)
    return fail(CLOUDSC_EHIP);
  if (hipStreamSynchronize(s->stream) != hipSuccess) return fail(CLOUDSC_EHIP);
  *out = s;
  return CLOUDSC_OK;
}

int cloudsc_state_fields(const cloudsc_gpu_state_t* s, cloudsc_fields_t* out) {
  if (!s || !out) return CLOUDSC_EINVAL;
  *out = s->f;
  return CLOUDSC_OK;
}

int cloudsc_state_reset(cloudsc_gpu_state_t* s) {
  if (!s) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(hipMemcpyAsync(s->f.plude, s->plude_pristine, field_elems(s, 0) * s->es, hipMemcpyDeviceToDevice,
                        s->stream));
  return CLOUDSC_OK;
}

int cloudsc_state_run(cloudsc_gpu_state_t* s, int variant, int reps, float* ms) {
  if (!s || reps <= 0) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(s->device));
  void* scratch = nullptr;
  if (variant == CLOUDSC_VARIANT_SCC || variant == CLOUDSC_VARIANT_KSEG) {   // workspaces, allocated on first use
    void*& ws = variant == CLOUDSC_VARIANT_SCC ? s->scratch : s->kseg_ws;
    if (!ws) {
      const long long nb = cloudsc_gpu_scratch_bytes(s->precision, variant, s->ngptot, s->nproma, s->klev);
      if (nb <= 0) return CLOUDSC_EINVAL;
      int rc0 = dalloc(s, &ws, (size_t)nb);
      if (rc0) return rc0;
    }
    scratch = ws;
  }
  std::vector<hipEvent_t> ev(2 * (size_t)reps);
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  int rc = CLOUDSC_OK;
  for (int r = 0; r < reps && rc == CLOUDSC_OK; r++) {
    // out of place: every step reads the pristine plude and writes the INOUT
    // result to f.plude, so repeated steps see the same input with no restore copy
    HIPCHK(hipEventRecord(ev[2 * r], s->stream));
    rc = gpu_run_impl(s->device, s->stream, s->precision, variant, s->ngptot, s->nproma, s->klev, &s->f, scratch,
                      s->plude_pristine);
    HIPCHK(hipEventRecord(ev[2 * r + 1], s->stream));
  }
  hipError_t e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess && rc == CLOUDSC_OK) rc = hip_fail(e, "hipStreamSynchronize");
  for (int r = 0; r < reps && rc == CLOUDSC_OK; r++) {
    float t = 0.f;
    e = hipEventElapsedTime(&t, ev[2 * r], ev[2 * r + 1]);
    if (e != hipSuccess) rc = hip_fail(e, "hipEventElapsedTime");
    if (ms) ms[r] = t;
  }
  for (auto& x : ev) (void)hipEventDestroy(x);
  if (rc == CLOUDSC_OK && variant == CLOUDSC_VARIANT_KSEG) {
    // a segment whose predecessor never arrived gives up after a bounded spin
    // and counts itself here: its results are invalid
    unsigned err = 0;
    HIPCHK(hipMemcpy(&err, (unsigned*)scratch + 1, sizeof(err), hipMemcpyDeviceToHost));
    if (err) {
      std::snprintf(g_hip_err, sizeof(g_hip_err), "KSEG: %u segment hand-offs timed out", err);
      rc = CLOUDSC_EHIP;
    }
  }
  return rc;
}

int cloudsc_state_sync(cloudsc_gpu_state_t* s) {
  if (!s) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(hipStreamSynchronize(s->stream));
  return CLOUDSC_OK;
}

long long cloudsc_state_field_elems(const cloudsc_gpu_state_t* s, int id) {
  if (!s || id < 0 || id >= CLOUDSC_NVALID) return -1;
  int kind;
  valid_slot(s, id, &kind);
  return (long long)field_elems(s, kind);
}

int cloudsc_state_download(cloudsc_gpu_state_t* s, int id, double* host) {
  if (!s || !host || id < 0 || id >= CLOUDSC_NVALID) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(s->device));
  int kind;
  void* const* slot = valid_slot(s, id, &kind);
  const size_t n = field_elems(s, kind);
  HIPCHK(hipStreamSynchronize(s->stream));
  if (s->precision == CLOUDSC_FP64) {
    HIPCHK(hipMemcpy(host, *slot, n * sizeof(double), hipMemcpyDeviceToHost));
  } else {
    std::vector<float> tmp(n);
    HIPCHK(hipMemcpy(tmp.data(), *slot, n * sizeof(float), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++) host[i] = tmp[i];
  }
  return CLOUDSC_OK;
}

int cloudsc_state_validate(cloudsc_gpu_state_t* s, const cloudsc_reference_t* ref, cloudsc_stats_t* stats) {
  if (!s || !ref || !stats || ref->klon <= 0 || ref->klev != s->klev) return CLOUDSC_EINVAL;
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(hipStreamSynchronize(s->stream));
  double* part = nullptr;
  double* dref = nullptr;
  HIPCHK(hipMalloc(&part, (size_t)s->nblocks * 5 * sizeof(double)));
  const size_t max_ref = (size_t)5 * (s->klev + 1) * ref->klon;
  hipError_t e = hipMalloc(&dref, max_ref * sizeof(double));
  std::vector<double> h((size_t)s->nblocks * 5);
  for (int id = 0; id < CLOUDSC_NVALID && e == hipSuccess; id++) {
    int kind;
    void* const* slot = valid_slot(s, id, &kind);
    const int nlev = kind == 0 ? s->klev : kind == 1 ? s->klev + 1 : kind == 2 ? 5 * s->klev : 1;
    if (!ref->field[id]) { e = hipErrorInvalidValue; break; }
    e = hipMemcpy(dref, ref->field[id], (size_t)nlev * ref->klon * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) break;
    if (s->precision == CLOUDSC_FP64)
      hipLaunchKernelGGL(stats_kernel<double>, dim3(s->nblocks), dim3(256), 0, s->stream, (const double*)*slot,
                         dref, nlev, ref->klon, s->nproma, (long long)s->ngptot, s->col_offset, part);
    else
      hipLaunchKernelGGL(stats_kernel<float>, dim3(s->nblocks), dim3(256), 0, s->stream, (const float*)*slot,
                         dref, nlev, ref->klon, s->nproma, (long long)s->ngptot, s->col_offset, part);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess) e = hipMemcpy(h.data(), part, h.size() * sizeof(double), hipMemcpyDeviceToHost);
    if (e != hipSuccess) break;
    cloudsc_stats_t t = {__DBL_MAX__, -__DBL_MAX__, 0.0, 0.0, 0.0};
    for (int b = 0; b < s->nblocks; b++) {            // block order: deterministic
      t.minval = fmin(t.minval, h[b * 5 + 0]); t.maxval = fmax(t.maxval, h[b * 5 + 1]);
      t.maxerr = fmax(t.maxerr, h[b * 5 + 2]); t.errsum += h[b * 5 + 3]; t.refsum += h[b * 5 + 4];
    }
    stats[id] = t;
  }
  (void)hipFree(part);
  (void)hipFree(dref);
  if (e != hipSuccess) return hip_fail(e, "validate");
  return CLOUDSC_OK;
}

int cloudsc_state_destroy(cloudsc_gpu_state_t* s) {
  if (!s) return CLOUDSC_OK;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  for (void* p : s->allocs) (void)hipFree(p);
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
  return CLOUDSC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// C ABI: host-buffer pipeline
// ---------------------------------------------------------------------------
// The reference GPU drivers copy every block-layout host array to the device,
// run, and copy the outputs back (cloudsc_driver.cu:344-456; the "field"
// variant of README.md:311-330 overlaps them).  Here the blocks are cut into
// chunks of `chunk_blocks` NPROMA blocks -- one contiguous range of every
// field, because the layout is block-major -- and chunk c runs on stream
// c % nstreams: H2D of its inputs, the kernel, D2H of its outputs.  The host
// arrays are pinned in place (hipHostRegister) once, at creation.
namespace {

enum FieldKind { FK_LEVEL, FK_HALF, FK_SPECIES, FK_SURFACE };
enum FieldDir { FD_IN, FD_INOUT, FD_OUT, FD_AEROSOL };
struct FieldDesc { int kind, dir, is_int; };
// cloudsc_fields_t member order (include/cloudsc_amd.h)
constexpr FieldDesc kFieldTable[] = {
    {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_IN, 0},   {FK_SPECIES, FD_IN, 0}, {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_HALF, FD_IN, 0},    {FK_SURFACE, FD_IN, 0}, {FK_SURFACE, FD_IN, 1}, {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_SPECIES, FD_IN, 0}, {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_AEROSOL, 0}, {FK_LEVEL, FD_AEROSOL, 0}, {FK_LEVEL, FD_AEROSOL, 0},
    {FK_LEVEL, FD_AEROSOL, 0}, {FK_LEVEL, FD_AEROSOL, 0},
    {FK_LEVEL, FD_INOUT, 0},
    {FK_LEVEL, FD_OUT, 0},  {FK_LEVEL, FD_OUT, 0},  {FK_LEVEL, FD_OUT, 0},  {FK_SPECIES, FD_OUT, 0},
    {FK_LEVEL, FD_OUT, 0},  {FK_SURFACE, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0}};
constexpr int kNumFields = (int)(sizeof(kFieldTable) / sizeof(kFieldTable[0]));
static_assert(sizeof(cloudsc_fields_t) == kNumFields * sizeof(void*), "field table out of sync with the header");

size_t per_block_elems(int kind, int nproma, int klev) {
  switch (kind) {
    case FK_LEVEL: return (size_t)klev * nproma;
    case FK_HALF: return (size_t)(klev + 1) * nproma;
    case FK_SPECIES: return (size_t)CLOUDSC_NCLV * klev * nproma;
    default: return (size_t)nproma;
  }
}

}  // namespace

struct cloudsc_host_pipeline {
  int device, precision, ngptot, nproma, klev, nblocks, chunk_blocks, nstreams;
  size_t es;
  cloudsc_fields_t host;
  std::vector<void*> pinned;
  struct Slot {
    hipStream_t st = nullptr;
    cloudsc_fields_t dev{};
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    int scratch_variant = 0;
  };
  std::vector<Slot> slots;
  std::vector<void*> allocs;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

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
  void* const* hf = (void* const*)&p->host;
  // pin the caller's arrays in place (already-pinned memory is fine)
  for (int i = 0; i < kNumFields; i++) {
    if (!hf[i]) continue;
    const FieldDesc& d = kFieldTable[i];
    const size_t bytes = (size_t)p->nblocks * per_block_elems(d.kind, nproma, klev) * (d.is_int ? sizeof(int) : p->es);
    hipError_t e = hipHostRegister(hf[i], bytes, hipHostRegisterDefault);
    if (e == hipSuccess) p->pinned.push_back(hf[i]);
    else if (e != hipErrorHostMemoryAlreadyRegistered) { hip_fail(e, "hipHostRegister"); return fail(CLOUDSC_EHIP); }
    else (void)hipGetLastError();
  }
  p->slots.resize(nstreams);
  for (auto& s : p->slots) {
    if (hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking) != hipSuccess) return fail(CLOUDSC_EHIP);
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
  *out = p;
  return CLOUDSC_OK;
}

int cloudsc_host_pipeline_run(cloudsc_host_pipeline_t* p, int variant, double* ms) {
  if (!p) return CLOUDSC_EINVAL;
  int rc = validate_run_args(p->device, p->precision, variant, p->ngptot, p->nproma, p->klev);
  if (rc) return rc;
  HIPCHK(hipSetDevice(p->device));
  const int nchunks = (p->nblocks + p->chunk_blocks - 1) / p->chunk_blocks;
  // workspaces for the chunk size (SCC / KSEG), allocated on first use
  for (auto& s : p->slots) {
    if (variant == CLOUDSC_VARIANT_KCACHE || s.scratch_variant == variant) continue;
    const long long nb = cloudsc_gpu_scratch_bytes(p->precision, variant, p->chunk_blocks * p->nproma, p->nproma,
                                                   p->klev);
    if (nb <= 0) return CLOUDSC_EINVAL;
    if ((size_t)nb > s.scratch_bytes) {
      void* q = nullptr;
      if (hipMalloc(&q, (size_t)nb) != hipSuccess) return CLOUDSC_ENOMEM;
      p->allocs.push_back(q);
      s.scratch = q;
      s.scratch_bytes = (size_t)nb;
    }
    s.scratch_variant = variant;
  }
  const void* const* hf = (const void* const*)&p->host;
  // all streams start after ev0 (recorded on the null stream) and ev1 waits for all of them
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipEventRecord(p->ev0, nullptr));
  for (auto& s : p->slots) HIPCHK(hipStreamWaitEvent(s.st, p->ev0, 0));
  for (int c = 0; c < nchunks && rc == CLOUDSC_OK; c++) {
    auto& s = p->slots[c % p->nstreams];
    const int b0 = c * p->chunk_blocks;
    const int nb = (b0 + p->chunk_blocks <= p->nblocks) ? p->chunk_blocks : p->nblocks - b0;
    const long long col0 = (long long)b0 * p->nproma;
    const int ncols = (int)((col0 + (long long)nb * p->nproma <= p->ngptot) ? (long long)nb * p->nproma
                                                                            : p->ngptot - col0);
    void* const* df = (void* const*)&s.dev;
    for (int i = 0; i < kNumFields; i++) {
      const FieldDesc& d = kFieldTable[i];
      if (!hf[i] || d.dir == FD_OUT) continue;
      const size_t eb = d.is_int ? sizeof(int) : p->es;
      const size_t per = per_block_elems(d.kind, p->nproma, p->klev) * eb;
      HIPCHK(hipMemcpyAsync(df[i], (const char*)hf[i] + (size_t)b0 * per, (size_t)nb * per, hipMemcpyHostToDevice,
                            s.st));
    }
    rc = cloudsc_gpu_run(p->device, s.st, p->precision, variant, ncols, p->nproma, p->klev, &s.dev, s.scratch);
    if (rc) break;
    for (int i = 0; i < kNumFields; i++) {
      const FieldDesc& d = kFieldTable[i];
      if (!hf[i] || !(d.dir == FD_OUT || d.dir == FD_INOUT)) continue;
      const size_t per = per_block_elems(d.kind, p->nproma, p->klev) * p->es;
      HIPCHK(hipMemcpyAsync((char*)hf[i] + (size_t)b0 * per, df[i], (size_t)nb * per, hipMemcpyDeviceToHost, s.st));
    }
  }
  for (auto& s : p->slots) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e, s.st));
    HIPCHK(hipStreamWaitEvent(nullptr, e, 0));
    (void)hipEventDestroy(e);
  }
  HIPCHK(hipEventRecord(p->ev1, nullptr));
  HIPCHK(hipEventSynchronize(p->ev1));
  if (rc) return rc;
  float t = 0.f;
  HIPCHK(hipEventElapsedTime(&t, p->ev0, p->ev1));
  if (ms) *ms = t;
  return CLOUDSC_OK;
}

int cloudsc_host_pipeline_destroy(cloudsc_host_pipeline_t* p) {
  if (!p) return CLOUDSC_EINVAL;
  (void)hipSetDevice(p->device);
  for (auto& s : p->slots)
    if (s.st) { (void)hipStreamSynchronize(s.st); (void)hipStreamDestroy(s.st); }
  for (void* q : p->allocs) (void)hipFree(q);
  for (void* h : p->pinned) (void)hipHostUnregister(h);
  if (p->ev0) (void)hipEventDestroy(p->ev0);
  if (p->ev1) (void)hipEventDestroy(p->ev1);
  delete p;
  return CLOUDSC_OK;
}

}  // extern "C"
