// cloudsc_dev.h -- device-side parameter block and thermodynamic helpers shared
// by the CLOUDSC kernels (k-caching and SCC) for CDNA4 / gfx950.
//
// The YOMCST / YOETHF constants and the TECLDP tuning parameters the kernel
// reads (reference: src/cloudsc_c/cloudsc/{yomcst_c,yoethf_c,yoecldp_c}.h) live
// in a device-memory block per parameter set, one mirror per precision, passed
// to every launch by pointer and read through the constant address space:
// uniform across the grid, so every access is a scalar (s_load) read.  A few derived constants that the
// reference recomputes per point (1/PTSPHY, RD/RCPD, 1/(PTSPHY*RG), ...) are
// folded on the host with the SAME IEEE operation, so results do not change.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "cloudsc_libm.h"

namespace cloudsc {

#if !defined(__HIP_DEVICE_COMPILE__)
// host pass: the float overloads of the C math functions the phase functions
// call (in the device pass the HIP device library's overloads are used)
using std::copysign;
using std::fabs;
using std::fmax;
using std::fmin;
using std::sqrt;
#endif

template <typename real>
struct DevParams {
  // YOMCST / YOETHF
  real ptsphy, rg, rd, retv, rlvtt, rlstt, rtt, rv;
  real r2es, r3les, r3ies, r4les, r4ies, r5les, r5ies, r5alvcp, r5alscp;
  real ralvdcp, ralsdcp, ralfdcp, rtwat, rtice, rtwat_rtice_r, rkoop1, rkoop2;
  // TECLDP (subset the kernel reads)
  real ramid, rprecrhmax, rtaumel, ramin, rlmin, rlcritsnow, rsnowlin2;
  real riceinit, rvice, rvrain, rvsnow, rthomo, rcovpmin, rnice, rcldtopcf, rdepliqrefrate;
  real rdepliqrefdepth, rvrfactor, rclcrit_sea, rclcrit_land;
  real rcl_kkaac, rcl_kkbac, rcl_kkaau, rcl_kkbauq, rcl_kkbaun, rcl_kk_cloud_num_sea, rcl_kk_cloud_num_land;
  real rcl_const1s, rcl_const7s, rcl_const8s, rdensref, rcl_cdenom1, rcl_cdenom2, rcl_cdenom3;
  real rcl_const1r, rcl_const2r, rcl_const3r, rcl_const4r, rcl_fac1, rcl_fac2, rcl_const5r, rcl_const6r;
  real rcl_fzrab;
  // host-folded (each is exactly the reference's own expression, evaluated once)
  real zqtmst;        // 1/ptsphy                       cloudsc_c.c:385
  real zrdcp;         // rd/rcpd                        :387
  real zrg_r;         // 1/rg                           :390
  real zrldcp;        // 1/(ralsdcp-ralvdcp)            :391
  real zinv_tsrg;     // 1/(ptsphy*rg)                  :807
  real half_rg;       // 0.5*rg                         :1146
  real zldifdt0;      // rcldiff*ptsphy                 :1088
  real zldifdt_conv;  // rcldiff_convi*(rcldiff*ptsphy) :1091
  real zfaci_koop;    // ptsphy/rkooptau                :889
  real zzco_snow;     // ptsphy*rsnowlin1               :1624
  real rv_rd;         // rv/rd                          :2011
  real rg_rpecons;    // rg*rpecons                     :2065
  real one_m_ramin;   // 1-ramin                        :898
  // host reciprocals RN(1/d) of the parameters the kernel divides by: cl_div(n, {d, RN(1/d)}) is n/d (below)
  real rd_rcp, rtaumel_rcp, rdepliqrefdepth_rcp, rvrfactor_rcp;
  int nssopt, ncldtop, laericesed, laericeauto;
};

// The parameter block as the kernels see it: the same memory, with the choice
// of the single-precision exp/pow forms carried in the type (FAST = the
// float-internal device forms below; false = the reference CPU build's
// algorithms).  The phase functions take the block as `const P& c` and pass it
// to cl_exp / cl_pow, so the choice costs nothing at run time.  fp64 is always
// the reference's algorithms (FAST is only instantiated for float).
// VREG: the block copied into VGPRs for the level loop (fp32 k-caching kernels,
// kcache_levels) instead of being read with a scalar load at each use.
template <typename real, bool FAST, bool VREG = false>
struct DevParamsT : DevParams<real> {};
template <typename P>
struct LibmFast {
  static constexpr bool value = false;
};
template <bool VREG>
struct LibmFast<DevParamsT<float, true, VREG>> {
  static constexpr bool value = true;
};
template <typename P>
struct ParamsInVgprs {
  static constexpr bool value = false;
};
template <typename real, bool FAST>
struct ParamsInVgprs<DevParamsT<real, FAST, true>> {
  static constexpr bool value = true;
};
template <typename P>
struct WithVgprParams;
template <typename real, bool FAST, bool VREG>
struct WithVgprParams<DevParamsT<real, FAST, VREG>> {
  using type = DevParamsT<real, FAST, true>;
};

// The phase functions of the physics (cloudsc_kcache.h) and the helpers below
// compile for the device (the kernels) and for the host (cloudsc_cpu_run,
// cloudsc_cpu.hip: the same source as the explicitly selected CPU variant).
// The few helpers whose device form is target-specific (register laundering,
// the reciprocal-based division, the LDS-table exp/pow) have a plain host form
// selected on __HIP_DEVICE_COMPILE__; both forms round identically.
#define CLOUDSC_HD __host__ __device__ __forceinline__

// Address-space-4 (constant) pointer: loads through it are scalar (s_load).
#define CLOUDSC_AS4 __attribute__((address_space(4)))
template <typename T>
using cptr = const CLOUDSC_AS4 T*;

// Hide a uniform constant-space pointer from the optimiser.  The ~90 parameters
// and ~45 field base pointers are all uniform and read with scalar loads; left
// alone, LLVM hoists every one of them out of the 137-level loop, runs out of
// SGPRs and spills them into VGPR lanes (v_writelane/v_readlane), or keeps
// per-field 64-bit VGPR pointers alive (~90 VGPRs).  Laundering the address once
// per level (or per phase) keeps each scalar load next to its use -- a scalar
// cache hit -- at no register cost.
template <typename T>
__device__ __forceinline__ cptr<T> launder_uniform(cptr<T> p) {
  asm volatile("" : "+s"(p));
  return p;
}
// A parameter value materialised as a value (scalar register) at this point.
// Without it, `cond ? c.a : c.b` and `x = c.a; if (flag) x = v;` are turned
// into ONE load through a selected address -- a per-lane (vector, or flat via
// a stack slot) load with a full memory wait inside the level loop.
template <typename T>
CLOUDSC_HD T sval(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(v));
#endif
  return v;
}
// sval for a parameter of the block `c`: a no-op when the block already lives
// in VGPRs (an SGPR constraint on a VGPR value would be an illegal copy)
template <typename P, typename T>
CLOUDSC_HD T pval(const P&, T v) {
  if constexpr (ParamsInVgprs<P>::value) return v;
  else return sval(v);
}
template <typename T>
CLOUDSC_HD T launder_vgpr(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(v));
#endif
  return v;
}

// Real-typed literal: R(0.5) is a double for fp64 and a float for fp32
// (the JPRB=sp semantics, parkind1.F90:40-43).
#define R(x) (real)(x)

// Device math used by the kernels.
//
// fp64 exp/pow: the reference CPU build's own algorithms (cloudsc_libm.h),
// so that the GPU rounds every exp/pow exactly as the reference kernel does.
// Their tables (5 KB) are copied from __constant__ memory into LDS at the start
// of every physics kernel (libm_tables_to_lds) and read there with per-lane
// indices: one ds_read_b128 per exp, b128 + b64 per log of a pow.  A table
// read from global memory instead would be counted by vmcnt, and waiting for
// it inside a physics branch would drain the software-pipelined level loads
// (vmcnt(0)); LDS reads are counted by lgkmcnt.
__constant__ __attribute__((aligned(16))) unsigned long long g_cl_exp_tab[2 * 128] = {CLOUDSC_LIBM_EXP_TAB};
__constant__ __attribute__((aligned(16))) double g_cl_log_tab[4 * 128] = {CLOUDSC_LIBM_LOG_TAB};
typedef unsigned long long cl_u64x2 __attribute__((ext_vector_type(2)));
typedef double cl_f64x2 __attribute__((ext_vector_type(2)));
__shared__ cl_u64x2 s_cl_exp_tab[128];       // {tail, sbits}
__shared__ cl_f64x2 s_cl_log_tab[128];       // {invc, logc}
__shared__ double s_cl_logtail_tab[128];     // logctail
// the addends of the polynomials' two-constant fmas: {C4, C2} of exp, {A5, A3, A1, -} of log.
// Read from LDS (one ds_read_b128 per exp, two per log), they arrive in VGPRs without VALU
// moves; a VOP3 fma reads at most one scalar and no literal, so one of the two constants of
// fma(r, C5, C4) has to come from a VGPR.  (The plain exp table read is already waited for
// right there, so the extra LDS latency hides under it.)
__shared__ cl_f64x2 s_cl_poly[3];
// single precision (expf/powf): 32 x 2^(i/32) bits, 16 x {invc, logc}
__constant__ __attribute__((aligned(16))) unsigned long long g_cl_exp2f_tab[32] = {CLOUDSC_LIBM_EXP2F_TAB};
__constant__ __attribute__((aligned(16))) double g_cl_powf_tab[2 * 16] = {CLOUDSC_LIBM_POWF_LOG2_TAB};
__shared__ unsigned long long s_cl_exp2f_tab[32];
__shared__ cl_f64x2 s_cl_powf_tab[16];
struct LdsLibmTabsF {
  __device__ __forceinline__ uint64_t exp2f_entry(uint32_t i) const { return s_cl_exp2f_tab[i]; }
  __device__ __forceinline__ void powf_log2_entry(uint32_t i, double* invc, double* logc) const {
    const cl_f64x2 a = s_cl_powf_tab[i];
    *invc = a.x;
    *logc = a.y;
  }
};
struct ConstLibmTabsF {
  __device__ __forceinline__ uint64_t exp2f_entry(uint32_t i) const { return g_cl_exp2f_tab[i]; }
  __device__ __forceinline__ void powf_log2_entry(uint32_t i, double* invc, double* logc) const {
    *invc = g_cl_powf_tab[2 * i];
    *logc = g_cl_powf_tab[2 * i + 1];
  }
};
struct LdsLibmTabs {
  __device__ __forceinline__ cloudsc_libm::ExpAddends exp_addends() const {
    const cl_f64x2 a = s_cl_poly[0];
    return {a.x, a.y};
  }
  __device__ __forceinline__ cloudsc_libm::LogAddends log_addends() const {
    const cl_f64x2 a = s_cl_poly[1], b = s_cl_poly[2];
    return {a.x, a.y, b.x};
  }
  __device__ __forceinline__ cloudsc_libm::ExpEntry exp_entry(uint32_t k) const {
    const cl_u64x2 e = s_cl_exp_tab[k];
    return {e.x, e.y};
  }
  __device__ __forceinline__ cloudsc_libm::LogEntry log_entry(uint32_t i) const {
    const cl_f64x2 a = s_cl_log_tab[i];
    return {a.x, a.y, s_cl_logtail_tab[i]};
  }
};
// The complete functions, out of line, for the arguments outside the hot
// range (tables from __constant__ memory; never taken by CLOUDSC's data).
struct ConstLibmTabs {
  __device__ __forceinline__ cloudsc_libm::ExpAddends exp_addends() const {
    return {cloudsc_libm::kC4, cloudsc_libm::kC2};
  }
  __device__ __forceinline__ cloudsc_libm::LogAddends log_addends() const {
    return {cloudsc_libm::kA5, cloudsc_libm::kA3, cloudsc_libm::kA1};
  }
  __device__ __forceinline__ cloudsc_libm::ExpEntry exp_entry(uint32_t k) const {
    const cl_u64x2 e = ((const cl_u64x2*)g_cl_exp_tab)[k];
    return {e.x, e.y};
  }
  __device__ __forceinline__ cloudsc_libm::LogEntry log_entry(uint32_t i) const {
    const cl_f64x2 a = ((const cl_f64x2*)g_cl_log_tab)[2 * i];
    return {a.x, a.y, g_cl_log_tab[4 * i + 2]};
  }
};
// (inlining them at every call site measured +35 % kernel time: code size and
// register pressure)
#define CLOUDSC_LIBM_COLD_ATTR __noinline__ __attribute__((pure))
__device__ CLOUDSC_LIBM_COLD_ATTR double cl_exp_cold(double x) { return cloudsc_libm::exp(x, ConstLibmTabs{}); }
__device__ CLOUDSC_LIBM_COLD_ATTR double cl_pow_cold(double x, double y) { return cloudsc_libm::pow(x, y, ConstLibmTabs{}); }
__device__ CLOUDSC_LIBM_COLD_ATTR float cl_expf_cold(float x) { return cloudsc_libm::expf(x, ConstLibmTabsF{}); }
__device__ CLOUDSC_LIBM_COLD_ATTR float cl_powf_cold(float x, float y) {
  return cloudsc_libm::powf(x, y, ConstLibmTabsF{});
}
struct DevLibmCold {
  __device__ __forceinline__ double exp(double x) const { return cl_exp_cold(x); }
  __device__ __forceinline__ double pow(double x, double y) const { return cl_pow_cold(x, y); }
  __device__ __forceinline__ float expf(float x) const { return cl_expf_cold(x); }
  __device__ __forceinline__ float powf(float x, float y) const { return cl_powf_cold(x, y); }
};
// Every thread of the workgroup must call this before the physics (it ends in
// a barrier).
template <typename real>
__device__ __forceinline__ void libm_tables_to_lds() {
  if constexpr (std::is_same<real, double>::value) {
    for (int i = threadIdx.x; i < 128; i += blockDim.x) {
      s_cl_exp_tab[i] = ((const cl_u64x2*)g_cl_exp_tab)[i];
      s_cl_log_tab[i] = ((const cl_f64x2*)g_cl_log_tab)[2 * i];
      s_cl_logtail_tab[i] = g_cl_log_tab[4 * i + 2];
    }
    if (threadIdx.x == 0) {
      s_cl_poly[0] = cl_f64x2{cloudsc_libm::kC4, cloudsc_libm::kC2};
      s_cl_poly[1] = cl_f64x2{cloudsc_libm::kA5, cloudsc_libm::kA3};
      s_cl_poly[2] = cl_f64x2{cloudsc_libm::kA1, 0.0};
    }
    __syncthreads();
  } else {
    for (int i = threadIdx.x; i < 32; i += blockDim.x) {
      s_cl_exp2f_tab[i] = g_cl_exp2f_tab[i];
      if (i < 16) s_cl_powf_tab[i] = ((const cl_f64x2*)g_cl_powf_tab)[i];
    }
    __syncthreads();
  }
}

// pow is only ever applied to non-negative bases here (densities, ratios of
// positive quantities, temperatures, slope parameters): the hot path of
// cloudsc_libm::pow_split handles exactly those, everything else goes to the
// complete out-of-line function.
__device__ __forceinline__ double cl_powr(double x, double y) {
  return cloudsc_libm::pow_split(x, y, LdsLibmTabs{}, DevLibmCold{});
}
__device__ __forceinline__ float cl_powr(float x, float y) {
  return cloudsc_libm::powf_split(x, y, LdsLibmTabsF{}, DevLibmCold{});
}
__device__ __forceinline__ double cl_exp_impl(double x) { return cloudsc_libm::exp_split(x, LdsLibmTabs{}, DevLibmCold{}); }
__device__ __forceinline__ float cl_exp_impl(float x) { return cloudsc_libm::expf_split(x, LdsLibmTabsF{}, DevLibmCold{}); }
// host forms: the same algorithms with the tables read from host memory
struct HostLibmCold {
  double exp(double x) const { return cloudsc_libm::exp(x, cloudsc_libm::HostTabs{}); }
  double pow(double x, double y) const { return cloudsc_libm::pow(x, y, cloudsc_libm::HostTabs{}); }
  float expf(float x) const { return cloudsc_libm::expf(x, cloudsc_libm::HostTabsF{}); }
  float powf(float x, float y) const { return cloudsc_libm::powf(x, y, cloudsc_libm::HostTabsF{}); }
};
inline double cl_powr_host(double x, double y) {
  return cloudsc_libm::pow_split(x, y, cloudsc_libm::HostTabs{}, HostLibmCold{});
}
inline float cl_powr_host(float x, float y) {
  return cloudsc_libm::powf_split(x, y, cloudsc_libm::HostTabsF{}, HostLibmCold{});
}
inline double cl_exp_host(double x) { return cloudsc_libm::exp_split(x, cloudsc_libm::HostTabs{}, HostLibmCold{}); }
inline float cl_exp_host(float x) { return cloudsc_libm::expf_split(x, cloudsc_libm::HostTabsF{}, HostLibmCold{}); }
// Single precision, float-internal (CLOUDSC_FP32 default; the glibc forms
// above with CLOUDSC_FP32_EXACT_LIBM).  expf: x*log2(e) as an exact
// head + tail (Cody-Waite with an fma), the hardware 2^f (v_exp_f32, 1 ulp on
// |f| <= 1/2) and ldexp.  powf: log2 of the mantissa in [1/2, 1) by the
// hardware log2 (v_log_f32) plus the exponent as a float-float (Fast2Sum),
// y*log2(x) as a float-float (one product split with fma), then the same
// exp2 + ldexp (about 20 operations, was 30 with a full TwoSum of two split
// products; same accuracy, -0.3 % fp32 KSEG: the pow sites sit in branches most
// waves skip, profiles/r03/experiment_fp32_powf_fast2sum_ab.txt).  Every
// operation is float (2-cycle issue on gfx950, against 4 for the double
// internals of glibc's forms).  No out-of-line calls: the special cases are
// branch-free (expf: the argument clamped to [-104, 89], where ldexp over- and
// underflows to +inf / 0 as expf does, NaN passed through; powf: the exponent
// clamped likewise, a zero or infinite base gives 0 or +inf) -- a call site in the level
// loop costs the register allocation 5 % of the fp32 kernel time even when it
// is never taken (profiles/r03/experiment_fp32_nocold_ab.txt).  Accuracy:
// tests/test_gpu_parity.py (test_fp32_fast_libm_ulp) measures <= 2 ulp against
// the glibc forms over the argument ranges CLOUDSC uses.
__device__ __forceinline__ float cl_expf_fast(float x0) {
  // |x| clamped: e^89 overflows to +inf and e^-104 underflows to 0 through ldexp as they should
  const float x = __builtin_fminf(__builtin_fmaxf(x0, -104.0f), 89.0f);
  const float kL2e = 0x1.715476p+0f, kL2eLo = 0x1.4ae0bep-26f;   // log2(e) = kL2e + kL2eLo (+ O(2^-50))
  const float ph = x * kL2e;
  float pl = __builtin_fmaf(x, kL2e, -ph);                         // exact: x*kL2e = ph + pl
  pl = __builtin_fmaf(x, kL2eLo, pl);
  const float e = __builtin_rintf(ph);
  const float f = (ph - e) + pl;                                    // |f| <= 1/2 + tiny
  const float r = __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f), (int)e);
  return x0 != x0 ? x0 : r;                                         // NaN stays NaN
}
__device__ __forceinline__ float cl_powf_fast(float x, float y) {
  const float m = __builtin_amdgcn_frexp_mantf(x);                 // x = m * 2^E, m in [1/2, 1)
  const float E = (float)__builtin_amdgcn_frexp_expf(x);
  const float l = __builtin_amdgcn_logf(m);                         // log2(m), in [-1, 0)
  const float t = E + l, t_lo = l - (t - E);                        // Fast2Sum (|E| >= |l| or E == 0): E + l = t + t_lo
  const float p = y * t;
  const float p_lo = __builtin_fmaf(y, t_lo, __builtin_fmaf(y, t, -p));   // y*(t + t_lo) = p + p_lo (+ O(2^-48 p))
  // k clamped (NaN -> -256): ldexp over- and underflows from there, and the conversion is always defined
  const float k = __builtin_fminf(__builtin_fmaxf(__builtin_rintf(p), -256.0f), 256.0f);
  const float r = __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f((p - k) + p_lo), (int)k);
  // x == 0 (log2 -inf) or +inf: p = +-inf, pow is +inf or 0 (CLOUDSC: bases >= 0); NaN in, NaN out through r
  return __builtin_isinf(p) ? (p > 0.0f ? __builtin_inff() : 0.0f) : r;
}

template <typename real>
CLOUDSC_HD real cl_pow(real x, real y) {
#if defined(__HIP_DEVICE_COMPILE__)
  return cl_powr(x, y);
#else
  return cl_powr_host(x, y);
#endif
}
template <typename real>
CLOUDSC_HD real cl_exp(real x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return cl_exp_impl(x);
#else
  return cl_exp_host(x);
#endif
}
// the physics' exp / pow: the form is chosen by the parameter block's type
template <typename real, typename P>
CLOUDSC_HD real cl_exp(const P&, typename std::common_type<real>::type x) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return cl_expf_fast(x);
#endif
  return cl_exp<real>(x);
}
template <typename real, typename P>
CLOUDSC_HD real cl_pow(const P&, typename std::common_type<real>::type x, typename std::common_type<real>::type y) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return cl_powf_fast(x, y);
#endif
  return cl_pow<real>(x, y);
}

// Division.  The IEEE sequence hipcc emits for a / b is
//   div_scale(b), div_scale(a), rcp, 2 Newton steps (fp64; 1 in fp32), q = a*r,
//   residual fma, div_fmas (= fma(residual, r, q) unless div_scale rescaled),
//   div_fixup (inf / nan / zero operands)
// -- 11 instructions.  cl_div is the same arithmetic without the range
// scaling and the special-case fix-up: 8 instructions, and the reciprocal of a
// repeated divisor is shared (CSE).  div_scale only rescales operands whose
// exponents are near the ends of the range (quotient or divisor beyond about
// 2^+-1000, denormals), and the fix-up only changes non-finite or zero
// divisors, so for every finite, normal-range operand pair the result is
// bit-identical to a / b (correctly rounded).  CLOUDSC's divisions are all
// guarded (divisors are max(x, eps), 1 + positive sums, or branch-protected
// ratios of physical quantities), and the A/B identity check
// (tools/ab_compare.py: reference state, scenarios, random perturbations,
// NSSOPT, aerosol flags, fp32, 163840 columns) confirms identical output bits.
CLOUDSC_HD double cl_div(double n, double d) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return n / d;       // host: the IEEE division itself
#else
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = n * r;
  const double rem = __builtin_fma(-d, q, n);
  return __builtin_fma(rem, r, q);
#endif
}
CLOUDSC_HD float cl_div(float n, float d) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return n / d;
#else
  float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  r = __builtin_fmaf(e, r, r);
  float q = n * r;
  float rem = __builtin_fmaf(-d, q, n);
  q = __builtin_fmaf(rem, r, q);
  rem = __builtin_fmaf(-d, q, n);
  return __builtin_fmaf(rem, r, q);
#endif
}
// A divisor together with its refined reciprocal, for divisions that share a
// divisor: cl_div(n, cl_recip(d)) runs exactly the steps of cl_div(n, d) with
// the same reciprocal r, so the quotient is bit-identical -- the reciprocal
// (v_rcp + its Newton steps) is computed once instead of once per division.
template <typename real>
struct Recip {
  real d, r;
};
CLOUDSC_HD Recip<double> cl_recip(double d) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return {d, 0.0};      // host: the divisions below use d itself
#else
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  return {d, r};
#endif
}
CLOUDSC_HD Recip<float> cl_recip(float d) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return {d, 0.0f};
#else
  float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  r = __builtin_fmaf(e, r, r);
  return {d, r};
#endif
}
CLOUDSC_HD double cl_div(double n, const Recip<double>& rd) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return n / rd.d;
#else
  const double q = n * rd.r;
  const double rem = __builtin_fma(-rd.d, q, n);
  return __builtin_fma(rem, rd.r, q);
#endif
}
CLOUDSC_HD float cl_div(float n, const Recip<float>& rd) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return n / rd.d;
#else
  float q = n * rd.r;
  float rem = __builtin_fmaf(-rd.d, q, n);
  q = __builtin_fmaf(rem, rd.r, q);
  rem = __builtin_fmaf(-rd.d, q, n);
  return __builtin_fmaf(rem, rd.r, q);
#endif
}
// A divisor known before the launch -- a parameter (its RN(1/d) folded on the
// host, DevParams::*_rcp) or a literal (folded by the compiler): the division
// is the correction step alone (fp64: mul + 2 fma instead of 8 instructions
// with the quarter-rate v_rcp).  With r = RN(1/d) the corrected quotient is
// n/d correctly rounded (Markstein's theorem; tools/div_const_check.c: 0
// mismatches over 1.4e8 numerators for CLOUDSC's divisors, and 1000 random
// divisors, in fp64 and fp32).
// (real is deduced from the divisor; the numerator converts, e.g. from an LDS-carried value)
template <typename real>
CLOUDSC_HD real cl_div_known(typename std::common_type<real>::type n, real d, real rcp_d) {
  return cl_div(n, Recip<real>{d, rcp_d});
}
template <typename real>
CLOUDSC_HD real cl_div_lit(typename std::common_type<real>::type n, real d) {
  return cl_div(n, Recip<real>{d, real(1) / d});
}
// explicit-precision form, cl_div<real>(a, b)
template <typename real>
CLOUDSC_HD real cl_div(typename std::common_type<real>::type n, typename std::common_type<real>::type d) {
  return cl_div(static_cast<real>(n), static_cast<real>(d));
}

// The physics' divisions: cl_div_p<real>(c, n, d), the form chosen by the
// parameter block's type like cl_exp / cl_pow.  fp32 FAST kernels (the
// CLOUDSC_FP32 default, tolerance-gated like the float-internal expf/powf):
// v_rcp_f32 (1 ulp) and ONE residual correction,
//   q0 = n*r,  q = fma(fma(-d, q0, n), r, q0)
// -- the reciprocal + 3 operations instead of + 7 (cl_div's Newton-refined
// reciprocal and two corrections, which make every quotient the IEEE one).
// The correction leaves q within 1 ulp of n/d (almost always the IEEE
// quotient).  fp64 and the exact fp32 forms (CLOUDSC_FP32_EXACT_LIBM) are cl_div.
// Valid range of the fast forms (no div_scale / div_fixup): a divisor with
// 2^-126 <= |d| < 2^126 (a normal float whose reciprocal is normal) and a
// quotient that is finite and normal; then 0/d = 0 exactly and every other
// quotient is within 1 ulp.  A smaller |d| makes v_rcp_f32 overflow, so the
// result is NaN (0/d) or inf/NaN where IEEE gives a finite value; zero and
// non-finite divisors give NaN.  Every division of the physics has a divisor in
// that range: max(x, epsilon) clamps, 1 + positive sums, temperatures and
// pressures (tests/test_gpu_parity.py::test_fp32_fast_division_range checks
// the contract and the out-of-range behaviour on the device).
__device__ __forceinline__ float cl_divf_fast(float n, float d) {
  const float r = __builtin_amdgcn_rcpf(d), q = n * r;
  return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
}
template <typename real, typename P>
CLOUDSC_HD real cl_div_p(const P&, typename std::common_type<real>::type n, typename std::common_type<real>::type d) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return cl_divf_fast(n, d);
#endif
  return cl_div(static_cast<real>(n), static_cast<real>(d));
}
template <typename real, typename P>
CLOUDSC_HD Recip<real> cl_recip_p(const P&, typename std::common_type<real>::type d) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return {d, __builtin_amdgcn_rcpf(d)};
#endif
  return cl_recip(static_cast<real>(d));
}
template <typename real, typename P>
CLOUDSC_HD real cl_div_p(const P&, typename std::common_type<real>::type n, const Recip<real>& rd) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) {
    const float q = n * rd.r;
    return __builtin_fmaf(__builtin_fmaf(-rd.d, q, n), rd.r, q);
  }
#endif
  return cl_div(static_cast<real>(n), rd);
}
// a known divisor with its RN(1/d): the FAST form is one multiply by it (within
// 1.5 ulp), the exact one cl_div's correction steps (the IEEE quotient); the
// FAST square root is v_sqrt_f32 (1 ulp) instead of the correctly rounded
// sequence (-0.6 % fp32, profiles/r03/experiment_fp32_sqrt_known_div_ab.txt)
template <typename real, typename P>
CLOUDSC_HD real cl_div_known_p(const P& c, typename std::common_type<real>::type n, real d, real rcp_d) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return n * rcp_d;
#endif
  return cl_div_p<real>(c, n, Recip<real>{d, rcp_d});
}
template <typename real, typename P>
CLOUDSC_HD real cl_sqrt_p(const P&, typename std::common_type<real>::type x) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return __builtin_amdgcn_sqrtf(x);
#endif
  return sqrt(x);
}
template <typename real, typename P>
CLOUDSC_HD real cl_div_lit_p(const P& c, typename std::common_type<real>::type n, real d) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return n * (real(1) / d);
#endif
  return cl_div_p<real>(c, n, Recip<real>{d, real(1) / d});
}

// FOEALFA (src/common/include/fcttre.func.h; inlined at cloudsc_c.c:588,831,1162-1174)
template <typename real, typename P>
CLOUDSC_HD real foealfa(const P& c, real t) {
  real x = (fmax(c.rtice, fmin(c.rtwat, t)) - c.rtice) * c.rtwat_rtice_r;
  return fmin(R(1.0), x * x);            // pow(x,2) == x*x (both rounded once)
}
template <typename real, typename P>
CLOUDSC_HD real exp_liq(const P& c, real t) { return cl_exp<real>(c, cl_div_p<real>(c, c.r3les * (t - c.rtt), t - c.r4les)); }
template <typename real, typename P>
CLOUDSC_HD real exp_ice(const P& c, real t) { return cl_exp<real>(c, cl_div_p<real>(c, c.r3ies * (t - c.rtt), t - c.r4ies)); }
// exp_liq and exp_ice of one temperature (the saturation values at T and in each
// Newton step): the two divisions and exps are independent; in fp64 the exps
// run as a pair with one range check (cloudsc_libm::exp_pair_split), so the
// two chains interleave in one basic block (round 4, with the late range check
// of exp_split: -1.3 % fp64 KSEG on the same box,
// profiles/r04/experiment_exp_pair_ab.txt).  Same bits as the two calls.
template <typename real, typename P>
CLOUDSC_HD void exp_liq_ice(const P& c, real t, real& el, real& ei) {
  const real ql = cl_div_p<real>(c, c.r3les * (t - c.rtt), t - c.r4les);
  const real qi = cl_div_p<real>(c, c.r3ies * (t - c.rtt), t - c.r4ies);
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (std::is_same<real, double>::value) {
    cloudsc_libm::exp_pair_split(ql, qi, &el, &ei, LdsLibmTabs{}, DevLibmCold{});
    return;
  }
#endif
  el = cl_exp<real>(c, ql);
  ei = cl_exp<real>(c, qi);
}

// alfa*R5ALVCP/(T-R4LES)^2 + (1-alfa)*R5ALSCP/(T-R4IES)^2 (cloudsc_c.c:1166,1220)
template <typename real, typename P>
CLOUDSC_HD real foedem_term(const P& c, real t, real alfa) {
  real dl = t - c.r4les, di = t - c.r4ies;
  return ((alfa * c.r5alvcp) * cl_div_p<real>(c, R(1.0), dl * dl)) + (((R(1.0) - alfa) * c.r5alscp) * cl_div_p<real>(c, R(1.0), di * di));
}

}  // namespace cloudsc
