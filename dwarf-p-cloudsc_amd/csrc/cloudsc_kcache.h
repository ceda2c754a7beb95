// cloudsc_kcache.h -- the CLOUDSC column physics for CDNA4 (gfx950), split into
// per-level phases, and the SCC-k-caching kernel body built from them.
//
// Semantics: the reference kernel src/cloudsc_c/cloudsc/cloudsc_c.c:19-2587
// (restated, bit-exact on the CPU, by oracle/cloudsc_oracle.c).  Structure:
// the k-caching layout of src/cloudsc_gpu/cloudsc_gpu_scc_k_caching_mod.F90 --
// an NPROMA block is one workgroup, a column is one lane, and ONE fused loop
// walks the levels top-down.  Everything the reference keeps in level-sized
// temporaries (ztp1, za, zqx, zqx0, zlneg, zqxn2d, zfoealfa, zpfplsx, ...) is
// consumed at the level that produces it, so the only state that survives an
// iteration is a handful of registers (CarryState): T/A/PAP of the level above,
// zanewm1, zqxnm1[ql,qi], zpfplsx[qi,qr,qs], zcovptot, zcovpmax, zcldtopdist,
// prainfrac, and the six running flux sums of section 8 (which the CUDA
// k-caching kernel re-reads from HBM every level, cloudsc_c_k_caching.cu:2557-2576;
// here they never leave the register file).  HBM traffic is the compulsory
// one: each input element read once, each output element written once
// (56,036 B/column in fp64).
//
// Latency hiding: only NGPTOT/64 waves exist (2560 at 163840 columns, 2.5 per
// SIMD), so the loop software-pipelines its loads: the inputs of level k+1 are
// issued before the physics of level k runs (LevelIn `nxt`), and the fields the
// physics needs one level ahead (paph, pmfu, pmfd, plu) two levels ahead.
//
// Arithmetic keeps the reference's operand order (hipcc -ffp-contract=off, so
// no FMA contraction), divisions are correctly rounded (cl_div) and fp64
// exp/pow are the reference CPU build's own algorithms (cloudsc_libm.h): the
// fp64 output is the reference kernel's, bit for bit.
#pragma once
#include "cloudsc_dev.h"
#define CLOUDSC_PARAMS_HERE const PT& c = *(const PT*)launder_uniform(cpar)

namespace cloudsc {

template <typename real>
struct KArgs {
  const real *pt, *pq, *ttt, *ttq, *tta, *ttcld, *pvfl, *pvfi, *phrsw, *phrlw, *pvervel;
  const real *pap, *paph, *plsm;
  const int *ktype;
  const real *plu, *psnde, *pmfu, *pmfd, *pa, *pclv, *psupsat, *picrit_aer, *pre_ice, *pnice;
  const real *plude_in;   // plude as read: == plude (in place, the C ABI) or a pristine copy (state runs)
  real *plude, *tlt, *tlq, *tla, *tlcld, *pcovptot, *prainfrac;
  real *pfsqlf, *pfsqif, *pfcqnng, *pfcqlng, *pfsqrf, *pfsqsf, *pfcqrng, *pfcqsng;
  real *pfsqltur, *pfsqitur, *pfplsl, *pfplsn, *pfhpsl, *pfhpsn;
  const DevParams<real>* par;   // the launch's parameter set (device memory, read with scalar loads)
  int ngptot, nproma, klev;
};

enum { QL = 0, QI = 1, QR = 2, QS = 3, QV = 4 };

// Field access = uniform element index (SGPR arithmetic on a uniform base
// pointer) + the lane's byte offset (one shared 32-bit VGPR).  This is the
// global_load/store "saddr" form: no per-field 64-bit VGPR pointers.
template <typename T>
CLOUDSC_HD T ldg(const T* ubase, size_t uidx, unsigned lane_bytes) {
  return *(const T*)((const char*)(ubase + uidx) + lane_bytes);
}
// Outputs are written once and never read back by the kernel, and the level
// inputs are read once: the inputs are non-temporal (streaming) loads, so the
// caches keep what is re-read (the neighbour levels, the hand-off state)
// (-1.9 % kernel time with nt loads and stores, profiles/r01/ab_nontemporal.txt).
// The outputs are write-through stores (sc1: an agent-scope relaxed atomic store
// lowers to global_store ... sc1, which leaves no line of it in the XCD's L2;
// plain and nt stores keep theirs, MI355X_MICROARCH.md): -0.7...-0.8 % fp64 and
// -0.5 % fp32 against nt stores, the same bits (profiles/r05/experiments_kernel_ab.txt).
// stg_cached is for scratch that is read back (the SCC variant's temporaries).
template <typename T>
CLOUDSC_HD void stg_cached(T* ubase, size_t uidx, unsigned lane_bytes,
                                           typename std::common_type<T>::type v) {
  *(T*)((char*)(ubase + uidx) + lane_bytes) = v;
}
#if defined(__HIP_DEVICE_COMPILE__)
// the write-through store of one output element (4 or 8 bytes, naturally aligned)
template <typename T, typename P>
__device__ __forceinline__ void st_wt(P* p, T v) {
  using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned>::type;
  U bits;
  __builtin_memcpy(&bits, &v, sizeof(T));
  __hip_atomic_store((U*)p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#endif
template <typename T>
CLOUDSC_HD void stg(T* ubase, size_t uidx, unsigned lane_bytes, typename std::common_type<T>::type v) {
#if defined(__HIP_DEVICE_COMPILE__)
  st_wt<T>((char*)(ubase + uidx) + lane_bytes, (T)v);
#else
  *(T*)((char*)(ubase + uidx) + lane_bytes) = v;
#endif
}
// a level input, read exactly once
template <typename T>
CLOUDSC_HD T ldg1(const T* ubase, size_t uidx, unsigned lane_bytes) {
  return __builtin_nontemporal_load((const T*)((const char*)(ubase + uidx) + lane_bytes));
}

// The same accesses with the uniform address made opaque first (fp32): several
// accesses of one field at different uniform indices (the species planes)
// otherwise share one 64-bit VGPR pointer, base + lane offset, and each adds its
// index to it with a VALU op; with the uniform pointer opaque, every access is
// the saddr + voffset form.  fp32 only: its level loop is VALU-issue-bound.
template <typename T>
CLOUDSC_HD T ldg1_u(const T* ubase, size_t uidx, unsigned lane_bytes) {
#if defined(__HIP_DEVICE_COMPILE__)
  const T* p = ubase + uidx;
  asm("" : "+s"(p));   // (the asm's output is a generic pointer: global address space restated below)
  using GT = const __attribute__((address_space(1))) T;
  return __builtin_nontemporal_load((GT*)((const __attribute__((address_space(1))) char*)p + lane_bytes));
#else
  return ldg1(ubase, uidx, lane_bytes);
#endif
}
template <typename T>
CLOUDSC_HD void stg_u(T* ubase, size_t uidx, unsigned lane_bytes, typename std::common_type<T>::type v) {
#if defined(__HIP_DEVICE_COMPILE__)
  T* p = ubase + uidx;
  asm("" : "+s"(p));
  st_wt<T>((__attribute__((address_space(1))) char*)p + lane_bytes, (T)v);
#else
  stg(ubase, uidx, lane_bytes, v);
#endif
}
// species planes: the opaque-pointer form in fp32, the plain one in fp64
template <typename T>
CLOUDSC_HD T ldg1_sp(const T* ubase, size_t uidx, unsigned lane_bytes) {
  if constexpr (sizeof(T) == 4) return ldg1_u(ubase, uidx, lane_bytes);
  else return ldg1(ubase, uidx, lane_bytes);
}
template <typename T>
CLOUDSC_HD void stg_sp(T* ubase, size_t uidx, unsigned lane_bytes, typename std::common_type<T>::type v) {
  if constexpr (sizeof(T) == 4) stg_u(ubase, uidx, lane_bytes, v);
  else stg(ubase, uidx, lane_bytes, v);
}

// Per-level inputs of one column (the prefetch unit).
template <typename real>
struct LevelIn {
  real pt, pq, ttt, ttq, tta, pa, pap, phrsw, phrlw, pvervel, plude, psnde, psupsat, pvfl, pvfi;
  real pclv[4], ttcld[4];
  real pre_ice, picrit_aer, pnice;      // aerosol inputs, loaded only under LAERICESED/LAERICEAUTO
};

// PF 3: the inputs section 1 and the start of section 3 consume first
// (init_level, the saturation values), prefetched for level k+1 in the middle
// of level k; the rest is loaded at the top of its own level.
template <typename real>
struct EarlyIn {
  real pt, pq, ttt, ttq, tta, pa, pap;
  real pclv[4], ttcld[4];
};
template <typename real>
CLOUDSC_HD void load_early(EarlyIn<real>& E, const KArgs<real>& A, size_t u2, size_t u3, int k, int klev,
                           int nproma, unsigned lo) {
  const size_t i = u2 + (size_t)k * nproma;
  E.pt = ldg1(A.pt, i, lo); E.pq = ldg1(A.pq, i, lo); E.ttt = ldg1(A.ttt, i, lo); E.ttq = ldg1(A.ttq, i, lo);
  E.tta = ldg1(A.tta, i, lo); E.pa = ldg1(A.pa, i, lo); E.pap = ldg1(A.pap, i, lo);
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const size_t j = u3 + ((size_t)m * klev + k) * nproma;
    E.pclv[m] = ldg1_sp(A.pclv, j, lo);
    E.ttcld[m] = ldg1_sp(A.ttcld, j, lo);
  }
}
template <typename real, bool AER>
CLOUDSC_HD void load_late(LevelIn<real>& L, const KArgs<real>& A, size_t u2, int k, int nproma, unsigned lo) {
  const size_t i = u2 + (size_t)k * nproma;
  L.plude = ldg1(A.plude_in, i, lo); L.pvfl = ldg1(A.pvfl, i, lo); L.pvfi = ldg1(A.pvfi, i, lo);
  L.phrsw = ldg1(A.phrsw, i, lo); L.phrlw = ldg1(A.phrlw, i, lo); L.pvervel = ldg1(A.pvervel, i, lo);
  L.psnde = ldg1(A.psnde, i, lo); L.psupsat = ldg1(A.psupsat, i, lo);
  if (AER) {
    L.pre_ice = ldg1(A.pre_ice, i, lo); L.picrit_aer = ldg1(A.picrit_aer, i, lo); L.pnice = ldg1(A.pnice, i, lo);
  } else {
    L.pre_ice = R(0.0); L.picrit_aer = R(1.0); L.pnice = R(1.0);
  }
}
template <typename real>
CLOUDSC_HD void take_early(LevelIn<real>& L, const EarlyIn<real>& E) {
  L.pt = E.pt; L.pq = E.pq; L.ttt = E.ttt; L.ttq = E.ttq; L.tta = E.tta; L.pa = E.pa; L.pap = E.pap;
#pragma unroll
  for (int m = 0; m < 4; m++) { L.pclv[m] = E.pclv[m]; L.ttcld[m] = E.ttcld[m]; }
}

// Values of the neighbouring levels the physics of level k reads.
template <typename real>
struct Neighbors {
  real paph_k, paph_n;                  // paph(k), paph(k+1)
  real pmfu_k, pmfd_k, pmfu_n, pmfd_n;  // mass fluxes at k and k+1
  real plu_n;                           // plu(k+1)
};

// Column constants.
template <typename real>
struct ColConst {
  real paph_sfc, kk_const, kk_lcrit, kk_pow;
  int ktype;
};

// State carried from level k to level k+1.
template <typename real>
struct CarryState {
  real t_prev, a_prev, pap_prev, zanewm1, zcovptot, zcovpmax, zcldtopdist, rainfrac;
  real qxnm1_l, qxnm1_i;                // zqxnm1 of the non-falling condensates
  real pfx_i, pfx_r, pfx_s;             // zpfplsx[qi,qr,qs] arriving at level k
  real fl_lf, fl_if, fl_lng, fl_nng, fl_ltur, fl_itur;  // running flux sums (section 8)
};

// The same 19 values kept in LDS instead of registers: every wave owns 19
// planes of 64 lanes ([wave][slot][lane], conflict-free, constant ds offsets).
// They are touched a few times per level each, and taking them out of the
// register file is what lets the fp64 kernel fit more waves per SIMD.
// Accesses are volatile so that the compiler re-reads at each use instead of
// keeping a register copy alive across the level.
#define CLOUDSC_AS3 __attribute__((address_space(3)))
template <typename real, int Q>
struct LdsSlot {
  CLOUDSC_AS3 real* base;               // this lane's slot 0
  __device__ __forceinline__ operator real() const { return *(volatile CLOUDSC_AS3 real*)(base + Q * 64); }
  __device__ __forceinline__ LdsSlot& operator=(real v) {
    *(volatile CLOUDSC_AS3 real*)(base + Q * 64) = v;
    return *this;
  }
  __device__ __forceinline__ LdsSlot& operator=(const LdsSlot& o) { return *this = (real)o; }
};
template <typename real>
struct CarryLds {
  static constexpr int kSlots = 19;
  __device__ __forceinline__ explicit CarryLds(CLOUDSC_AS3 real* b)
      : t_prev{b}, a_prev{b}, pap_prev{b}, zanewm1{b}, zcovptot{b}, zcovpmax{b}, zcldtopdist{b}, rainfrac{b},
        qxnm1_l{b}, qxnm1_i{b}, pfx_i{b}, pfx_r{b}, pfx_s{b}, fl_lf{b}, fl_if{b}, fl_lng{b}, fl_nng{b},
        fl_ltur{b}, fl_itur{b} {}
  LdsSlot<real, 0> t_prev; LdsSlot<real, 1> a_prev; LdsSlot<real, 2> pap_prev; LdsSlot<real, 3> zanewm1;
  LdsSlot<real, 4> zcovptot; LdsSlot<real, 5> zcovpmax; LdsSlot<real, 6> zcldtopdist; LdsSlot<real, 7> rainfrac;
  LdsSlot<real, 8> qxnm1_l; LdsSlot<real, 9> qxnm1_i;
  LdsSlot<real, 10> pfx_i; LdsSlot<real, 11> pfx_r; LdsSlot<real, 12> pfx_s;
  LdsSlot<real, 13> fl_lf; LdsSlot<real, 14> fl_if; LdsSlot<real, 15> fl_lng; LdsSlot<real, 16> fl_nng;
  LdsSlot<real, 17> fl_ltur; LdsSlot<real, 18> fl_itur;
};
// LDS bytes of the carried state for a workgroup of nproma lanes
template <typename real>
constexpr size_t carry_lds_bytes(int nproma) {
  return (size_t)((nproma + 63) / 64) * CarryLds<real>::kSlots * 64 * sizeof(real);
}
template <typename real>
__device__ __forceinline__ CLOUDSC_AS3 real* carry_lds_base() {
  extern __shared__ __attribute__((aligned(16))) char cloudsc_dyn_lds[];
  const int t = threadIdx.x;
  return (CLOUDSC_AS3 real*)(CLOUDSC_AS3 char*)cloudsc_dyn_lds + (t >> 6) * (CarryLds<real>::kSlots * 64) + (t & 63);
}

// Result of section 1 at one level (the reference's level-sized temporaries).
template <typename real>
struct LevelState {
  real ztp1, za, zaorig, zfoealfa, ttend, qtend;
  real zqx[5], zqx0[5], zlneg[4];
};

// Result of the physics at one level.
template <typename real>
struct PhysOut {
  real zqxn[4];                         // zqxn2d(k), zero above NCLDTOP
  real plude_k, atend, ctend[4], zcovptot_out;
};

// All loads of a level are unconditional (the physics-only fields are read at
// every level): branches around memory operations make hipcc's vmcnt
// bookkeeping fall back to vmcnt(0), which drains the software pipeline.
template <typename real, bool AER>
CLOUDSC_HD void load_level(LevelIn<real>& L, const KArgs<real>& A, size_t u2, size_t u3, int k,
                                           int klev, int nproma, unsigned lo) {
  const size_t i = u2 + (size_t)k * nproma;
  L.pt = ldg1(A.pt, i, lo); L.pq = ldg1(A.pq, i, lo); L.ttt = ldg1(A.ttt, i, lo); L.ttq = ldg1(A.ttq, i, lo);
  L.tta = ldg1(A.tta, i, lo); L.pa = ldg1(A.pa, i, lo); L.pap = ldg1(A.pap, i, lo);
  L.plude = ldg1(A.plude_in, i, lo); L.pvfl = ldg1(A.pvfl, i, lo); L.pvfi = ldg1(A.pvfi, i, lo);
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const size_t j = u3 + ((size_t)m * klev + k) * nproma;
    L.pclv[m] = ldg1_sp(A.pclv, j, lo);
    L.ttcld[m] = ldg1_sp(A.ttcld, j, lo);
  }
  L.phrsw = ldg1(A.phrsw, i, lo); L.phrlw = ldg1(A.phrlw, i, lo); L.pvervel = ldg1(A.pvervel, i, lo);
  L.psnde = ldg1(A.psnde, i, lo); L.psupsat = ldg1(A.psupsat, i, lo);
  if (AER) {   // LAERICESED / LAERICEAUTO inputs; the launch picks AER from the flags
    L.pre_ice = ldg1(A.pre_ice, i, lo); L.picrit_aer = ldg1(A.picrit_aer, i, lo); L.pnice = ldg1(A.pnice, i, lo);
  } else {
    L.pre_ice = R(0.0); L.picrit_aer = R(1.0); L.pnice = R(1.0);
  }
}

// ===== 1. initial values, tidy-up, FOEALFA at one level (cloudsc_c.c:462-575, 588, 625) =====
template <typename real, typename P>
CLOUDSC_HD void init_level(const P& c, const LevelIn<real>& in, LevelState<real>& s) {
  s.ztp1 = in.pt + c.ptsphy * in.ttt;
  real* zqx = s.zqx;
  real* zlneg = s.zlneg;
  zqx[QV] = in.pq + c.ptsphy * in.ttq;
  s.zqx0[QV] = zqx[QV];
  real za = in.pa + c.ptsphy * in.tta;
  s.zaorig = za;
#pragma unroll
  for (int m = 0; m < 4; m++) {
    zqx[m] = in.pclv[m] + c.ptsphy * in.ttcld[m];
    s.zqx0[m] = zqx[m];
    zlneg[m] = R(0.0);
  }
  // The zero is opaque to the optimiser: with it visible, the fp32 SCC build
  // (packed v_pk_mul_f32 operands) folded (0 - a) - b into (-a) - b, which is
  // -0 instead of +0 when a = b = 0 -- a sign-of-zero change the IEEE
  // semantics (no nsz flag) do not allow.
  real ttend = launder_vgpr(R(0.0)), qtend = launder_vgpr(R(0.0));
  // tidy up very small cloud cover or total cloud water (:519-541)
  if (zqx[QL] + zqx[QI] < c.rlmin || za < c.ramin) {
    real zqadj;
    zlneg[QL] = zlneg[QL] + zqx[QL];
    zqadj = zqx[QL] * c.zqtmst;
    qtend = qtend + zqadj;
    ttend = ttend - c.ralvdcp * zqadj;
    zqx[QV] = zqx[QV] + zqx[QL];
    zqx[QL] = R(0.0);
    zlneg[QI] = zlneg[QI] + zqx[QI];
    zqadj = zqx[QI] * c.zqtmst;
    qtend = qtend + zqadj;
    ttend = ttend - c.ralsdcp * zqadj;
    zqx[QV] = zqx[QV] + zqx[QI];
    zqx[QI] = R(0.0);
    za = R(0.0);
  }
  // tidy up small CLV variables (:547-575)
#pragma unroll
  for (int m = 0; m < 4; m++) {
    if (zqx[m] < c.rlmin) {
      zlneg[m] = zlneg[m] + zqx[m];
      const real zqadj = zqx[m] * c.zqtmst;
      qtend = qtend + zqadj;
      if (m == QL || m == QR) ttend = ttend - c.ralvdcp * zqadj;   // iphase 1
      else ttend = ttend - c.ralsdcp * zqadj;                        // iphase 2
      zqx[QV] = zqx[QV] + zqx[m];
      zqx[m] = R(0.0);
    }
  }
  s.zfoealfa = foealfa<real>(c, s.ztp1);
  s.za = fmax(R(0.0), fmin(R(1.0), za));    // clip cloud fraction (:625)
  s.ttend = ttend;
  s.qtend = qtend;
}

// Per-phase cost ablation (timing-only experiment builds, tools/ablation.sh):
// -DCLOUDSC_ABLATE=<mask> skips the marked sections of the physics; the loads
// and stores stay, downstream sections see zero contributions (or, for the
// Newton chain, a cheap stand-in of the same sign), so the difference to the
// full kernel is the section's cost.  0 (the default) compiles nothing out.
#ifndef CLOUDSC_ABLATE
#define CLOUDSC_ABLATE 0
#endif
enum AblateBit : unsigned {
  AB_SUPSAT = 1u << 0,     // 3.1 supersaturation adjustment
  AB_CONV = 1u << 1,       // 3.2 detrainment, 3.3 subsidence source and sink
  AB_EROSION = 1u << 2,    // 3.4 erosion
  AB_NEWTON = 1u << 3,     // 3.4 dqs/dt: the two Newton steps
  AB_COND = 1u << 4,       // 3.4a/b evaporation, condensation, new clouds
  AB_DEPOS = 1u << 5,      // 3.7 ice deposition
  AB_SEDIM = 1u << 6,      // 4.2 sedimentation, precipitation cover
  AB_AUTO = 1u << 7,       // 4.3 autoconversion (snow, KK rain), riming
  AB_MELT = 1u << 8,       // 4.4 melting, freezing
  AB_EVAP = 1u << 9,       // 4.5 rain and snow evaporation
  AB_TRUNC = 1u << 10,     // 5.2 sink truncation
  AB_SOLVE = 1u << 11,     // 5.2.2 implicit solver (divisions and substitutions)
  AB_SAT = 1u << 12,       // saturation exponentials at T (e_liq, e_ice): cheap stand-ins
};
constexpr unsigned kAblate = CLOUDSC_ABLATE;
#define CLOUDSC_RUN(bit) ((kAblate & (bit)) == 0)

// ===== 3.-6. physics of one level ncldtop <= k (cloudsc_c.c:732-2508) =====
// Where in the level physics_level calls its mid hook: 0 (the default) after
// 5.1; experiment builds (VFLAGS=-DCLOUDSC_MID_AT=n) move it earlier -- 1 before
// the Newton steps of 3.4, 2 before 3.7, 3 before 4.2, 4 before 4.4, 5 before
// 4.5 -- trading a longer flight time of the next level's loads against their
// registers being live across more of the physics.
#ifndef CLOUDSC_MID_AT
#define CLOUDSC_MID_AT 0
#endif
#define CLOUDSC_MID_HOOK(n) do { if constexpr (CLOUDSC_MID_AT == (n)) mid(); } while (0)
// Nothing to do at the middle of a level (the default hook of physics_level).
struct NoMidHook {
  CLOUDSC_HD void operator()() const {}
};

template <typename real, typename P, typename CS, typename Mid = NoMidHook>
CLOUDSC_HD void physics_level(const P& c, const int k, const int klev,
                                              const int ncldtop0, const LevelIn<real>& in,
                                              const Neighbors<real>& nb, const ColConst<real>& cc,
                                              LevelState<real>& ls, CS& cs, PhysOut<real>& po,
                                              const Mid& mid = Mid{}) {
  const real zepsilon = R(100.0) * (sizeof(real) == 8 ? (real)__DBL_EPSILON__ : (real)__FLT_EPSILON__);
  const real zepsec = R(1.0e-14);
  const real ztw1 = R(1329.31000000000), ztw2 = R(0.00746150000000000), ztw3 = R(85000.0000000000);
  const real ztw4 = R(40.6370000000000), ztw5 = R(275.000000000000);
  const real ztp1 = ls.ztp1, za = ls.za, zaorig = ls.zaorig, zfoealfa = ls.zfoealfa;
  const real* zqx = ls.zqx;
  const real* zqx0 = ls.zqx0;
  real& ttend = ls.ttend;
  real& qtend = ls.qtend;
  real* zqxn = po.zqxn;
  real* ctend = po.ctend;
  real& plude_k = po.plude_k;
  real& atend = po.atend;

    const real pap_k = in.pap;
    // saturation values (:583-609)
    real e_liq, e_ice;
    if (CLOUDSC_RUN(AB_SAT)) {
      exp_liq_ice<real>(c, ztp1, e_liq, e_ice);
    } else {
      e_liq = launder_vgpr(ztp1 * R(0.02));
      e_ice = launder_vgpr(ztp1 * R(0.019));
    }
    // divisors shared by several divisions (cl_recip: one reciprocal, same quotient bits)
    const Recip<real> r_pap = cl_recip_p<real>(c, pap_k);
    const real zfoeewmt = fmin(cl_div_p<real>(c, (c.r2es * (zfoealfa * e_liq + (R(1.0) - zfoealfa) * e_ice)), r_pap), R(0.5));
    const Recip<real> r_mixd = cl_recip_p<real>(c, R(1.0) - c.retv * zfoeewmt);
    const real zqsmix = cl_div_p<real>(c, zfoeewmt, r_mixd);
    const real zalfa_d = fmax(R(0.0), copysign(R(1.0), ztp1 - c.rtt));
    real zfoeew = fmin(cl_div_p<real>(c, (zalfa_d * (c.r2es * e_liq) + (R(1.0) - zalfa_d) * (c.r2es * e_ice)), r_pap), R(0.5));
    zfoeew = fmin(R(0.5), zfoeew);
    const Recip<real> r_iced = cl_recip_p<real>(c, R(1.0) - c.retv * zfoeew);
    const real zqsice = cl_div_p<real>(c, zfoeew, r_iced);
    // (zqsliq, :601-604, is computed where rain evaporation, its only reader, runs)
    // liquid/ice fractions (:628-636)
    const real zli = zqx[QL] + zqx[QI];
    real zliqfrac = R(0.0), zicefrac = R(0.0);
    if (zli > c.rlmin) {
      zliqfrac = cl_div_p<real>(c, zqx[QL], zli);
      zicefrac = R(1.0) - zliqfrac;
    }

    // ===== 3. physics (:732-2508) =====
    real zqxfg[5];
  #pragma unroll
    for (int m = 0; m < 5; m++) zqxfg[m] = zqx[m];
    // zsolqa is dense in the reference; only 13 entries can become non-zero
    // here, kept as named scalars sa_<a><b> == zsolqa[a][b] (C indexing).  Every
    // off-diagonal pair is updated antisymmetrically (x to one, -x to the other,
    // in the same order, and scaled by the same factors in 5.2), and IEEE
    // negation is exact and sign-symmetric under round-to-nearest, so
    // zsolqa[b][a] == -zsolqa[a][b] exactly: only one of each pair is stored.
    //   stored: ll ii rr ss (diagonal)  lv iv li ls lr ir sr rv sv
    //   implied: vl=-lv vi=-iv il=-li sl=-ls rl=-lr ri=-ir rs=-sr vr=-rv vs=-sv
    real sa_ll = 0, sa_ii = 0, sa_rr = 0, sa_ss = 0;
    real sa_lv = 0, sa_iv = 0, sa_li = 0, sa_ls = 0, sa_lr = 0, sa_ir = 0, sa_sr = 0, sa_rv = 0, sa_sv = 0;
    // zsolqb non-zeros: [ql][ql], [qi][qi] (subsidence), [qi][qs] (snow autoconv), [ql][qs] (riming)
    real sb_ll = 0, sb_ii = 0, sb_is = 0, sb_ls = 0;
    real conv_src_l = 0, conv_src_i = 0, conv_sink = 0, psup_l = 0, psup_i = 0;
    real fsrc_i = 0, fsrc_r = 0, fsrc_s = 0;
    real zqpretot = R(0.0), zsolab = R(0.0), zsolac = R(0.0);

    // 3.0 derived variables (:799-841)
    const real zdp = nb.paph_n - nb.paph_k;
    const real zgdp = cl_div_p<real>(c, c.rg, zdp);
    const real zrho = cl_div_p<real>(c, pap_k, (c.rd * ztp1));
    const real zdtgdp = c.ptsphy * zgdp;
    const real zrdtgdp = zdp * c.zinv_tsrg;
    real zfacw, zfaci, zfac, zcor;
    { const real d = ztp1 - c.r4les; zfacw = cl_div_p<real>(c, c.r5les, (d * d)); }
    { const real d = ztp1 - c.r4ies; zfaci = cl_div_p<real>(c, c.r5ies, (d * d)); }
    zcor = cl_div_p<real>(c, R(1.0), r_iced);
    const real zdqsicedt = (zfaci * zcor) * zqsice;
    const real zcorqsice = R(1.0) + c.ralsdcp * zdqsicedt;
    zfac = zfoealfa * zfacw + (R(1.0) - zfoealfa) * zfaci;
    zcor = cl_div_p<real>(c, R(1.0), r_mixd);
    const real zdqsmixdt = (zfac * zcor) * zqsmix;
    const real zcorqsmix = R(1.0) + (zfoealfa * c.ralvdcp + (R(1.0) - zfoealfa) * c.ralsdcp) * zdqsmixdt;
    const real zevaplimmix = fmax(cl_div_p<real>(c, (zqsmix - zqx[QV]), zcorqsmix), R(0.0));
    real ztmpa = cl_div_p<real>(c, R(1.0), fmax(za, zepsec));
    const Recip<real> r_1mza = cl_recip_p<real>(c, fmax(zepsec, R(1.0) - za));
    real zliqcld = zqx[QL] * ztmpa;
    real zicecld = zqx[QI] * ztmpa;
    real zlicld = zliqcld + zicecld;

    // evaporate very small amounts of liquid and ice (:846-859)
    if (zqx[QL] < c.rlmin) { sa_lv = zqx[QL]; }
    if (zqx[QI] < c.rlmin) { sa_iv = zqx[QI]; }

    // 3.1 ice supersaturation adjustment (:874-954)
    const real zfokoop = fmin(c.rkoop1 - c.rkoop2 * ztp1, cl_div_p<real>(c, (c.r2es * e_liq) * R(1.0), (c.r2es * e_ice)));
    if (c.nssopt == 0 || ztp1 >= c.rtt) {
      zfac = R(1.0);
      zfaci = R(1.0);
    } else {
      zfac = za + zfokoop * (R(1.0) - za);
      zfaci = c.zfaci_koop;
    }
    real zsupsat = R(0.0);
    if (!CLOUDSC_RUN(AB_SUPSAT)) {
    } else if (za > c.one_m_ramin) {
      zsupsat = fmax(cl_div_p<real>(c, (zqx[QV] - zfac * zqsice), zcorqsice), R(0.0));
    } else {
      const real zqp1env = cl_div_p<real>(c, (zqx[QV] - za * zqsice), fmax(R(1.0) - za, zepsilon));
      zsupsat = fmax(cl_div_p<real>(c, ((R(1.0) - za) * (zqp1env - zfac * zqsice)), zcorqsice), R(0.0));
    }
    const bool warm_homo = ztp1 > c.rthomo;
    if (zsupsat > zepsec) {
      if (warm_homo) { sa_lv = sa_lv - zsupsat; zqxfg[QL] = zqxfg[QL] + zsupsat;
      } else { sa_iv = sa_iv - zsupsat; zqxfg[QI] = zqxfg[QI] + zsupsat;
      }
      zsolac = (R(1.0) - za) * zfaci;
    }
    if (CLOUDSC_RUN(AB_SUPSAT) && in.psupsat > zepsec) {
      if (warm_homo) {
        sa_ll = sa_ll + in.psupsat; psup_l = in.psupsat; zqxfg[QL] = zqxfg[QL] + in.psupsat;
      } else {
        sa_ii = sa_ii + in.psupsat; psup_i = in.psupsat; zqxfg[QI] = zqxfg[QI] + in.psupsat;
      }
      zsolac = (R(1.0) - za) * zfaci;
    }

    // 3.2 detrainment from convection (:967-987)
    if (CLOUDSC_RUN(AB_CONV) && k < klev - 1) {
      plude_k = plude_k * zdtgdp;
      if (nb.plu_n > zepsec && plude_k > c.rlmin) {
        zsolac = zsolac + cl_div_p<real>(c, plude_k, nb.plu_n);
        conv_src_l = zfoealfa * plude_k;
        conv_src_i = (R(1.0) - zfoealfa) * plude_k;
        sa_ll = sa_ll + conv_src_l;
        sa_ii = sa_ii + conv_src_i;
      } else {
        plude_k = R(0.0);
      }
      sa_ss = sa_ss + in.psnde * zdtgdp;
    }

    // 3.3 subsidence source from the layer above + evaporation (:1002-1058)
    if (CLOUDSC_RUN(AB_CONV) && k > ncldtop0) {
      const real zmf = fmax(R(0.0), (nb.pmfu_k + nb.pmfd_k) * zdtgdp);
      real zacust = zmf * cs.zanewm1;
      const real zlcust_l = zmf * cs.qxnm1_l;
      const real zlcust_i = zmf * cs.qxnm1_i;
      conv_src_l = conv_src_l + zlcust_l;
      conv_src_i = conv_src_i + zlcust_i;
      const real zdtdp = cl_div_p<real>(c, ((c.zrdcp * R(0.5)) * (cs.t_prev + ztp1)), nb.paph_k);
      const real zdtforc = zdtdp * (pap_k - cs.pap_prev);
      const real zdqs = (cs.zanewm1 * zdtforc) * zdqsmixdt;
      real zlfinalsum = R(0.0);
      {
        real zlfinal = fmax(R(0.0), zlcust_l - zdqs);
        const real zevap = fmin(zlcust_l - zlfinal, zevaplimmix);
        zlfinal = zlcust_l - zevap;
        zlfinalsum = zlfinalsum + zlfinal;
        sa_ll = sa_ll + zlcust_l; sa_lv = sa_lv + zevap;
      }
      {
        real zlfinal = fmax(R(0.0), zlcust_i - zdqs);
        const real zevap = fmin(zlcust_i - zlfinal, zevaplimmix);
        zlfinal = zlcust_i - zevap;
        zlfinalsum = zlfinalsum + zlfinal;
        sa_ii = sa_ii + zlcust_i; sa_iv = sa_iv + zevap;
      }
      if (zlfinalsum < zepsec) zacust = R(0.0);
      zsolac = zsolac + zacust;
    }

    // subsidence sink of cloud to the layer below (:1064-1075)
    if (CLOUDSC_RUN(AB_CONV) && k < klev - 1) {
      const real zmfdn = fmax(R(0.0), (nb.pmfu_n + nb.pmfd_n) * zdtgdp);
      zsolab = zsolab + zmfdn;
      sb_ll = sb_ll + zmfdn;
      sb_ii = sb_ii + zmfdn;
      conv_sink = zmfdn;
    }

    // 3.4 erosion of clouds by turbulent mixing (:1087-1118)
    const real zldifdt = (cc.ktype > 0 && plude_k > zepsec) ? pval(c, c.zldifdt_conv) : pval(c, c.zldifdt0);
    if (CLOUDSC_RUN(AB_EROSION) && zli > zepsec) {
      const real ze = zldifdt * fmax(zqsmix - zqx[QV], R(0.0));
      real zleros = za * ze;
      zleros = fmin(zleros, zevaplimmix);
      zleros = fmin(zleros, zli);
      const real zaeros = cl_div_p<real>(c, zleros, zlicld);
      zsolac = zsolac - zaeros;
      sa_lv = sa_lv + zliqfrac * zleros;
      sa_iv = sa_iv + zicefrac * zleros;
    }

    CLOUDSC_MID_HOOK(1);
    // 3.4 condensation/evaporation due to dqsat/dt: two Newton steps (:1137-1182)
    real zdqs;
    if (!CLOUDSC_RUN(AB_NEWTON)) {
      zdqs = launder_vgpr((zqsmix - zqx[QV]) * R(0.1));   // stand-in of the right sign
    } else {
      const real zdtdp = cl_div_p<real>(c, (c.zrdcp * ztp1), r_pap);
      const real zdpmxdt = zdp * c.zqtmst;
      const real zmfdn = (k < klev - 1) ? nb.pmfu_n + nb.pmfd_n : R(0.0);
      real zwtot = in.pvervel + c.half_rg * (nb.pmfu_k + nb.pmfd_k + zmfdn);
      zwtot = fmin(zdpmxdt, fmax(-zdpmxdt, zwtot));
      const real zzzdt = in.phrsw + in.phrlw;
      const real zdtdiab = fmin(zdpmxdt * zdtdp, fmax(-zdpmxdt * zdtdp, zzzdt)) * c.ptsphy + c.ralfdcp * R(0.0);
      const real zdtforc = (zdtdp * zwtot) * c.ptsphy + zdtdiab;
      real tt = fmax(ztp1 + zdtforc, R(160.0));
      real qsm = zqsmix;
      const real zqp = cl_div_p<real>(c, R(1.0), r_pap);
  #pragma unroll
      for (int it = 0; it < 2; it++) {
        const real a = foealfa<real>(c, tt);
        real el, ei;
        exp_liq_ice<real>(c, tt, el, ei);
        real zqsat = (c.r2es * (a * el + (R(1.0) - a) * ei)) * zqp;
        zqsat = fmin(R(0.5), zqsat);
        const real zcor2 = cl_div_p<real>(c, R(1.0), (R(1.0) - c.retv * zqsat));
        zqsat = zqsat * zcor2;
        const real zcond = cl_div_p<real>(c, (qsm - zqsat), (R(1.0) + (zqsat * zcor2) * foedem_term<real>(c, tt, a)));
        tt = tt + (a * c.ralvdcp + (R(1.0) - a) * c.ralsdcp) * zcond;
        qsm = qsm - zcond;
      }
      zdqs = qsm - zqsmix;
    }

    // 3.4a evaporation of clouds (:1189-1207)
    if (CLOUDSC_RUN(AB_COND) && zdqs > R(0.0)) {
      real zlevap = za * fmin(zdqs, zlicld);
      zlevap = fmin(zlevap, zevaplimmix);
      zlevap = fmin(zlevap, fmax(zqsmix - zqx[QV], R(0.0)));
      sa_lv = sa_lv + zliqfrac * zlevap;
      sa_iv = sa_iv + zicefrac * zlevap;
    }
    // 3.4b(1) increase of cloud water in existing clouds (:1213-1250)
    if (CLOUDSC_RUN(AB_COND) && zdqs <= -c.rlmin && za > zepsec) {
      real zlcond1 = fmax(-zdqs, R(0.0));
      real zcdmax;
      if (za > R(0.99)) {
        const real zcor3 = cl_div_p<real>(c, R(1.0), (R(1.0) - c.retv * zqsmix));
        zcdmax = cl_div_p<real>(c, (zqx[QV] - zqsmix), (R(1.0) + (zcor3 * zqsmix) * foedem_term<real>(c, ztp1, zfoealfa)));
      } else {
        zcdmax = cl_div_p<real>(c, (zqx[QV] - za * zqsmix), za);
      }
      zlcond1 = fmax(fmin(zlcond1, zcdmax), R(0.0));
      zlcond1 = za * zlcond1;
      if (zlcond1 < c.rlmin) zlcond1 = R(0.0);
      if (warm_homo) { sa_lv = sa_lv - zlcond1; zqxfg[QL] = zqxfg[QL] + zlcond1;
      } else { sa_iv = sa_iv - zlcond1; zqxfg[QI] = zqxfg[QI] + zlcond1;
      }
    }
    // 3.4b(2) generation of new clouds (:1253-1363)
    if (CLOUDSC_RUN(AB_COND) && zdqs <= -c.rlmin && za < R(1.0) - zepsec) {
      real zrhc = c.ramid;
      const real zsigk = cl_div_p<real>(c, pap_k, cc.paph_sfc);
      if (zsigk > R(0.8)) {
        const real s = cl_div_lit_p<real>(c, (zsigk - R(0.8)), R(0.2));
        zrhc = c.ramid + (R(1.0) - c.ramid) * (s * s);
      }
      real zqe = R(0.0);
      if (c.nssopt == 0 || c.nssopt == 1) {
        zqe = cl_div_p<real>(c, (zqx[QV] - za * zqsice), r_1mza);
        zqe = fmax(R(0.0), zqe);
      } else if (c.nssopt == 2) {
        zqe = zqx[QV];
      } else if (c.nssopt == 3) {
        zqe = zqx[QV] + zli;
      }
      const real zfacn = (c.nssopt == 0 || ztp1 >= c.rtt) ? R(1.0) : zfokoop;
      if (zqe >= zqsice * zfacn * zrhc && zqe < zqsice * zfacn) {
        real zacond = cl_div_p<real>(c, -((R(1.0) - za) * zfacn) * zdqs, fmax(R(2.0) * (zfacn * zqsice - zqe), zepsec));
        zacond = fmin(zacond, R(1.0) - za);
        real zlcond2 = -(zfacn * zdqs) * R(0.5) * zacond;
        const real zzdl = cl_div_p<real>(c, (R(2.0) * (zfacn * zqsice - zqe)), fmax(zepsec, R(1.0) - za));
        if (zdqs * zfacn < -zzdl) {
          const real zlcondlim = ((za - R(1.0)) * zfacn) * zdqs - zfacn * zqsice + zqx[QV];
          zlcond2 = fmin(zlcond2, zlcondlim);
        }
        zlcond2 = fmax(zlcond2, R(0.0));
        if (R(1.0) - za < zepsec || zlcond2 < c.rlmin) {
          zlcond2 = R(0.0);
          zacond = R(0.0);
        }
        if (zlcond2 == R(0.0)) zacond = R(0.0);
        zsolac = zsolac + zacond;
        if (warm_homo) { sa_lv = sa_lv - zlcond2; zqxfg[QL] = zqxfg[QL] + zlcond2;
        } else { sa_iv = sa_iv - zlcond2; zqxfg[QI] = zqxfg[QI] + zlcond2;
        }
      }
    }

    CLOUDSC_MID_HOOK(2);
    // 3.7 growth of ice by vapour deposition, Rotstayn (:1382-1447)
    if (za >= c.rcldtopcf && cs.a_prev < c.rcldtopcf) cs.zcldtopdist = R(0.0);
    else cs.zcldtopdist = cs.zcldtopdist + cl_div_p<real>(c, zdp, (zrho * c.rg));
    if (CLOUDSC_RUN(AB_DEPOS) && zqxfg[QL] > c.rlmin && ztp1 < c.rtt) {
      const real zvpice = cl_div_known_p<real>(c, ((c.r2es * e_ice) * c.rv), c.rd, c.rd_rcp);
      const real zvpliq = zvpice * zfokoop;
      const real zicenuclei = R(1000.0) * cl_exp<real>(c, cl_div_p<real>(c, (R(12.96) * (zvpliq - zvpice)), zvpliq) - R(0.639));
      const real zadd = cl_div_p<real>(c, (c.rlstt * (cl_div_p<real>(c, c.rlstt, (c.rv * ztp1)) - R(1.0))), (R(0.024) * ztp1));
      const real zbdd = cl_div_p<real>(c, ((c.rv * ztp1) * pap_k), (R(2.21) * zvpice));
      const real zcvds = cl_div_p<real>(c, ((R(7.8) * cl_pow<real>(c, cl_div_p<real>(c, zicenuclei, zrho), R(0.666))) * (zvpliq - zvpice)), ((R(8.87) * (zadd + zbdd)) * zvpice));
      const real zice0 = fmax(zicecld, cl_div_p<real>(c, (zicenuclei * c.riceinit), zrho));
      const real zinew = cl_pow<real>(c, (R(0.666) * zcvds) * c.ptsphy + cl_pow<real>(c, zice0, R(0.666)), R(1.5));
      real zdepos = fmax(za * (zinew - zice0), R(0.0));
      zdepos = fmin(zdepos, zqxfg[QL]);
      const real zinfactor = fmin(cl_div_lit_p<real>(c, zicenuclei, R(15000.0)), R(1.0));
      zdepos = zdepos * fmin(zinfactor + (R(1.0) - zinfactor) * (c.rdepliqrefrate + cl_div_known_p<real>(c, cs.zcldtopdist, c.rdepliqrefdepth, c.rdepliqrefdepth_rcp)), R(1.0));
      sa_li = sa_li + zdepos;
      zqxfg[QI] = zqxfg[QI] + zdepos; zqxfg[QL] = zqxfg[QL] - zdepos;
    }

    // 4. revise in-cloud condensate (:1528-1533)
    ztmpa = cl_div_p<real>(c, R(1.0), fmax(za, zepsec));
    zliqcld = zqxfg[QL] * ztmpa;
    zicecld = zqxfg[QI] * ztmpa;
    zlicld = zliqcld + zicecld;

    CLOUDSC_MID_HOOK(3);
    // 4.2 sedimentation of ice, rain, snow (:1541-1576)
    if (CLOUDSC_RUN(AB_SEDIM) && k > ncldtop0) {
      fsrc_i = cs.pfx_i * zdtgdp; sa_ii = sa_ii + fsrc_i; zqxfg[QI] = zqxfg[QI] + fsrc_i; zqpretot = zqpretot + zqxfg[QI];
      fsrc_r = cs.pfx_r * zdtgdp; sa_rr = sa_rr + fsrc_r; zqxfg[QR] = zqxfg[QR] + fsrc_r; zqpretot = zqpretot + zqxfg[QR];
      fsrc_s = cs.pfx_s * zdtgdp; sa_ss = sa_ss + fsrc_s; zqxfg[QS] = zqxfg[QS] + fsrc_s; zqpretot = zqpretot + zqxfg[QS];
    }
    const real vqx_i = c.laericesed ? R(0.002) * in.pre_ice : pval(c, c.rvice);
    const real fsink_i = zdtgdp * (vqx_i * zrho);
    const real fsink_r = zdtgdp * (c.rvrain * zrho);
    const real fsink_s = zdtgdp * (c.rvsnow * zrho);

    // precip cover overlap, MAX-RAN (:1594-1611)
    real zcovpclr, zraincld, zsnowcld;
    if (CLOUDSC_RUN(AB_SEDIM) && zqpretot > zepsec) {
      cs.zcovptot = R(1.0) - cl_div_p<real>(c, (R(1.0) - cs.zcovptot) * (R(1.0) - fmax(za, cs.a_prev)), (R(1.0) - fmin(cs.a_prev, R(1.0) - R(1.0e-6))));
      cs.zcovptot = fmax(cs.zcovptot, c.rcovpmin);
      zcovpclr = fmax(R(0.0), cs.zcovptot - za);
      zraincld = cl_div_p<real>(c, zqxfg[QR], cs.zcovptot);
      zsnowcld = cl_div_p<real>(c, zqxfg[QS], cs.zcovptot);
      cs.zcovpmax = fmax(cs.zcovptot, cs.zcovpmax);
    } else {
      zraincld = R(0.0); zsnowcld = R(0.0); cs.zcovptot = R(0.0); zcovpclr = R(0.0); cs.zcovpmax = R(0.0);
    }

    const bool cold = ztp1 <= c.rtt;
    // 4.3a autoconversion to snow (:1616-1637)
    if (CLOUDSC_RUN(AB_AUTO) && cold && zicecld > zepsec) {
      real zzco = c.zzco_snow * cl_exp<real>(c, c.rsnowlin2 * (ztp1 - c.rtt));
      real zlcrit = pval(c, c.rlcritsnow);
      if (c.laericeauto) {
        zlcrit = in.picrit_aer;
        zzco = zzco * cl_pow<real>(c, cl_div_p<real>(c, c.rnice, in.pnice), R(0.333));
      }
      const real r = cl_div_p<real>(c, zicecld, zlcrit);
      sb_is = sb_is + zzco * (R(1.0) - cl_exp<real>(c, -(r * r)));
    }
    // 4.3b warm rain, Khairoutdinov and Kogan 2000 (:1644-1761)
    if (CLOUDSC_RUN(AB_AUTO) && zliqcld > zepsec) {
      real zrainaut = R(0.0), zrainacc = R(0.0);
      if (zliqcld > cc.kk_lcrit) {
        zrainaut = ((((R(1.5) * za) * c.ptsphy) * c.rcl_kkaau) * cl_pow<real>(c, zliqcld, c.rcl_kkbauq)) * cc.kk_pow;
        zrainaut = fmin(zrainaut, zqxfg[QL]);
        if (zrainaut < zepsec) zrainaut = R(0.0);
        zrainacc = (((R(2.0) * za) * c.ptsphy) * c.rcl_kkaac) * cl_pow<real>(c, zliqcld * zraincld, c.rcl_kkbac);
        zrainacc = fmin(zrainacc, zqxfg[QL]);
        if (zrainacc < zepsec) zrainacc = R(0.0);
      }
      if (cold) {
        sa_ls = sa_ls + zrainaut; sa_ls = sa_ls + zrainacc;
      } else {
        sa_lr = sa_lr + zrainaut; sa_lr = sa_lr + zrainacc;
      }
    }
    // riming of snow by cloud water (:1768-1808)
    if (CLOUDSC_RUN(AB_AUTO) && cold && zliqcld > zepsec && cs.zcovptot > R(0.01) && zsnowcld > zepsec) {
      const real zfallcorr = cl_pow<real>(c, cl_div_p<real>(c, c.rdensref, zrho), R(0.4));
      real zsnowrime = ((((R(0.3) * cs.zcovptot) * c.ptsphy) * c.rcl_const7s) * zfallcorr) *
                       cl_pow<real>(c, (zrho * zsnowcld) * c.rcl_const1s, c.rcl_const8s);
      zsnowrime = fmin(zsnowrime, R(1.0));
      sb_ls = sb_ls + zsnowrime;
    }

    CLOUDSC_MID_HOOK(4);
    // 4.4a melting of snow and ice (:1817-1859)
    const real zicetot = zqxfg[QI] + zqxfg[QS];
    if (CLOUDSC_RUN(AB_MELT) && zicetot > zepsec && ztp1 > c.rtt) {
      const real zsubsat = fmax(zqsice - zqx[QV], R(0.0));
      const real ztdmtw0 = ztp1 - c.rtt - zsubsat * (ztw1 + ztw2 * (pap_k - ztw3) - ztw4 * (ztp1 - ztw5));
      const real zcons1 = fabs(cl_div_known_p<real>(c, (c.ptsphy * (R(1.0) + R(0.5) * ztdmtw0)), c.rtaumel, c.rtaumel_rcp));
      const real zmeltmax = fmax((ztdmtw0 * zcons1) * c.zrldcp, R(0.0));
      if (zmeltmax > zepsec) {
        {   // ice -> rain
          const real zalfa = cl_div_p<real>(c, zqxfg[QI], zicetot);
          const real zmelt = fmin(zqxfg[QI], zalfa * zmeltmax);
          zqxfg[QI] = zqxfg[QI] - zmelt; zqxfg[QR] = zqxfg[QR] + zmelt;
          sa_ir = sa_ir + zmelt;
        }
        {   // snow -> rain
          const real zalfa = cl_div_p<real>(c, zqxfg[QS], zicetot);
          const real zmelt = fmin(zqxfg[QS], zalfa * zmeltmax);
          zqxfg[QS] = zqxfg[QS] - zmelt; zqxfg[QR] = zqxfg[QR] + zmelt;
          sa_sr = sa_sr + zmelt;
        }
      }
    }

    // 4.4b freezing of rain (:1864-1908)
    if (CLOUDSC_RUN(AB_MELT) && zqx[QR] > zepsec) {
      if (cold && cs.t_prev > c.rtt) {
        const real tot = fmax(zqx[QS] + zqx[QR], zepsec);
        cs.rainfrac = cl_div_p<real>(c, zqx[QR], tot);
      }
      if (ztp1 < c.rtt) {
        real zfrzmax;
        if (cs.rainfrac > R(0.8)) {
          const real zlambda = cl_pow<real>(c, cl_div_p<real>(c, c.rcl_fac1, (zrho * zqx[QR])), c.rcl_fac2);
          const real ztemp = c.rcl_fzrab * (ztp1 - c.rtt);
          const real zfrz = ((c.ptsphy * (cl_div_p<real>(c, c.rcl_const5r, zrho))) * (cl_exp<real>(c, ztemp) - R(1.0))) * cl_pow<real>(c, zlambda, c.rcl_const6r);
          zfrzmax = fmax(zfrz, R(0.0));
        } else {
          const real zcons1 = fabs(cl_div_known_p<real>(c, (c.ptsphy * (R(1.0) + R(0.5) * (c.rtt - ztp1))), c.rtaumel, c.rtaumel_rcp));
          zfrzmax = fmax(((c.rtt - ztp1) * zcons1) * c.zrldcp, R(0.0));
        }
        if (zfrzmax > zepsec) {
          const real zfrz = fmin(zqx[QR], zfrzmax); sa_sr = sa_sr - zfrz;
        }
      }
    }
    // 4.4c freezing of liquid (:1913-1928)
    {
      const real zfrzmax = fmax((c.rthomo - ztp1) * c.zrldcp, R(0.0));
      if (CLOUDSC_RUN(AB_MELT) && zfrzmax > zepsec && zqxfg[QL] > zepsec) {
        const real zfrz = fmin(zqxfg[QL], zfrzmax);
        sa_li = sa_li + zfrz;
      }
    }

    CLOUDSC_MID_HOOK(5);
    // 4.5 evaporation of rain, Abel and Boutle (:1982-2040).  The humidity
    // threshold zzrh0, zqsliq and zqe are pure functions of values fixed by now
    // (cs.zcovpmax is not changed by either evaporation): they are evaluated
    // inside the precipitation tests that guard their only uses, so a wave
    // without rain or snow skips their divisions.  Same operations, same bits.
    auto zzrh0_of = [&]() {
      return fmin(fmax(c.rprecrhmax + cl_div_p<real>(c, ((R(1.0) - c.rprecrhmax) * cs.zcovpmax), r_1mza), c.rprecrhmax), R(1.0));
    };
    if (CLOUDSC_RUN(AB_EVAP) && zcovpclr > zepsec && zqxfg[QR] > zepsec) {
      const real zfoeeliqt = fmin(cl_div_p<real>(c, (c.r2es * e_liq), r_pap), R(0.5));
      const real zqsliq = cl_div_p<real>(c, zfoeeliqt, (R(1.0) - c.retv * zfoeeliqt));
      const real zzrh = fmin(R(0.8), zzrh0_of());
      const real zqe = fmax(R(0.0), fmin(zqx[QV], zqsliq));
      if (zqe < zzrh * zqsliq) {
        const real zpreclr = cl_div_p<real>(c, zqxfg[QR], cs.zcovptot);
        const real zfallcorr = cl_pow<real>(c, cl_div_p<real>(c, c.rdensref, zrho), R(0.4));
        const real zesatliq = c.rv_rd * (c.r2es * e_liq);
        const real zlambda = cl_pow<real>(c, cl_div_p<real>(c, c.rcl_fac1, (zrho * zpreclr)), c.rcl_fac2);
        const real zevap_denom = c.rcl_cdenom1 * zesatliq - c.rcl_cdenom2 * ztp1 * zesatliq + (c.rcl_cdenom3 * cl_pow<real>(c, ztp1, R(3.0))) * pap_k;
        const real zcorr2 = cl_div_p<real>(c, (cl_pow<real>(c, cl_div_lit_p<real>(c, ztp1, R(273.0)), R(1.5)) * R(393.0)), (ztp1 + R(120.0)));
        const real zsubsat = fmax(zzrh * zqsliq - zqe, R(0.0));
        const real zbeta = ((((cl_div_p<real>(c, R(0.5), zqsliq)) * (ztp1 * ztp1)) * zesatliq) * c.rcl_const1r) * (cl_div_p<real>(c, zcorr2, zevap_denom)) *
                           (cl_div_p<real>(c, R(0.78), cl_pow<real>(c, zlambda, c.rcl_const4r)) + cl_div_p<real>(c, (c.rcl_const2r * cl_sqrt_p<real>(c, zrho * zfallcorr)), (cl_sqrt_p<real>(c, zcorr2) * cl_pow<real>(c, zlambda, c.rcl_const3r))));
        const real zdenom = R(1.0) + zbeta * c.ptsphy;
        const real zdpevap = cl_div_p<real>(c, (((zcovpclr * zbeta) * c.ptsphy) * zsubsat), zdenom);
        const real zevap = fmin(zdpevap, zqxfg[QR]);
        sa_rv = sa_rv + zevap;
        cs.zcovptot = fmax(c.rcovpmin, cs.zcovptot - fmax(R(0.0), cl_div_p<real>(c, ((cs.zcovptot - za) * zevap), zqxfg[QR])));
        zqxfg[QR] = zqxfg[QR] - zevap;
      }
    }
    // 4.5 evaporation of snow, Sundqvist (:2048-2087)
    if (CLOUDSC_RUN(AB_EVAP) && zcovpclr > zepsec && zqxfg[QS] > zepsec) {
      const real zzrh = zzrh0_of();
      real zqe = cl_div_p<real>(c, (zqx[QV] - za * zqsice), r_1mza);
      zqe = fmax(R(0.0), fmin(zqe, zqsice));
      if (zqe < zzrh * zqsice) {
        const real x = cs.zcovptot * zdtgdp;
        const real zpreclr = cl_div_p<real>(c, (zqxfg[QS] * zcovpclr), copysign(fmax(fabs(x), zepsilon), x));
        const real zbeta1 = cl_div_p<real>(c, ((cl_div_known_p<real>(c, cl_sqrt_p<real>(c, cl_div_p<real>(c, pap_k, cc.paph_sfc)), c.rvrfactor, c.rvrfactor_rcp)) * zpreclr), fmax(zcovpclr, zepsec));
        const real zbeta = c.rg_rpecons * cl_pow<real>(c, zbeta1, R(0.5777));
        const real zdenom = R(1.0) + (zbeta * c.ptsphy) * zcorqsice;
        const real zdpr = ((cl_div_p<real>(c, ((zcovpclr * zbeta) * (zqsice - zqe)), zdenom)) * zdp) * c.zrg_r;
        const real zdpevap = zdpr * zdtgdp;
        const real zevap = fmin(zdpevap, zqxfg[QS]);
        sa_sv = sa_sv + zevap;
        cs.zcovptot = fmax(c.rcovpmin, cs.zcovptot - fmax(R(0.0), cl_div_p<real>(c, ((cs.zcovptot - za) * zevap), zqxfg[QS])));
        zqxfg[QS] = zqxfg[QS] - zevap;
      }
    }
    // evaporate small precipitation amounts (:2144-2158)
    if (zqxfg[QR] < c.rlmin) { sa_rv = sa_rv + zqxfg[QR]; }
    if (zqxfg[QS] < c.rlmin) { sa_sv = sa_sv + zqxfg[QS]; }

    // 5.1 cloud cover (:2168-2180)
    real zanew = cl_div_p<real>(c, (za + zsolac), (R(1.0) + zsolab));
    zanew = fmin(zanew, R(1.0));
    if (zanew < c.ramin) zanew = R(0.0);
    const real zda = zanew - zaorig;
    cs.zanewm1 = zanew;
    // the hook: the k-caching kernel issues the next level's first-consumed
    // loads here (PF 3), after the physics' peak of live temporaries
    CLOUDSC_MID_HOOK(0);

    // 5.2 truncate explicit sinks, species in order (:2233-2286).
    // Column m of zsolqa (zsolqa[n][m], n=0..4) in C indexing; for each m the
    // sum runs n = ql, qi, qr, qs, qv and every negative entry scales
    // zsolqa[n][m] and its transpose zsolqa[m][n] (the diagonal twice).
    // The structurally-zero entries are kept as literal zeros so the
    // summation order (and hence rounding) matches the dense reference.
    // Where the sinks do not exceed what is there, max(-psum, zmm) is zmm and
    // the reference's ratio zmm/zmm is exactly 1 (zmm >= zepsec, finite): its
    // scaling multiplies by 1 and changes no bit, so the division and the
    // scaling run only where they can change something (a wave skips them
    // when none of its columns needs them).
    {
      real z = R(0.0), psum, zrat;
      // m = ql: zsolqa[n][ql] = {ll, il, rl, sl, vl}
      psum = R(0.0) + sa_ll; psum = psum + (-sa_li); psum = psum + (-sa_lr); psum = psum + (-sa_ls); psum = psum + (-sa_lv);
      {
        const real zmm = fmax(zqx[QL], zepsec), den = fmax(R(0.0) - psum, zmm);
        if (CLOUDSC_RUN(AB_TRUNC) && (den != zmm || zmm == (real)__builtin_inf())) {   // else zrat = 1: identity
          zrat = cl_div_p<real>(c, zmm, den);
          if (sa_ll < R(0.0)) { sa_ll = sa_ll * zrat; sa_ll = sa_ll * zrat; }
          if (-sa_li < R(0.0)) sa_li = sa_li * zrat;
          if (-sa_lr < R(0.0)) sa_lr = sa_lr * zrat;
          if (-sa_ls < R(0.0)) sa_ls = sa_ls * zrat;
          if (-sa_lv < R(0.0)) sa_lv = sa_lv * zrat;
        }
      }
      // m = qi: {li, ii, ri, si(0), vi}
      psum = R(0.0) + sa_li; psum = psum + sa_ii; psum = psum + (-sa_ir); psum = psum + z; psum = psum + (-sa_iv);
      {
        const real zmm = fmax(zqx[QI], zepsec), den = fmax(R(0.0) - psum, zmm);
        if (CLOUDSC_RUN(AB_TRUNC) && (den != zmm || zmm == (real)__builtin_inf())) {   // else zrat = 1: identity
          zrat = cl_div_p<real>(c, zmm, den);
          if (sa_li < R(0.0)) sa_li = sa_li * zrat;
          if (sa_ii < R(0.0)) { sa_ii = sa_ii * zrat; sa_ii = sa_ii * zrat; }
          if (-sa_ir < R(0.0)) sa_ir = sa_ir * zrat;
          if (-sa_iv < R(0.0)) sa_iv = sa_iv * zrat;
        }
      }
      // m = qr: {lr, ir, rr, sr, vr}
      psum = R(0.0) + sa_lr; psum = psum + sa_ir; psum = psum + sa_rr; psum = psum + sa_sr; psum = psum + (-sa_rv);
      {
        const real zmm = fmax(zqx[QR], zepsec), den = fmax(R(0.0) - psum, zmm);
        if (CLOUDSC_RUN(AB_TRUNC) && (den != zmm || zmm == (real)__builtin_inf())) {   // else zrat = 1: identity
          zrat = cl_div_p<real>(c, zmm, den);
          if (sa_lr < R(0.0)) sa_lr = sa_lr * zrat;
          if (sa_ir < R(0.0)) sa_ir = sa_ir * zrat;
          if (sa_rr < R(0.0)) { sa_rr = sa_rr * zrat; sa_rr = sa_rr * zrat; }
          if (sa_sr < R(0.0)) sa_sr = sa_sr * zrat;
          if (-sa_rv < R(0.0)) sa_rv = sa_rv * zrat;
        }
      }
      // m = qs: {ls, is(0), rs, ss, vs}
      psum = R(0.0) + sa_ls; psum = psum + z; psum = psum + (-sa_sr); psum = psum + sa_ss; psum = psum + (-sa_sv);
      {
        const real zmm = fmax(zqx[QS], zepsec), den = fmax(R(0.0) - psum, zmm);
        if (CLOUDSC_RUN(AB_TRUNC) && (den != zmm || zmm == (real)__builtin_inf())) {   // else zrat = 1: identity
          zrat = cl_div_p<real>(c, zmm, den);
          if (sa_ls < R(0.0)) sa_ls = sa_ls * zrat;
          if (-sa_sr < R(0.0)) sa_sr = sa_sr * zrat;
          if (sa_ss < R(0.0)) { sa_ss = sa_ss * zrat; sa_ss = sa_ss * zrat; }
          if (-sa_sv < R(0.0)) sa_sv = sa_sv * zrat;
        }
      }
      // m = qv: {lv, iv, rv, sv, vv(0)}
      psum = R(0.0) + sa_lv; psum = psum + sa_iv; psum = psum + sa_rv; psum = psum + sa_sv; psum = psum + z;
      {
        const real zmm = fmax(zqx[QV], zepsec), den = fmax(R(0.0) - psum, zmm);
        if (CLOUDSC_RUN(AB_TRUNC) && (den != zmm || zmm == (real)__builtin_inf())) {   // else zrat = 1: identity
          zrat = cl_div_p<real>(c, zmm, den);
          if (sa_lv < R(0.0)) sa_lv = sa_lv * zrat;
          if (sa_iv < R(0.0)) sa_iv = sa_iv * zrat;
          if (sa_rv < R(0.0)) sa_rv = sa_rv * zrat;
          if (sa_sv < R(0.0)) sa_sv = sa_sv * zrat;
        }
      }
    }

    // 5.2.2 implicit solver (:2294-2397).  With the zsolqb sparsity above,
    //   zqlhs = I + diag(fallsink) + diag(row sums of zsolqb) - offdiag(zsolqb)
    // has off-diagonal entries only at [ql][qs] and [qi][qs] (C indexing), so
    // the unpivoted LU leaves every multiplier but those two at (signed) zero
    // and the forward/back substitutions reduce to the terms below.  The
    // skipped updates are x - (+/-0)*y == x exactly, so the results are
    // bit-identical to the dense elimination for finite data.
    {
      // RHS: zqxn[m] = zqx[m] + sum_n zsolqa[n][m], n ascending from 0.0
      real ex;
      ex = R(0.0) + sa_ll; ex = ex + (-sa_li); ex = ex + (-sa_lr); ex = ex + (-sa_ls); ex = ex + (-sa_lv);
      real qn_l = zqx[QL] + ex;
      ex = R(0.0) + sa_li; ex = ex + sa_ii; ex = ex + (-sa_ir); ex = ex + R(0.0); ex = ex + (-sa_iv);
      real qn_i = zqx[QI] + ex;
      ex = R(0.0) + sa_lr; ex = ex + sa_ir; ex = ex + sa_rr; ex = ex + sa_sr; ex = ex + (-sa_rv);
      real qn_r = zqx[QR] + ex;
      ex = R(0.0) + sa_ls; ex = ex + R(0.0); ex = ex + (-sa_sr); ex = ex + sa_ss; ex = ex + (-sa_sv);
      real qn_s = zqx[QS] + ex;
      ex = R(0.0) + sa_lv; ex = ex + sa_iv; ex = ex + sa_rv; ex = ex + sa_sv; ex = ex + R(0.0);
      real qn_v = zqx[QV] + ex;
      // LHS diagonal: 1 + fallsink + sum_o zsolqb[m][o] (o ascending)
      real d_l = R(1.0) + R(0.0);
      d_l = d_l + sb_ll; d_l = d_l + R(0.0); d_l = d_l + R(0.0); d_l = d_l + sb_ls; d_l = d_l + R(0.0);
      real d_i = R(1.0) + fsink_i;
      d_i = d_i + R(0.0); d_i = d_i + sb_ii; d_i = d_i + R(0.0); d_i = d_i + sb_is; d_i = d_i + R(0.0);
      const real d_r = R(1.0) + fsink_r;   // + five zeros
      const real d_s = R(1.0) + fsink_s;
      // off-diagonals zqlhs[ql][qs] = -sb_ls, zqlhs[qi][qs] = -sb_is; LU scales row-wise by
      // the pivot of the eliminating column: zqlhs[n][m] /= zqlhs[n][n] for m > n.
      const Recip<real> r_dl = cl_recip_p<real>(c, d_l), r_di = cl_recip_p<real>(c, d_i);
      const real u_ls = cl_div_p<real>(c, (-sb_ls), r_dl);    // zqlhs[ql][qs] after jn = ql
      const real u_is = cl_div_p<real>(c, (-sb_is), r_di);    // zqlhs[qi][qs] after jn = qi
      // forward substitution (step 1): zqxn[qs] -= zqlhs[ql][qs]*zqxn[ql] + zqlhs[qi][qs]*zqxn[qi]
      qn_s = qn_s - u_ls * qn_l;
      qn_s = qn_s - u_is * qn_i;
      // back substitution (step 2): vapour and the diagonal solves
      // qn_v = qn_v / zqlhs[qv][qv] with a pivot of exactly 1: x / 1 == x in IEEE arithmetic
      // (signed zeros and NaN included), so the division is dropped
      if (CLOUDSC_RUN(AB_SOLVE)) {
        qn_s = cl_div_p<real>(c, qn_s, d_s);
        qn_r = cl_div_p<real>(c, qn_r, d_r);
        qn_i = cl_div_p<real>(c, qn_i, r_di);
        qn_l = cl_div_p<real>(c, qn_l, r_dl);
      }
      // no small values (:2402-2412)
      if (qn_l < zepsec) { qn_v = qn_v + qn_l; qn_l = R(0.0); }
      if (qn_i < zepsec) { qn_v = qn_v + qn_i; qn_i = R(0.0); }
      if (qn_r < zepsec) { qn_v = qn_v + qn_r; qn_r = R(0.0); }
      if (qn_s < zepsec) { qn_v = qn_v + qn_s; qn_s = R(0.0); }
      zqxn[QL] = qn_l; zqxn[QI] = qn_i; zqxn[QR] = qn_r; zqxn[QS] = qn_s;
      cs.qxnm1_l = qn_l; cs.qxnm1_i = qn_i;

      // 5.3 precipitation fluxes to the next level (:2430-2448)
      cs.pfx_i = (fsink_i * qn_i) * zrdtgdp;
      cs.pfx_r = (fsink_r * qn_r) * zrdtgdp;
      cs.pfx_s = (fsink_s * qn_s) * zrdtgdp;
      if (cs.pfx_s + cs.pfx_r < zepsec) cs.zcovptot = R(0.0);

      // 6. tendencies (:2456-2506)
      {
        const real fq_l = psup_l + conv_src_l + R(0.0) - (R(0.0) + conv_sink) * qn_l;
        ttend = ttend + (c.ralvdcp * (qn_l - zqx[QL] - fq_l)) * c.zqtmst;
        const real fq_i = psup_i + conv_src_i + fsrc_i - (fsink_i + conv_sink) * qn_i;
        ttend = ttend + (c.ralsdcp * (qn_i - zqx[QI] - fq_i)) * c.zqtmst;
        const real fq_r = R(0.0) + R(0.0) + fsrc_r - (fsink_r + R(0.0)) * qn_r;
        ttend = ttend + (c.ralvdcp * (qn_r - zqx[QR] - fq_r)) * c.zqtmst;
        const real fq_s = R(0.0) + R(0.0) + fsrc_s - (fsink_s + R(0.0)) * qn_s;
        ttend = ttend + (c.ralsdcp * (qn_s - zqx[QS] - fq_s)) * c.zqtmst;
      }
  #pragma unroll
      for (int m = 0; m < 4; m++) ctend[m] = R(0.0) + (zqxn[m] - zqx0[m]) * c.zqtmst;
      qtend = qtend + (qn_v - zqx[QV]) * c.zqtmst;
      atend = R(0.0) + zda * c.zqtmst;
      po.zcovptot_out = cs.zcovptot;
    }
}

// ===== 8. flux diagnostics of one level (cloudsc_c.c:2521-2582), written at half level k+1 =====
template <typename real, typename P, typename CS>
CLOUDSC_HD void flux_level(const P& c, const KArgs<real>& A, size_t h, unsigned lo,
                                           const LevelIn<real>& in, const LevelState<real>& ls,
                                           const PhysOut<real>& po, real paph_k, real paph_n,
                                           CS& cs) {
  const real zgdph_r = -c.zrg_r * (paph_n - paph_k) * c.zqtmst;
  const real lf = cs.fl_lf, fi = cs.fl_if, lng = cs.fl_lng, nng = cs.fl_nng;
  const real* zqxn = po.zqxn;
  const real* zqx0 = ls.zqx0;
  const real* zlneg = ls.zlneg;
  const real plude_k = po.plude_k, zfoealfa = ls.zfoealfa;
  cs.fl_lf = lf + (zqxn[QL] - zqx0[QL] + in.pvfl * c.ptsphy - zfoealfa * plude_k) * zgdph_r;
  cs.fl_lng = lng + zlneg[QL] * zgdph_r;
  cs.fl_ltur = cs.fl_ltur + (in.pvfl * c.ptsphy) * zgdph_r;
  const real rf = lf + (zqxn[QR] - zqx0[QR]) * zgdph_r;
  const real rng = lng + zlneg[QR] * zgdph_r;
  cs.fl_if = fi + (zqxn[QI] - zqx0[QI] + in.pvfi * c.ptsphy - (R(1.0) - zfoealfa) * plude_k) * zgdph_r;
  cs.fl_nng = nng + zlneg[QI] * zgdph_r;
  cs.fl_itur = cs.fl_itur + (in.pvfi * c.ptsphy) * zgdph_r;
  const real sf = fi + (zqxn[QS] - zqx0[QS]) * zgdph_r;
  const real sng = nng + zlneg[QS] * zgdph_r;
  stg(A.pfsqlf, h, lo, cs.fl_lf); stg(A.pfsqif, h, lo, cs.fl_if);
  stg(A.pfcqlng, h, lo, cs.fl_lng); stg(A.pfcqnng, h, lo, cs.fl_nng);
  stg(A.pfsqltur, h, lo, cs.fl_ltur); stg(A.pfsqitur, h, lo, cs.fl_itur);
  stg(A.pfsqrf, h, lo, rf); stg(A.pfcqrng, h, lo, rng); stg(A.pfsqsf, h, lo, sf); stg(A.pfcqsng, h, lo, sng);
  const real plsl = cs.pfx_r + R(0.0);      // zpfplsx[qr] + zpfplsx[ql] (ql flux is +0)
  const real plsn = cs.pfx_s + cs.pfx_i;
  stg(A.pfplsl, h, lo, plsl); stg(A.pfplsn, h, lo, plsn);
  stg(A.pfhpsl, h, lo, -c.rlvtt * plsl); stg(A.pfhpsn, h, lo, -c.rlstt * plsn);
}

// level-0 half-level outputs (cloudsc_c.c:2523-2543, 2578-2579)
template <typename real, typename P>
CLOUDSC_HD void flux_top(const P& c, const KArgs<real>& A, size_t h0, unsigned lo) {
  stg(A.pfsqlf, h0, lo, R(0.0)); stg(A.pfsqif, h0, lo, R(0.0)); stg(A.pfsqrf, h0, lo, R(0.0));
  stg(A.pfsqsf, h0, lo, R(0.0)); stg(A.pfcqlng, h0, lo, R(0.0)); stg(A.pfcqnng, h0, lo, R(0.0));
  stg(A.pfcqrng, h0, lo, R(0.0)); stg(A.pfcqsng, h0, lo, R(0.0));
  stg(A.pfsqltur, h0, lo, R(0.0)); stg(A.pfsqitur, h0, lo, R(0.0));
  const real plsl = R(0.0) + R(0.0), plsn = R(0.0) + R(0.0);
  stg(A.pfplsl, h0, lo, plsl); stg(A.pfplsn, h0, lo, plsn);
  stg(A.pfhpsl, h0, lo, -c.rlvtt * plsl); stg(A.pfhpsn, h0, lo, -c.rlstt * plsn);
}

template <typename real, typename P>
CLOUDSC_HD ColConst<real> column_constants(const P& c, const KArgs<real>& A,
                                                           size_t u1, size_t uh, unsigned lo) {
  ColConst<real> cc;
  const real plsm = ldg(A.plsm, u1, lo);
  cc.ktype = ldg(A.ktype, u1, lo * (unsigned)(sizeof(int)) / (unsigned)sizeof(real));
  cc.paph_sfc = ldg(A.paph, uh + (size_t)A.klev * A.nproma, lo);
  const bool land = plsm > R(0.5);
  cc.kk_const = land ? pval(c, c.rcl_kk_cloud_num_land) : pval(c, c.rcl_kk_cloud_num_sea);
  cc.kk_lcrit = land ? pval(c, c.rclcrit_land) : pval(c, c.rclcrit_sea);
  cc.kk_pow = cl_pow<real>(c, cc.kk_const, c.rcl_kkbaun);   // loop-invariant factor of the KK autoconversion (:1721)
  return cc;
}

template <typename real>
CLOUDSC_HD void store_level(const KArgs<real>& A, size_t u2, size_t u3, int k, int klev,
                                            int nproma, unsigned lo, bool physics, const LevelState<real>& ls,
                                            const PhysOut<real>& po) {
  const size_t i = u2 + (size_t)k * nproma;
  stg(A.tlt, i, lo, ls.ttend);
  stg(A.tlq, i, lo, ls.qtend);
  stg(A.tla, i, lo, po.atend);
  stg(A.pcovptot, i, lo, po.zcovptot_out);
  stg(A.plude, i, lo, po.plude_k);   // INOUT: rewritten unchanged where not rescaled (no branch on a store)
#pragma unroll
  for (int m = 0; m < 4; m++) stg_sp(A.tlcld, u3 + ((size_t)m * klev + k) * nproma, lo, po.ctend[m]);
  stg_sp(A.tlcld, u3 + ((size_t)4 * klev + k) * nproma, lo, R(0.0));
}

template <typename real, typename CS>
CLOUDSC_HD void init_carry(CS& cs) {
  cs.t_prev = cs.a_prev = cs.pap_prev = R(0.0);
  cs.zanewm1 = cs.zcovptot = cs.zcovpmax = cs.zcldtopdist = cs.rainfrac = R(0.0);
  cs.qxnm1_l = cs.qxnm1_i = R(0.0);
  cs.pfx_i = cs.pfx_r = cs.pfx_s = R(0.0);
  cs.fl_lf = cs.fl_if = cs.fl_lng = cs.fl_nng = cs.fl_ltur = cs.fl_itur = R(0.0);
}

// The level loop's parameter block: the VGPR copy (fp32) or the constant-space
// block read with scalar loads (laundered: loads issued where used).
template <bool PVR, typename PV, typename PT>
__device__ __forceinline__ const auto& params_here(const PV& pv, cptr<PT> cpar) {
  if constexpr (PVR) return pv;
  else return *(const PT*)launder_uniform(cpar);
}

// ===================== SCC-k-caching kernel body =====================
// `ka` points at the kernel's KArgs in the kernarg segment and `cpar` at the
// __constant__ parameter block, both in the constant address space; they are
// re-laundered every level so that scalar loads are issued where needed.
// PF selects the load schedule: 1 = level k+1 prefetched into registers while
// level k computes; 0 = loads issued at the top of their own level.
//
// kcache_levels runs levels [lev0, lev1) of block b for one (active) lane with
// the carried state `cs`; the plain kernel runs [0, klev) in one go, the
// persistent kernel (below) runs a column in level segments.
template <typename real, int PF, bool AER, typename PT, typename CS>
__device__ __forceinline__ void kcache_levels(cptr<KArgs<real>> ka, cptr<PT> cpar, int b,
                                              unsigned lo0, int lev0, int lev1, CS& cs) {
  if (lev0 >= lev1) return;
  const unsigned lo = lo0;                         // empty segment: no loads at lev0 (may be == klev)
  // PF: 0 = loads at the top of their level, 1 = level k+1 prefetched into
  // registers, 2 = like 0, and the neighbour-level values (paph/pmfu/pmfd/plu of
  // k, k+1) re-read every level instead of carried (fewer live registers,
  // more L2 traffic)
  // 3 = the first-consumed inputs of level k+1 (EarlyIn) issued in the middle
  // of level k (the physics' mid hook), the rest at the top of level k+1;
  // 4 = all inputs of level k+1 issued in the middle of level k
  constexpr bool PFX = PF == 1, NBR = PF == 2, PFM = PF == 3, PFA = PF == 4;
  const KArgs<real>& A0 = *(const KArgs<real>*)ka;
  const int nproma = A0.nproma, klev = A0.klev;
  const size_t u1 = (size_t)b * nproma;                            // [nblocks][nproma]
  const size_t u2 = (size_t)b * klev * nproma;                     // [nblocks][klev][nproma]
  const size_t uh = (size_t)b * (klev + 1) * nproma;               // [nblocks][klev+1][nproma]
  const size_t u3 = (size_t)b * 5 * klev * nproma;                 // [nblocks][5][klev][nproma]

  ColConst<real> cc;
  Neighbors<real> nb;
  LevelIn<real> cur, nxt;
  EarlyIn<real> nxt_e;
  int ncldtop0;
  {
    CLOUDSC_PARAMS_HERE;
    const KArgs<real>& A = A0;
    ncldtop0 = c.ncldtop - 1;
    cc = column_constants(c, A, u1, uh, lo);
    const int l1 = lev0 + 1 < klev ? lev0 + 1 : klev - 1;
    nb.paph_k = ldg(A.paph, uh + (size_t)lev0 * nproma, lo);
    nb.paph_n = ldg(A.paph, uh + (size_t)(lev0 + 1) * nproma, lo);
    nb.pmfu_k = ldg(A.pmfu, u2 + (size_t)lev0 * nproma, lo);
    nb.pmfd_k = ldg(A.pmfd, u2 + (size_t)lev0 * nproma, lo);
    nb.pmfu_n = ldg(A.pmfu, u2 + (size_t)l1 * nproma, lo);
    nb.pmfd_n = ldg(A.pmfd, u2 + (size_t)l1 * nproma, lo);
    nb.plu_n = ldg(A.plu, u2 + (size_t)l1 * nproma, lo);
    if (PFX) load_level<real, AER>(cur, A, u2, u3, lev0, klev, nproma, lo);
    if (PFM) load_early<real>(nxt_e, A, u2, u3, lev0, klev, nproma, lo);
    if (PFA) load_level<real, AER>(nxt, A, u2, u3, lev0, klev, nproma, lo);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // PF 1: drain the prologue's loads once (per segment) before the level loop.
  // The level-(k+1) prefetch at the top of each level first copies the previous
  // prefetch (cur = nxt); the waitcnt pass merges the loop header's two entries
  // (prologue, latch) conservatively and then made EVERY level wait for part of
  // the loads it had just issued -- a full memory round trip per level.  With
  // the prologue drained, the header needs no vmcnt wait: fp32 KSEG -3.7 %
  // (profiles/r03/experiment_prologue_drain_ab.txt).  (PF 3, the fp64 default,
  // measured neutral and keeps its schedule.)
  if constexpr (PFX) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt(7), lgkmcnt(15)
#endif

  // fp32: the parameter block copied into VGPRs once per call (each value an
  // opaque per-lane copy), so the level loop reads every parameter from a
  // register instead of a scalar load + lgkmcnt(0) wait at each use -- 5 %
  // (profiles/r03/experiment_fp32_params_in_vgprs_ab.txt).  fp32 has the
  // registers for it (~95 VGPRs on top of ~155 at 2 waves/SIMD); fp64 would
  // need twice as many and keeps the scalar loads.
  constexpr bool PVR = sizeof(real) == 4;
  using PV = typename std::conditional<PVR, typename WithVgprParams<PT>::type, PT>::type;
  PV pv;
  if constexpr (PVR) {
    pv = *(const PV*)(const PT*)cpar;
    float* q = (float*)&pv;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(PV) / sizeof(float)) - 4; i++) asm volatile("" : "+v"(q[i]));   // not the 4 ints
  }
  for (int kloop = lev0; kloop < lev1; kloop++) {
    // the level index is laundered too, so no per-field induction pointers are formed
    int k = kloop;
    asm volatile("" : "+s"(k));
    // and so is the lane's 32-bit byte offset: its zero-extension is then formed
    // in this block, where the level loads fold it into the saddr + voffset form
    // instead of a 64-bit VGPR address add per load
    const unsigned lo = launder_vgpr(lo0);
    const bool physics = k >= ncldtop0;
    // ---- issue the loads of the next levels (software pipelining) ----
    real paph_nn, pmfu_nn, pmfd_nn, plu_nn;
    {
      const KArgs<real>& A = *(const KArgs<real>*)launder_uniform(ka);
      // indices clamped instead of branched: the last levels re-read valid data
      const int k1 = k + 1 < klev ? k + 1 : klev - 1;
      const int k2 = k + 2 < klev ? k + 2 : klev - 1;
      const int kh2 = k + 2 < klev + 1 ? k + 2 : klev;
      if (!PFX && !PFM && !PFA) load_level<real, AER>(cur, A, u2, u3, k, klev, nproma, lo);
      if (PFA) cur = nxt;
      if (PFM) {
        load_late<real, AER>(cur, A, u2, k, nproma, lo);
        take_early(cur, nxt_e);
      }
      if (PFX) load_level<real, AER>(nxt, A, u2, u3, k1, klev, nproma, lo);
      if (NBR) {
        nb.paph_k = ldg(A.paph, uh + (size_t)k * nproma, lo);
        nb.paph_n = ldg(A.paph, uh + (size_t)(k + 1) * nproma, lo);
        const size_t i0 = u2 + (size_t)k * nproma, i1 = u2 + (size_t)k1 * nproma;
        nb.pmfu_k = ldg(A.pmfu, i0, lo); nb.pmfd_k = ldg(A.pmfd, i0, lo);
        nb.pmfu_n = ldg(A.pmfu, i1, lo); nb.pmfd_n = ldg(A.pmfd, i1, lo); nb.plu_n = ldg(A.plu, i1, lo);
        paph_nn = pmfu_nn = pmfd_nn = plu_nn = R(0.0);
      } else {
        // read once each (levels k+2 rotate through registers): streaming loads,
        // -0.4 % fp64 / -0.7 % fp32 against cached ones (profiles/r05/experiments_kernel_ab.txt)
        paph_nn = ldg1(A.paph, uh + (size_t)kh2 * nproma, lo);
        const size_t i2 = u2 + (size_t)k2 * nproma;
        pmfu_nn = ldg1(A.pmfu, i2, lo); pmfd_nn = ldg1(A.pmfd, i2, lo); plu_nn = ldg1(A.plu, i2, lo);
      }
    }

    LevelState<real> ls;
    PhysOut<real> po;
    {
      const auto& c = params_here<PVR>(pv, cpar);
      init_level(c, cur, ls);
#pragma unroll
      for (int m = 0; m < 4; m++) { po.zqxn[m] = R(0.0); po.ctend[m] = R(0.0); }
      po.plude_k = cur.plude;
      po.atend = R(0.0);
      po.zcovptot_out = R(0.0);
      // PF 3: the next level's early inputs, issued in the middle of this level
      // (clamped at the last level: a re-read of valid data, never consumed)
      const auto mid = [&]() {
        if (PFM || PFA) {
          const int k1 = k + 1 < klev ? k + 1 : klev - 1;
          if (PFM)
            load_early<real>(nxt_e, *(const KArgs<real>*)launder_uniform(ka), u2, u3, k1, klev, nproma,
                             launder_vgpr(lo0));
          else
            load_level<real, AER>(nxt, *(const KArgs<real>*)launder_uniform(ka), u2, u3, k1, klev, nproma,
                                  launder_vgpr(lo0));
        }
      };
#ifndef CLOUDSC_ABLATE_PHYSICS   // timing-only diagnostic build: the level loop without sections 3-6
      if (physics) physics_level(c, k, klev, ncldtop0, cur, nb, cc, ls, cs, po, mid);
      else mid();
#else                            // (every load kept alive, so the bytes moved are the same)
      asm volatile("" :: "v"(cur.phrsw), "v"(cur.phrlw), "v"(cur.pvervel), "v"(cur.psnde), "v"(cur.psupsat),
                   "v"(nb.pmfu_k), "v"(nb.pmfd_k), "v"(nb.plu_n), "v"(cc.kk_pow));
      asm volatile("" :: "v"(cur.pclv[0]), "v"(cur.pclv[1]), "v"(cur.pclv[2]), "v"(cur.pclv[3]),
                   "v"(cur.ttcld[0]), "v"(cur.ttcld[1]), "v"(cur.ttcld[2]), "v"(cur.ttcld[3]));
      mid();
#endif
    }
    {
      const KArgs<real>& A = *(const KArgs<real>*)launder_uniform(ka);
      const auto& c = params_here<PVR>(pv, cpar);
      const unsigned los = PVR ? launder_vgpr(lo0) : lo;
      store_level(A, u2, u3, k, klev, nproma, los, physics, ls, po);
      flux_level(c, A, uh + (size_t)(k + 1) * nproma, los, cur, ls, po, nb.paph_k, nb.paph_n, cs);
    }

    // ---- rotate carried state ----
    cs.t_prev = ls.ztp1; cs.a_prev = ls.za; cs.pap_prev = cur.pap;
    if (!NBR) {
      nb.paph_k = nb.paph_n; nb.paph_n = paph_nn;
      nb.pmfu_k = nb.pmfu_n; nb.pmfd_k = nb.pmfd_n;
      nb.pmfu_n = pmfu_nn; nb.pmfd_n = pmfd_nn; nb.plu_n = plu_nn;
    }
    if (PFX) cur = nxt;
  }
}

// carried state in registers (LDSC = false) or in LDS (LDSC = true)
template <typename real>
struct CarryRegs : CarryState<real> {
  __device__ __forceinline__ explicit CarryRegs(CLOUDSC_AS3 real*) {}
};
template <typename real, bool LDSC>
using CarryOf = typename std::conditional<LDSC, CarryLds<real>, CarryRegs<real>>::type;

template <typename real, int PF, bool AER, bool LDSC, typename PT>
__device__ __forceinline__ void cloudsc_kcache_body(cptr<KArgs<real>> ka, cptr<PT> cpar) {
  const KArgs<real>& A = *(const KArgs<real>*)ka;
  const int b = blockIdx.x, jl = threadIdx.x;
  if (jl >= A.nproma || b * A.nproma + jl >= A.ngptot) return;
  const unsigned lo = (unsigned)jl * (unsigned)sizeof(real);
  CarryOf<real, LDSC> cs(carry_lds_base<real>());
  init_carry<real>(cs);
  {
    CLOUDSC_PARAMS_HERE;
    flux_top(c, A, (size_t)b * (A.klev + 1) * A.nproma, lo);
  }
  kcache_levels<real, PF, AER>(ka, cpar, b, lo, 0, A.klev, cs);
  stg(((const KArgs<real>*)launder_uniform(ka))->prainfrac, (size_t)b * A.nproma, lo, cs.rainfrac);
}

// ===================== persistent (work-queue) SCC-k-caching =====================
// Each column's level loop is cut into NSEG segments; an item is (segment s,
// block b), dequeued in order s-major from an atomic counter.  Segment s of
// block b waits for segment s-1 of b (flag[b] >= s) and resumes from the carried
// state it left in HBM ([nblocks][kCarryN][nproma], 19 values per column), so
// the result is bit-identical to the one-shot kernel.  Dequeue order guarantees
// progress: an item's predecessor was dequeued earlier by a running workgroup.
// The point: 2560 waves on 2048 wave slots leave the second round 75 % idle;
// with NSEG segments the tail shrinks to a fraction of a segment.
constexpr int kCarryN = 19;
constexpr int kMaxSeg = 16;
// Dequeue stripes (round 4): the items are split into kKsegStripes independent
// queues -- stripe s holds every segment of the blocks b with b % nstripes == s,
// in the same (segment, block, sub-block) order -- each with its own counter on
// its own 128-byte line, and workgroup w takes its items from stripe
// w % nstripes (the round-robin dispatch puts it on XCD w % 8).  At start-up
// 2048 workgroups then queue on 8 counters instead of one (round 3: the last
// first item began 23 us after the first).  Progress needs no residency: within
// a stripe items are dequeued in order, so an item's predecessor (the same
// block's previous segment, same stripe) was dequeued earlier by a running
// workgroup.  A stripe's counter advances by exactly its items plus the
// workgroups of the stripe per launch (each takes one ticket past the end).
constexpr int kKsegStripes = 8;
constexpr int kKsegCtrStride = 32;   // words between stripe counters (128 B)

#ifdef CLOUDSC_KSEG_TRACE
constexpr int kTraceMax = 1 << 16;
__device__ unsigned long long g_kseg_trace[4 * kTraceMax];
#endif

template <typename real>
struct PersistArgs {
  // The workspace is zeroed before the first launch on it; later launches on
  // the same workspace (a state's steps) need no zeroing: each launch takes
  // exactly nitems + grid tickets, so the host passes the counter's value at
  // its start (base), and flags are stamped per launch (stamp + segments done;
  // an older launch's flag compares as "not yet": signed difference).
  unsigned* ctr;          // stripe s's dequeue counter at ctr[s * kKsegCtrStride]: its tickets are
                          // base[s], base[s] + 1, ...
  unsigned* flags;        // [nblocks * nsub] stamp + segments completed
  unsigned* err;          // spin-limit violations (sticky until read, cloudsc_gpu_check)
  unsigned base[kKsegStripes];   // 0 right after zeroing
  unsigned stamp;         // 0 right after zeroing
  int nstripes;           // 1..kKsegStripes, <= grid
  real* state;            // [nblocks][kCarryN][nproma]
  int nseg, nitems, nblocks;
  int nsub;               // 64-column sub-blocks per NPROMA block (one wave each)
  int sb_major;           // item order (segment, sub-block, block) instead of (segment, block, sub-block)
  unsigned spin_limit;    // polls before a consumer gives up (and counts an error)
  // [0] += shader-clock cycles (s_memtime), [1] += 100 MHz real-time ticks
  // (s_memrealtime) each workgroup spends in the kernel: their ratio is the
  // effective shader clock of the launches (cloudsc_state_kseg_clock)
  unsigned long long* clk;
  int lev[kMaxSeg + 1];
};

// write-through (sc1) store of a handed-off value: an agent-scope relaxed atomic
// store lowers to global_store sc1, so the hand-off needs no L2 write-back
// (release fence) on the producer side (cdna_hip_programming.md G16, R1)
__device__ __forceinline__ void stg_sc1(double* ubase, size_t uidx, unsigned lane_bytes, double v) {
  __hip_atomic_store((unsigned long long*)((char*)(ubase + uidx) + lane_bytes), __double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stg_sc1(float* ubase, size_t uidx, unsigned lane_bytes, float v) {
  __hip_atomic_store((unsigned*)((char*)(ubase + uidx) + lane_bytes), __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

template <typename real, typename CS>
__device__ __forceinline__ void carry_io(real* st, size_t u, size_t plane, unsigned lo, CS& cs, bool save) {
#define CLOUDSC_CARRY_IO(q, m)                                                  \
  if (save) stg_sc1(st, u + (size_t)(q) * plane, lo, (real)cs.m);               \
  else cs.m = ldg((const real*)st, u + (size_t)(q) * plane, lo);
  CLOUDSC_CARRY_IO(0, t_prev) CLOUDSC_CARRY_IO(1, a_prev) CLOUDSC_CARRY_IO(2, pap_prev)
  CLOUDSC_CARRY_IO(3, zanewm1) CLOUDSC_CARRY_IO(4, zcovptot) CLOUDSC_CARRY_IO(5, zcovpmax)
  CLOUDSC_CARRY_IO(6, zcldtopdist) CLOUDSC_CARRY_IO(7, rainfrac) CLOUDSC_CARRY_IO(8, qxnm1_l)
  CLOUDSC_CARRY_IO(9, qxnm1_i) CLOUDSC_CARRY_IO(10, pfx_i) CLOUDSC_CARRY_IO(11, pfx_r)
  CLOUDSC_CARRY_IO(12, pfx_s) CLOUDSC_CARRY_IO(13, fl_lf) CLOUDSC_CARRY_IO(14, fl_if)
  CLOUDSC_CARRY_IO(15, fl_lng) CLOUDSC_CARRY_IO(16, fl_nng) CLOUDSC_CARRY_IO(17, fl_ltur)
  CLOUDSC_CARRY_IO(18, fl_itur)
#undef CLOUDSC_CARRY_IO
}

template <typename real, int PF, bool AER, bool LDSC, typename PT>
__device__ __forceinline__ void cloudsc_kcache_persistent_body(cptr<KArgs<real>> ka, cptr<PT> cpar,
                                                               const PersistArgs<real>& P) {
  __shared__ int s_item;
  const KArgs<real>& A = *(const KArgs<real>*)ka;
  const int nproma = A.nproma, nsub = P.nsub;
  // Every branch around a barrier is wave-uniform, and visibly so to the
  // compiler (SGPR conditions): the first wave of the workgroup does the
  // dequeue, the polling and the flag store with all of its lanes (same address,
  // same value), never a lane-0-only region.  A divergent `if (lane == 0)`
  // inside this loop gets restructured into nested exec-masked loops whose
  // barriers no longer pair up across waves.
  const bool wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x) < 64;
  const unsigned one = threadIdx.x == 0 ? 1u : 0u;  // lane 0 counts, the others add 0
  const unsigned long long clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
  // this workgroup's stripe: blocks b = lb * S + st, lb < nbs (all wave-uniform)
  const int S = P.nstripes;
  const int st = (int)(blockIdx.x % (unsigned)S);
  const int nbs = (P.nblocks - st + S - 1) / S;
  const int nsbs = nbs * nsub;                        // items per segment in the stripe
  const int items = P.nseg * nsbs;
  unsigned* const ctr = P.ctr + st * kKsegCtrStride;
  const unsigned base = P.base[st];
  for (;;) {
    if (wave0) {
      const unsigned old = __hip_atomic_fetch_add(ctr, one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_item = (int)(__builtin_amdgcn_readfirstlane(old) - base);   // lane 0's value: the ticket
    }
    __syncthreads();
    const int item = __builtin_amdgcn_readfirstlane(s_item);
    __syncthreads();                                   // s_item is rewritten next iteration
    if (item >= items) break;
    // item = (segment, stripe block lb, 64-column sub-block h), segment-major
    // (or (segment, h, lb) with sb_major): a block of NPROMA > 64 columns is run
    // as nsub one-wave items over the same block layout (sub-block h is the 64
    // contiguous columns h*64.. of each plane); flags are per (b, h)
    const int seg = item / nsbs, r = item - seg * nsbs;
    const int lb = P.sb_major ? r % nbs : r / nsub;
    const int hh = P.sb_major ? r / nbs : r - lb * nsub;
    const int b = lb * S + st;
    const int sb = b * nsub + hh;
    const int jl = hh * 64 + (int)threadIdx.x;
    const unsigned lo = (unsigned)jl * (unsigned)sizeof(real);
#ifdef CLOUDSC_KSEG_TRACE
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_ready = t_start;
#endif
    const bool active = jl < nproma && b * nproma + jl < A.ngptot;
    const size_t ust = (size_t)b * kCarryN * nproma;
    CarryOf<real, LDSC> cs(carry_lds_base<real>());
    if (seg == 0) {
      init_carry<real>(cs);
      if (active) {
        CLOUDSC_PARAMS_HERE;
        flux_top(c, A, (size_t)b * (A.klev + 1) * nproma, lo);
      }
    } else {
      // consumer: one relaxed poll (bounded, with s_sleep), one agent acquire,
      // wait, barrier, plain loads
      if (wave0) {
        for (unsigned spins = 0;; spins++) {
          if (spins >= P.spin_limit) {                   // bounded: never hang; the host reports it
            __hip_atomic_fetch_add(P.err, one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          const unsigned f = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(P.flags + sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          if ((int)(f - (P.stamp + (unsigned)seg)) >= 0) break;
          __builtin_amdgcn_s_sleep(4);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#ifdef CLOUDSC_KSEG_TRACE
      t_ready = __builtin_amdgcn_s_memrealtime();
#endif
      if (active) carry_io(P.state, ust, (size_t)nproma, lo, cs, false);
    }
    if (active) kcache_levels<real, PF, AER>(ka, cpar, b, lo, P.lev[seg], P.lev[seg + 1], cs);
    if (seg + 1 < P.nseg) {
      // producer (G16 R1): sc1 payload stores, every wave drains, barrier, the
      // flag stored with an agent atomic
      if (active) carry_io(P.state, ust, (size_t)nproma, lo, cs, true);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (wave0) __hip_atomic_store(P.flags + sb, P.stamp + (unsigned)(seg + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (active) {
      stg(((const KArgs<real>*)launder_uniform(ka))->prainfrac, (size_t)b * nproma, lo, cs.rainfrac);
    }
#ifdef CLOUDSC_KSEG_TRACE
    const int gitem = seg * P.nblocks * nsub + sb;   // the item's index in the unstriped order
    if (threadIdx.x == 0 && gitem < kTraceMax) {   // diagnostic build only: schedule of every item
      g_kseg_trace[4 * gitem + 0] = t_start;
      g_kseg_trace[4 * gitem + 1] = __builtin_amdgcn_s_memrealtime();
      g_kseg_trace[4 * gitem + 2] = blockIdx.x;
      g_kseg_trace[4 * gitem + 3] = t_ready;
    }
#endif
  }
  // the workgroup's time in the kernel, in shader cycles and real-time ticks
  // (one vector atomic each, after the last item; no barrier follows)
  const unsigned long long dclk = __builtin_amdgcn_s_memtime() - clk0, drt = __builtin_amdgcn_s_memrealtime() - rt0;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(P.clk, dclk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(P.clk + 1, drt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace cloudsc
