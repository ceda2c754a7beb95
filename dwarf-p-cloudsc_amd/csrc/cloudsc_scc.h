// cloudsc_scc.h -- the SCC baseline CLOUDSC kernel (BASELINE config 2):
// NPROMA block -> workgroup, column -> lane, but organised like the reference
// C kernel (src/cloudsc_c/cloudsc/cloudsc_c.c) as separate sweeps over the
// levels with LEVEL-SIZED temporaries ("heap temporaries"):
//   sweep 1  (:462-640)   initial values, tidy-up, FOEALFA for every level
//                         -> ztp1, za, zaorig, zqx, zqx0, zlneg, ... in scratch
//   sweep 2  (:732-2508)  physics loop, reads sweep-1 temporaries back,
//                         writes tendencies and zqxn2d / zpfplsx to scratch
//   sweep 3  (:2521-2582) flux diagnostics from the scratch temporaries
// The temporaries live in HBM in the coalesced [nblocks][lev][nproma] layout of
// the reference's hoisted variant (src/cloudsc_cuda/cloudsc/cloudsc_c_hoist.cu:454-471).
// The per-level arithmetic is the very same code as the k-caching kernel
// (init_level / physics_level / flux_level), so both variants give bit-identical
// results; only the data movement differs.  It exists as the measured baseline
// the k-caching layout is compared against.
#pragma once
#include "cloudsc_kcache.h"

namespace cloudsc {

constexpr int kSccLsPlanes = 6 + 5 + 4 + 4;   // scalars, zqx, zqx0[0..3], zlneg

template <typename real>
struct SccScratch {
  real* ls;      // [nblocks][kSccLsPlanes][klev][nproma]: LevelState without zqx0[qv]
  real* qxn;     // [nblocks][4][klev][nproma]: zqxn2d
  real* pfx;     // [nblocks][3][klev+1][nproma]: zpfplsx[qi,qr,qs]
};

template <typename real>
inline long long scc_scratch_bytes(long long nblocks, long long nproma, long long klev) {
  return (long long)sizeof(real) * nblocks * nproma * (kSccLsPlanes * klev + 4 * klev + 3 * (klev + 1));
}

template <typename real>
inline SccScratch<real> scc_scratch_carve(char* base, long long nblocks, long long nproma, long long klev) {
  SccScratch<real> s;
  s.ls = (real*)base;
  s.qxn = s.ls + nblocks * nproma * kSccLsPlanes * klev;
  s.pfx = s.qxn + nblocks * nproma * 4 * klev;
  return s;
}

template <typename real>
__device__ __forceinline__ void scc_put_ls(real* base, size_t idx, size_t plane, unsigned lo, const LevelState<real>& s) {
  stg_cached(base, idx + 0 * plane, lo, s.ztp1); stg_cached(base, idx + 1 * plane, lo, s.za);
  stg_cached(base, idx + 2 * plane, lo, s.zaorig); stg_cached(base, idx + 3 * plane, lo, s.zfoealfa);
  stg_cached(base, idx + 4 * plane, lo, s.ttend); stg_cached(base, idx + 5 * plane, lo, s.qtend);
#pragma unroll
  for (int m = 0; m < 5; m++) stg_cached(base, idx + (6 + m) * plane, lo, s.zqx[m]);
#pragma unroll
  for (int m = 0; m < 4; m++) stg_cached(base, idx + (11 + m) * plane, lo, s.zqx0[m]);
#pragma unroll
  for (int m = 0; m < 4; m++) stg_cached(base, idx + (15 + m) * plane, lo, s.zlneg[m]);
}
template <typename real>
__device__ __forceinline__ void scc_get_ls(const real* base, size_t idx, size_t plane, unsigned lo, LevelState<real>& s) {
  s.ztp1 = ldg(base, idx + 0 * plane, lo); s.za = ldg(base, idx + 1 * plane, lo);
  s.zaorig = ldg(base, idx + 2 * plane, lo); s.zfoealfa = ldg(base, idx + 3 * plane, lo);
  s.ttend = ldg(base, idx + 4 * plane, lo); s.qtend = ldg(base, idx + 5 * plane, lo);
#pragma unroll
  for (int m = 0; m < 5; m++) s.zqx[m] = ldg(base, idx + (6 + m) * plane, lo);
#pragma unroll
  for (int m = 0; m < 4; m++) s.zqx0[m] = ldg(base, idx + (11 + m) * plane, lo);
  s.zqx0[QV] = R(0.0);   // not used after sweep 1
#pragma unroll
  for (int m = 0; m < 4; m++) s.zlneg[m] = ldg(base, idx + (15 + m) * plane, lo);
}

// Where the SCC sweeps keep their level temporaries.  HbmTemps: planes of the
// caller's workspace in the coalesced [nblocks][plane][klev][nproma] layout (the
// hoisted variant, config 2).  PrivTemps: per-thread private arrays, the
// reference's own SCC form (cloudsc_c.cu:60-317, klev = 137 at compile time
// there, :53) -- on CDNA4 they live in the private segment (scratch), which
// the hardware interleaves per lane, so a wave's same-index accesses coalesce.
template <typename real>
struct HbmTemps {
  SccScratch<real> S;
  size_t plane, pstride, ulsb, uqxb, upfb;
  int nproma_;
  unsigned lo;
  __device__ __forceinline__ HbmTemps(const SccScratch<real>& s, int b, int nproma, int klev, unsigned lane)
      : S(s), plane((size_t)klev * nproma), pstride((size_t)(klev + 1) * nproma),
        ulsb((size_t)b * kSccLsPlanes * plane),   // S.ls  [planes][klev][nproma]
        uqxb((size_t)b * 4 * plane),              // S.qxn [4][klev][nproma]
        upfb((size_t)b * 3 * pstride),            // S.pfx [3][klev+1][nproma]
        nproma_(nproma), lo(lane) {}
  __device__ __forceinline__ void put_ls(int k, const LevelState<real>& ls) {
    scc_put_ls(S.ls, ulsb + (size_t)k * nproma_, plane, lo, ls);
  }
  __device__ __forceinline__ void get_ls(int k, LevelState<real>& ls) const {
    scc_get_ls((const real*)S.ls, ulsb + (size_t)k * nproma_, plane, lo, ls);
  }
  // ztp1(k) and za(k): planes 0 and 1 of the level state
  __device__ __forceinline__ real ls_plane(int q, int k) const {
    return ldg((const real*)S.ls, ulsb + (size_t)k * nproma_ + (size_t)q * plane, lo);
  }
  __device__ __forceinline__ void put_qxn(int m, int k, real v) {
    stg_cached(S.qxn, uqxb + (size_t)m * plane + (size_t)k * nproma_, lo, v);
  }
  __device__ __forceinline__ real get_qxn(int m, int k) const {
    return ldg((const real*)S.qxn, uqxb + (size_t)m * plane + (size_t)k * nproma_, lo);
  }
  // zpfplsx at half level kh
  __device__ __forceinline__ void put_pfx(int m, int kh, real v) {
    stg_cached(S.pfx, upfb + (size_t)m * pstride + (size_t)kh * nproma_, lo, v);
  }
  __device__ __forceinline__ real get_pfx(int m, int kh) const {
    return ldg((const real*)S.pfx, upfb + (size_t)m * pstride + (size_t)kh * nproma_, lo);
  }
};

constexpr int kPrivKlev = 137;   // the reference SCC kernel's compile-time klev (cloudsc_c.cu:53)
template <typename real>
struct PrivTemps {
  real ls[kSccLsPlanes][kPrivKlev];
  real qxn[4][kPrivKlev];
  real pfx[3][kPrivKlev + 1];
  __device__ __forceinline__ void put_ls(int k, const LevelState<real>& s) {
    ls[0][k] = s.ztp1; ls[1][k] = s.za; ls[2][k] = s.zaorig; ls[3][k] = s.zfoealfa;
    ls[4][k] = s.ttend; ls[5][k] = s.qtend;
#pragma unroll
    for (int m = 0; m < 5; m++) ls[6 + m][k] = s.zqx[m];
#pragma unroll
    for (int m = 0; m < 4; m++) ls[11 + m][k] = s.zqx0[m];
#pragma unroll
    for (int m = 0; m < 4; m++) ls[15 + m][k] = s.zlneg[m];
  }
  __device__ __forceinline__ void get_ls(int k, LevelState<real>& s) const {
    s.ztp1 = ls[0][k]; s.za = ls[1][k]; s.zaorig = ls[2][k]; s.zfoealfa = ls[3][k];
    s.ttend = ls[4][k]; s.qtend = ls[5][k];
#pragma unroll
    for (int m = 0; m < 5; m++) s.zqx[m] = ls[6 + m][k];
#pragma unroll
    for (int m = 0; m < 4; m++) s.zqx0[m] = ls[11 + m][k];
    s.zqx0[QV] = R(0.0);   // not used after sweep 1
#pragma unroll
    for (int m = 0; m < 4; m++) s.zlneg[m] = ls[15 + m][k];
  }
  __device__ __forceinline__ real ls_plane(int q, int k) const { return ls[q][k]; }
  __device__ __forceinline__ void put_qxn(int m, int k, real v) { qxn[m][k] = v; }
  __device__ __forceinline__ real get_qxn(int m, int k) const { return qxn[m][k]; }
  __device__ __forceinline__ void put_pfx(int m, int kh, real v) { pfx[m][kh] = v; }
  __device__ __forceinline__ real get_pfx(int m, int kh) const { return pfx[m][kh]; }
};

template <typename real, bool AER, typename Temps, typename PT>
__device__ __forceinline__ void cloudsc_scc_sweeps(cptr<KArgs<real>> ka, Temps& T, cptr<PT> cpar) {
  const KArgs<real>& A0 = *(const KArgs<real>*)ka;
  const int nproma = A0.nproma, klev = A0.klev;
  const int b = blockIdx.x, jl = threadIdx.x;
  const unsigned lo = (unsigned)jl * (unsigned)sizeof(real);
  const size_t u1 = (size_t)b * nproma;
  const size_t u2 = (size_t)b * klev * nproma;
  const size_t uh = (size_t)b * (klev + 1) * nproma;
  const size_t u3 = (size_t)b * 5 * klev * nproma;
  const int ncldtop0 = ((const DevParams<real>*)cpar)->ncldtop - 1;
#define SCC_A (*(const KArgs<real>*)launder_uniform(ka))
#define SCC_C (*(const PT*)launder_uniform(cpar))

  // ---- sweep 1: section 1 for every level ----
  for (int k = 0; k < klev; k++) {
    LevelIn<real> in;
    load_level<real, AER>(in, SCC_A, u2, u3, k, klev, nproma, lo);
    LevelState<real> ls;
    init_level(SCC_C, in, ls);
    T.put_ls(k, ls);
  }

  // ---- sweep 2: physics (all levels written; physics from NCLDTOP down) ----
  const ColConst<real> cc = column_constants(SCC_C, SCC_A, u1, uh, lo);
  CarryState<real> cs;
  init_carry<real>(cs);
#pragma unroll
  for (int m = 0; m < 3; m++) T.put_pfx(m, 0, R(0.0));   // zpfplsx(:,1) = 0
  for (int k = 0; k < klev; k++) {
    const bool physics = k >= ncldtop0;
    const KArgs<real>& A = SCC_A;
    LevelIn<real> in;
    load_level<real, AER>(in, A, u2, u3, k, klev, nproma, lo);
    LevelState<real> ls;
    T.get_ls(k, ls);
    Neighbors<real> nb;
    nb.paph_k = ldg(A.paph, uh + (size_t)k * nproma, lo);
    nb.paph_n = ldg(A.paph, uh + (size_t)(k + 1) * nproma, lo);
    nb.pmfu_k = ldg(A.pmfu, u2 + (size_t)k * nproma, lo);
    nb.pmfd_k = ldg(A.pmfd, u2 + (size_t)k * nproma, lo);
    const bool has_next = k + 1 < klev;
    nb.pmfu_n = has_next ? ldg(A.pmfu, u2 + (size_t)(k + 1) * nproma, lo) : R(0.0);
    nb.pmfd_n = has_next ? ldg(A.pmfd, u2 + (size_t)(k + 1) * nproma, lo) : R(0.0);
    nb.plu_n = has_next ? ldg(A.plu, u2 + (size_t)(k + 1) * nproma, lo) : R(0.0);
    if (k > 0) {   // level-above temporaries read back (ztp1(jk-1), za(jk-1), pap(jk-1))
      cs.t_prev = T.ls_plane(0, k - 1);
      cs.a_prev = T.ls_plane(1, k - 1);
      cs.pap_prev = ldg(A.pap, u2 + (size_t)(k - 1) * nproma, lo);
    }
    PhysOut<real> po;
#pragma unroll
    for (int m = 0; m < 4; m++) { po.zqxn[m] = R(0.0); po.ctend[m] = R(0.0); }
    po.plude_k = in.plude;
    po.atend = R(0.0);
    po.zcovptot_out = R(0.0);
    if (physics) physics_level(SCC_C, k, klev, ncldtop0, in, nb, cc, ls, cs, po);
    store_level(SCC_A, u2, u3, k, klev, nproma, lo, physics, ls, po);
#pragma unroll
    for (int m = 0; m < 4; m++) T.put_qxn(m, k, po.zqxn[m]);
    T.put_pfx(0, k + 1, cs.pfx_i);
    T.put_pfx(1, k + 1, cs.pfx_r);
    T.put_pfx(2, k + 1, cs.pfx_s);
  }
  stg(SCC_A.prainfrac, u1, lo, cs.rainfrac);

  // ---- sweep 3: flux diagnostics from the stored temporaries ----
  flux_top(SCC_C, SCC_A, uh, lo);
  for (int k = 0; k < klev; k++) {
    const KArgs<real>& A = SCC_A;
    LevelIn<real> in;
    in.pvfl = ldg(A.pvfl, u2 + (size_t)k * nproma, lo);
    in.pvfi = ldg(A.pvfi, u2 + (size_t)k * nproma, lo);
    LevelState<real> ls;
    T.get_ls(k, ls);
    PhysOut<real> po;
#pragma unroll
    for (int m = 0; m < 4; m++) po.zqxn[m] = T.get_qxn(m, k);
    po.plude_k = ldg((const real*)A.plude, u2 + (size_t)k * nproma, lo);   // final (rescaled) value
    cs.pfx_i = T.get_pfx(0, k + 1);
    cs.pfx_r = T.get_pfx(1, k + 1);
    cs.pfx_s = T.get_pfx(2, k + 1);
    flux_level(SCC_C, A, uh + (size_t)(k + 1) * nproma, lo, in, ls, po,
               ldg(A.paph, uh + (size_t)k * nproma, lo), ldg(A.paph, uh + (size_t)(k + 1) * nproma, lo), cs);
  }
#undef SCC_A
#undef SCC_C
}

// config 2 / a4: the temporaries in the caller's HBM workspace
template <typename real, bool AER, typename PT>
__device__ __forceinline__ void cloudsc_scc_body(cptr<KArgs<real>> ka, const SccScratch<real> S, cptr<PT> cpar) {
  const KArgs<real>& A0 = *(const KArgs<real>*)ka;
  const int b = blockIdx.x, jl = threadIdx.x;
  if (jl >= A0.nproma || b * A0.nproma + jl >= A0.ngptot) return;
  HbmTemps<real> T(S, b, A0.nproma, A0.klev, (unsigned)jl * (unsigned)sizeof(real));
  cloudsc_scc_sweeps<real, AER>(ka, T, cpar);
}

// a3: the temporaries in per-thread private arrays (klev <= kPrivKlev, checked at launch)
template <typename real, bool AER, typename PT>
__device__ __forceinline__ void cloudsc_scc_private_body(cptr<KArgs<real>> ka, cptr<PT> cpar) {
  const KArgs<real>& A0 = *(const KArgs<real>*)ka;
  const int b = blockIdx.x, jl = threadIdx.x;
  if (jl >= A0.nproma || b * A0.nproma + jl >= A0.ngptot) return;
  PrivTemps<real> T;
  cloudsc_scc_sweeps<real, AER>(ka, T, cpar);
}

}  // namespace cloudsc
