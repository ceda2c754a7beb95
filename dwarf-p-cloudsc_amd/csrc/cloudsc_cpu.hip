// cloudsc_cpu.hip -- cloudsc_cpu_run: the CPU variant of the dwarf (BASELINE.json
// config 1, `dwarf-cloudsc-c 1 16384 32`), explicitly selected by the caller.
// It is never substituted for a GPU run: the GPU entry points have no fallback.
//
// Reference: the C dwarf's OpenMP block loop (src/cloudsc_c/cloudsc/cloudsc_driver.c:
// 183-217, schedule(runtime)) calling the kernel cloudsc_c() (cloudsc_c.c:19-2587)
// on one NPROMA block at a time.  Here the per-level phase functions are the
// ones the GPU kernels are built from (cloudsc_kcache.h: init_level,
// physics_level, flux_level, ... compiled for the host), run level-outer and
// column-inner over a block -- the same order of operations per column, so the
// output is the reference kernel's bit for bit (tests/test_cpu.py pins it
// against oracle/_ref, the reference kernel compiled from its sources).
// Host threads take blocks from a shared counter (dynamic schedule).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "cloudsc_amd.h"
#include "cloudsc_internal.h"
#include "cloudsc_kcache.h"
#include "cloudsc_params.h"

using namespace cloudsc;

namespace {

// The state of one column that crosses levels, as in kcache_levels
// (cloudsc_kcache.h), without the GPU's software pipelining of the loads.
template <typename real>
struct HostColumn {
  CarryState<real> cs;
  Neighbors<real> nb;
  ColConst<real> cc;
};

template <typename real, bool AER>
void run_block(const DevParams<real>& c, const KArgs<real>& A, int b, std::vector<HostColumn<real>>& col) {
  const int nproma = A.nproma, klev = A.klev;
  const int bsize = std::min(nproma, A.ngptot - b * nproma);
  const size_t u1 = (size_t)b * nproma;
  const size_t u2 = (size_t)b * klev * nproma;
  const size_t uh = (size_t)b * (klev + 1) * nproma;
  const size_t u3 = (size_t)b * 5 * klev * nproma;
  const int ncldtop0 = c.ncldtop - 1;
  const int l1 = 1 < klev ? 1 : klev - 1;
  for (int jl = 0; jl < bsize; jl++) {
    const unsigned lo = (unsigned)jl * (unsigned)sizeof(real);
    HostColumn<real>& h = col[jl];
    init_carry<real>(h.cs);
    flux_top(c, A, uh, lo);
    h.cc = column_constants(c, A, u1, uh, lo);
    h.nb.paph_k = ldg(A.paph, uh, lo);
    h.nb.paph_n = ldg(A.paph, uh + (size_t)nproma, lo);
    h.nb.pmfu_k = ldg(A.pmfu, u2, lo);
    h.nb.pmfd_k = ldg(A.pmfd, u2, lo);
    h.nb.pmfu_n = ldg(A.pmfu, u2 + (size_t)l1 * nproma, lo);
    h.nb.pmfd_n = ldg(A.pmfd, u2 + (size_t)l1 * nproma, lo);
    h.nb.plu_n = ldg(A.plu, u2 + (size_t)l1 * nproma, lo);
  }
  for (int k = 0; k < klev; k++) {
    const bool physics = k >= ncldtop0;
    const int k2 = k + 2 < klev ? k + 2 : klev - 1;
    const int kh2 = k + 2 < klev + 1 ? k + 2 : klev;
    for (int jl = 0; jl < bsize; jl++) {
      const unsigned lo = (unsigned)jl * (unsigned)sizeof(real);
      HostColumn<real>& h = col[jl];
      LevelIn<real> cur;
      load_level<real, AER>(cur, A, u2, u3, k, klev, nproma, lo);
      LevelState<real> ls;
      PhysOut<real> po;
      init_level(c, cur, ls);
      for (int m = 0; m < 4; m++) { po.zqxn[m] = R(0.0); po.ctend[m] = R(0.0); }
      po.plude_k = cur.plude;
      po.atend = R(0.0);
      po.zcovptot_out = R(0.0);
      if (physics) physics_level(c, k, klev, ncldtop0, cur, h.nb, h.cc, ls, h.cs, po);
      store_level(A, u2, u3, k, klev, nproma, lo, physics, ls, po);
      flux_level(c, A, uh + (size_t)(k + 1) * nproma, lo, cur, ls, po, h.nb.paph_k, h.nb.paph_n, h.cs);
      h.cs.t_prev = ls.ztp1;
      h.cs.a_prev = ls.za;
      h.cs.pap_prev = cur.pap;
      h.nb.paph_k = h.nb.paph_n;
      h.nb.paph_n = ldg(A.paph, uh + (size_t)kh2 * nproma, lo);
      h.nb.pmfu_k = h.nb.pmfu_n;
      h.nb.pmfd_k = h.nb.pmfd_n;
      h.nb.pmfu_n = ldg(A.pmfu, u2 + (size_t)k2 * nproma, lo);
      h.nb.pmfd_n = ldg(A.pmfd, u2 + (size_t)k2 * nproma, lo);
      h.nb.plu_n = ldg(A.plu, u2 + (size_t)k2 * nproma, lo);
    }
  }
  for (int jl = 0; jl < bsize; jl++) stg(A.prainfrac, u1, (unsigned)jl * (unsigned)sizeof(real), col[jl].cs.rainfrac);
}

KArgs<double> host_args(const cloudsc_fields_t* f, int ngptot, int nproma, int klev) {
  KArgs<double> a;
  std::memset(&a, 0, sizeof(a));
  a.pt = (const double*)f->pt; a.pq = (const double*)f->pq;
  a.ttt = (const double*)f->tendency_tmp_t; a.ttq = (const double*)f->tendency_tmp_q;
  a.tta = (const double*)f->tendency_tmp_a; a.ttcld = (const double*)f->tendency_tmp_cld;
  a.pvfl = (const double*)f->pvfl; a.pvfi = (const double*)f->pvfi;
  a.phrsw = (const double*)f->phrsw; a.phrlw = (const double*)f->phrlw; a.pvervel = (const double*)f->pvervel;
  a.pap = (const double*)f->pap; a.paph = (const double*)f->paph; a.plsm = (const double*)f->plsm;
  a.ktype = f->ktype;
  a.plu = (const double*)f->plu; a.psnde = (const double*)f->psnde; a.pmfu = (const double*)f->pmfu;
  a.pmfd = (const double*)f->pmfd; a.pa = (const double*)f->pa; a.pclv = (const double*)f->pclv;
  a.psupsat = (const double*)f->psupsat; a.picrit_aer = (const double*)f->picrit_aer;
  a.pre_ice = (const double*)f->pre_ice; a.pnice = (const double*)f->pnice;
  a.plude = (double*)f->plude; a.plude_in = (const double*)f->plude;
  a.tlt = (double*)f->tendency_loc_t; a.tlq = (double*)f->tendency_loc_q;
  a.tla = (double*)f->tendency_loc_a; a.tlcld = (double*)f->tendency_loc_cld;
  a.pcovptot = (double*)f->pcovptot; a.prainfrac = (double*)f->prainfrac_toprfz;
  a.pfsqlf = (double*)f->pfsqlf; a.pfsqif = (double*)f->pfsqif; a.pfcqnng = (double*)f->pfcqnng;
  a.pfcqlng = (double*)f->pfcqlng; a.pfsqrf = (double*)f->pfsqrf; a.pfsqsf = (double*)f->pfsqsf;
  a.pfcqrng = (double*)f->pfcqrng; a.pfcqsng = (double*)f->pfcqsng; a.pfsqltur = (double*)f->pfsqltur;
  a.pfsqitur = (double*)f->pfsqitur; a.pfplsl = (double*)f->pfplsl; a.pfplsn = (double*)f->pfplsn;
  a.pfhpsl = (double*)f->pfhpsl; a.pfhpsn = (double*)f->pfhpsn;
  a.ngptot = ngptot; a.nproma = nproma; a.klev = klev;
  return a;
}

}  // namespace

extern "C" int cloudsc_cpu_run_threads(int nthreads, int ngptot, int nproma, int klev,
                                       const cloudsc_params_t* params, const cloudsc_fields_t* f, double* seconds,
                                       double* thread_seconds, int* thread_blocks, int* thread_columns) {
  int rc = cloudsc_impl::check_params(params);
  if (rc) return rc;
  if (!f || !cloudsc_impl::fields_complete(f) || ngptot <= 0 || nproma <= 0 || klev < 2) return CLOUDSC_EINVAL;
  const bool aer = params->laericesed || params->laericeauto;
  if (aer && (!f->pre_ice || !f->picrit_aer || !f->pnice)) return CLOUDSC_EINVAL;
  if (nthreads <= 0 && (thread_seconds || thread_blocks || thread_columns)) return CLOUDSC_EINVAL;
  const DevParams<double> c = fold_params<double>(*params);
  const KArgs<double> A = host_args(f, ngptot, nproma, klev);
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  const int nreq = nthreads;                 // the caller's per-thread arrays have nreq entries
  nthreads = std::min(nthreads, nblocks);
  for (int t = 0; t < nreq; t++) {           // threads beyond the block count do nothing
    if (thread_seconds) thread_seconds[t] = 0.0;
    if (thread_blocks) thread_blocks[t] = 0;
    if (thread_columns) thread_columns[t] = 0;
  }
  std::atomic<int> next{0};
  // per thread, as the C dwarf's zinfo (cloudsc_driver.c:185-228): its own
  // wall time, NPROMA blocks taken (icalls) and columns computed (igpc)
  auto worker = [&](int tid) {
    const auto s0 = std::chrono::steady_clock::now();
    std::vector<HostColumn<double>> col((size_t)nproma);
    int icalls = 0, igpc = 0;
    for (int b = next.fetch_add(1); b < nblocks; b = next.fetch_add(1)) {
      if (aer) run_block<double, true>(c, A, b, col);
      else run_block<double, false>(c, A, b, col);
      icalls++;
      igpc += std::min(nproma, ngptot - b * nproma);
    }
    const auto s1 = std::chrono::steady_clock::now();
    if (thread_seconds) thread_seconds[tid] = std::chrono::duration<double>(s1 - s0).count();
    if (thread_blocks) thread_blocks[tid] = icalls;
    if (thread_columns) thread_columns[tid] = igpc;
  };
  const auto t0 = std::chrono::steady_clock::now();
  if (nthreads == 1) {
    worker(0);
  } else {
    std::vector<std::thread> pool;
    pool.reserve((size_t)nthreads);
    try {
      for (int t = 0; t < nthreads; t++) pool.emplace_back(worker, t);
    } catch (...) {
      rc = CLOUDSC_ENOMEM;          // the threads already started finish the blocks
    }
    for (auto& t : pool) t.join();
  }
  const auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  return rc;
}

extern "C" int cloudsc_cpu_run(int nthreads, int ngptot, int nproma, int klev, const cloudsc_params_t* params,
                               const cloudsc_fields_t* f, double* seconds) {
  return cloudsc_cpu_run_threads(nthreads, ngptot, nproma, klev, params, f, seconds, nullptr, nullptr, nullptr);
}
