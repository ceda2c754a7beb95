HOST_BUILD = r'''
// ---- experiment: McNaughton wrap schedule for KSEG (CLOUDSC_KSEG_WRAP) ----
// Per stripe: U units (64-column sub-blocks) on W workgroups, W < U <= 2W.
// Workgroup slot w covers the work interval [w U, (w+1) U) in units of 1/W of
// a column; a column straddling a slot boundary is split once: its FIRST part
// runs at the start of the later slot, its LAST part at the end of the earlier
// one.  Items: round 1 = every slot's first piece (slot order), later rounds =
// the remaining pieces, longest first.  A last part's first part is a round-1
// item, dequeued earlier: progress as with segments.
static int wrap_level(double f, int klev, int top, double beta) {
  const int phys = klev - top;
  double x = f;
  if (beta != 0.0) x = (-1.0 + std::sqrt(1.0 + 2.0 * beta * f * (1.0 + beta / 2.0))) / beta;
  int L = top + (int)std::lround(x * phys);
  if (L < 1) L = 1;
  if (L > klev - 1) L = klev - 1;
  return L;
}
static bool build_wrap(std::vector<unsigned>& tab, int* witems, int wstride, int grid, int S, int nblocks, int nsub,
                       int klev, int ncldtop, int split_pct) {
  const int top = ncldtop - 1 < 0 ? 0 : (ncldtop - 1 > klev ? klev : ncldtop - 1);
  const double p = split_pct / 100.0;
  const double den = p * p / 2.0 - 0.25;
  const double beta = (std::fabs(0.5 - p) < 1e-9 || std::fabs(den) < 1e-9) ? 0.0 : (0.5 - p) / den;
  tab.assign((size_t)S * wstride * 2, 0u);
  for (int st = 0; st < S; st++) {
    const long long nbs = (nblocks - st + S - 1) / S;
    const long long U = nbs * nsub, W = (grid - st + S - 1) / S;
    if (!(U > W && U <= 2 * W)) return false;
    struct Piece { unsigned unit; int seg; bool produce; int l0, l1; long long len; };
    std::vector<int> Lunit((size_t)U, -1);
    // first parts: the slot whose interval starts inside unit j runs levels [0, L) of j first
    // (rebuild round 1 from the slot starts)
    std::vector<Piece> later[3];
    for (long long w = 0; w < W; w++) {
      const long long a = w * U, e = (w + 1) * U;
      std::vector<Piece> pcs;
      long long q = a;
      if (a % W != 0) {
        const long long j = a / W;
        const long long f = (j + 1) * W - a;               // first-part length
        if (Lunit[j] < 0) Lunit[j] = wrap_level((double)f / W, klev, top, beta);
        pcs.push_back({(unsigned)j, 0, true, 0, Lunit[j], f});
        q = (j + 1) * W;
      }
      while (q < e) {
        const long long j = q / W;
        if ((j + 1) * W <= e) { pcs.push_back({(unsigned)j, 0, false, 0, klev, W}); q += W; }
        else {
          const long long g = e - q;
          if (Lunit[j] < 0) Lunit[j] = wrap_level((double)(W - g) / W, klev, top, beta);
          pcs.push_back({(unsigned)j, 1, false, Lunit[j], klev, g});
          q = e;
        }
      }
      if (pcs.size() > 3) return false;
      for (size_t k = 0; k < pcs.size(); k++) later[k].push_back(pcs[k]);
    }
    size_t n = 0;
    for (int k = 0; k < 3; k++) {
      if (k > 0)
        std::stable_sort(later[k].begin(), later[k].end(),
                         [](const Piece& x, const Piece& y) { return x.len > y.len; });
      for (const Piece& pc : later[k]) {
        if ((long long)n >= wstride) return false;
        unsigned* ent = &tab[((size_t)st * wstride + n) * 2];
        ent[0] = pc.unit | ((unsigned)pc.seg << 31) | ((pc.produce ? 1u : 0u) << 30);
        ent[1] = (unsigned)pc.l0 | ((unsigned)pc.l1 << 16);
        n++;
      }
    }
    witems[st] = (int)n;
  }
  return true;
}
'''
EDITS = [
 ("cloudsc_gpu.hip", "#include <cstring>", "#include <cstring>\n#include <cmath>\n#include <algorithm>"),
 # workspace grows by the table
 ("cloudsc_gpu.hip",
  """template <typename real>
size_t kseg_scratch_bytes(int nblocks, int nproma) {
  return kseg_ctl_bytes(nblocks, nproma) + (size_t)nblocks * kCarryN * nproma * sizeof(real);
}""",
  """int kseg_wrap_stride(int nblocks, int nsub) { return 2 * ((nblocks + kKsegStripes - 1) / kKsegStripes) * nsub + 4; }
template <typename real>
size_t kseg_scratch_bytes(int nblocks, int nproma) {
  return kseg_ctl_bytes(nblocks, nproma) + align256((size_t)nblocks * kCarryN * nproma * sizeof(real)) +
         (size_t)kKsegStripes * kseg_wrap_stride(nblocks, kseg_nsub(nproma)) * 8;
}"""),
 ("cloudsc_gpu.hip",
  """namespace {

template <typename real, int WAVES, int PF, bool AER, bool LDSC, bool FAST>
int launch_kseg_cfg(""",
  HOST_BUILD + """namespace {

template <typename real, int WAVES, int PF, bool AER, bool LDSC, bool FAST>
int launch_kseg_cfg("""),
 ("cloudsc_gpu.hip",
  """  PersistArgs<real> pg = pa;
  pg.nstripes = kseg_nstripes(grid);
  launch_physics(kern, dim3(grid), dim3(wg), lds, st, ev, a, pg);""",
  """  PersistArgs<real> pg = pa;
  pg.nstripes = kseg_nstripes(grid);
  pg.wtab = nullptr;
  {
    static thread_local std::vector<unsigned> tab;
    static thread_local unsigned* pinned = nullptr;
    static thread_local size_t pcap = 0;
    const int wstride = kseg_wrap_stride(pa.nblocks, pa.nsub);
    int witems[kKsegStripes] = {};
    if (build_wrap(tab, witems, wstride, grid, pg.nstripes, pa.nblocks, pa.nsub, a.klev, pa.ncldtop,
                   kKsegSplitPct<real>)) {
      const size_t bytes = tab.size() * sizeof(unsigned);
      if (bytes > pcap) {
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr; pcap = 0;
        if (hipHostMalloc((void**)&pinned, bytes, hipHostMallocDefault) != hipSuccess) return CLOUDSC_ENOMEM;
        pcap = bytes;
      }
      unsigned* dtab = (unsigned*)((char*)pa.state + ((size_t)pa.nblocks * kCarryN * nproma * sizeof(real) + 255) / 256 * 256);
      static thread_local const void* last_dtab = nullptr;
      static thread_local std::vector<unsigned> last_tab;
      if (dtab != last_dtab || tab != last_tab) {       // upload once per workspace and schedule
        std::memcpy(pinned, tab.data(), bytes);
        HIPCHK(hipMemcpyAsync(dtab, pinned, bytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        last_dtab = dtab;
        last_tab = tab;
      }
      pg.wtab = dtab;
      pg.wstride = wstride;
      for (int q = 0; q < kKsegStripes; q++) pg.witems[q] = witems[q];
    }
  }
  if (items_out) for (int q = 0; q < kKsegStripes; q++) items_out[q] = pg.wtab ? pg.witems[q] : -1;
  launch_physics(kern, dim3(grid), dim3(wg), lds, st, ev, a, pg);"""),
 ("cloudsc_gpu.hip",
  """int launch_kseg_cfg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems,
                    int* grid_out, const LaunchEvents* ev) {""",
  """int launch_kseg_cfg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems,
                    int* grid_out, const LaunchEvents* ev, int* items_out) {"""),
 ("cloudsc_gpu.hip",
  """int launch_kseg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems,
                int* grid_out, const LaunchEvents* ev) {""",
  """int launch_kseg(hipStream_t st, const KArgs<real>& a, const PersistArgs<real>& pa, int nproma, int nitems,
                int* grid_out, const LaunchEvents* ev, int* items_out) {"""),
 ("cloudsc_gpu.hip",
  """  return launch_kseg_cfg<real, DefaultCfg<real>::waves, DefaultCfg<real>::pf, AER, false, FAST>(st, a, pa, nproma, nitems,
                                                                                        grid_out, ev);""",
  """  return launch_kseg_cfg<real, DefaultCfg<real>::waves, DefaultCfg<real>::pf, AER, false, FAST>(st, a, pa, nproma, nitems,
                                                                                        grid_out, ev, items_out);"""),
 ("cloudsc_gpu.hip",
  """    int grid = 0;
    if constexpr (CLOUDSC_KEEP_KERNEL(real, true, true))
      rc = aer ? launch_kseg<real, true, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev)
               : launch_kseg<real, false, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev);
    else if constexpr (CLOUDSC_KEEP_KERNEL(real, true, false))
      rc = launch_kseg<real, false, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev);""",
  """    int grid = 0;
    int witems[kKsegStripes];
    pa.ncldtop = ps.ncldtop;
    if constexpr (CLOUDSC_KEEP_KERNEL(real, true, true))
      rc = aer ? launch_kseg<real, true, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev, witems)
               : launch_kseg<real, false, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev, witems);
    else if constexpr (CLOUDSC_KEEP_KERNEL(real, true, false))
      rc = launch_kseg<real, false, FAST>(st, a, pa, nproma, pa.nitems, &grid, ev, witems);"""),
 ("cloudsc_gpu.hip",
  """        const unsigned nbs = q < S ? (unsigned)((nblocks - q + S - 1) / S) : 0u;
        const unsigned wgs = q < S ? (unsigned)((grid - q + S - 1) / S) : 0u;
        ep->base[q] = pa.base[q] + (unsigned)pa.nseg * nbs * (unsigned)pa.nsub + wgs;""",
  """        const unsigned nbs = q < S ? (unsigned)((nblocks - q + S - 1) / S) : 0u;
        const unsigned wgs = q < S ? (unsigned)((grid - q + S - 1) / S) : 0u;
        const unsigned its = witems[q] >= 0 ? (unsigned)witems[q] : (unsigned)pa.nseg * nbs * (unsigned)pa.nsub;
        ep->base[q] = pa.base[q] + its + wgs;"""),
 # device side
 ("cloudsc_kcache.h",
  """  unsigned long long* clk;
  int lev[kMaxSeg + 1];
};""",
  """  unsigned long long* clk;
  int lev[kMaxSeg + 1];
  const unsigned* wtab;   // wrap schedule (experiment): per stripe [wstride] {unit|seg<<31|produce<<30, l0|l1<<16}
  int wstride;
  int witems[kKsegStripes];
  int ncldtop;            // host side: the wrap schedule's level model
};"""),
 ("cloudsc_kcache.h",
  """  const int items = P.nseg * nsbs;""",
  """  const int items = P.wtab ? P.witems[st] : P.nseg * nsbs;"""),
 ("cloudsc_kcache.h",
  """    const int seg = item / nsbs, r = item - seg * nsbs;""",
  """    int seg, r, l0, l1;
    bool produce;
    if (P.wtab) {
      const unsigned* e = P.wtab + 2 * ((size_t)st * P.wstride + item);
      const unsigned e0 = __builtin_amdgcn_readfirstlane(e[0]), e1 = __builtin_amdgcn_readfirstlane(e[1]);
      r = (int)(e0 & 0x3fffffffu);
      seg = (int)(e0 >> 31);
      produce = ((e0 >> 30) & 1u) != 0u;
      l0 = (int)(e1 & 0xffffu);
      l1 = (int)(e1 >> 16);
    } else {
      seg = item / nsbs;
      r = item - seg * nsbs;
      l0 = P.lev[seg];
      l1 = P.lev[seg + 1];
      produce = seg + 1 < P.nseg;
    }"""),
 ("cloudsc_kcache.h",
  """    if (active) kcache_levels<real, PF, AER>(ka, cpar, b, lo, P.lev[seg], P.lev[seg + 1], cs);
    if (seg + 1 < P.nseg) {""",
  """    if (active) kcache_levels<real, PF, AER>(ka, cpar, b, lo, l0, l1, cs);
    if (produce) {"""),
]
