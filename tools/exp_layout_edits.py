# Experiment build for the round-6 layout study in the REAL kernel (tools/layout_kernel_ab.py):
#   python tools/exp_variant.py layoutB tools/exp_layout_edits.py -DCLOUDSC_ONLY_KSEG=8
# KArgs gains two element strides between blocks, one for the inputs and one
# for the outputs (0 = the reference layout's per-kind strides), so the fields
# can live in per-block interleaved arenas ([block][field][rows][nproma]); the
# KSEG kernel computes its block offsets from them once per item (the level and
# species offsets inside a block are unchanged).  cloudsc_exp_set_block_strides
# sets them for the following launches; cloudsc_exp_run launches KSEG with an
# out-of-place plude (read from plude_in in the input arena, written to
# f->plude in the output arena).  Not product code.
EDITS = [
    ("cloudsc_kcache.h",
     """  const DevParams<real>* par;   // the launch's parameter set (device memory, read with scalar loads)
  int ngptot, nproma, klev;
};""",
     """  const DevParams<real>* par;   // the launch's parameter set (device memory, read with scalar loads)
  int ngptot, nproma, klev;
  long long exp_bsi, exp_bso;   // experiment: block strides of the input / output arenas (0 = reference layout)
};"""),
    ("cloudsc_kcache.h",
     """  const size_t u2 = (size_t)b * klev * nproma;                     // [nblocks][klev][nproma]
  const size_t uh = (size_t)b * (klev + 1) * nproma;               // [nblocks][klev+1][nproma]
  const size_t u3 = (size_t)b * 5 * klev * nproma;                 // [nblocks][5][klev][nproma]""",
     """  const size_t bsi = (size_t)A0.exp_bsi, bso = (size_t)A0.exp_bso;
  const size_t u2 = bsi ? (size_t)b * bsi : (size_t)b * klev * nproma;
  const size_t uh = bsi ? (size_t)b * bsi : (size_t)b * (klev + 1) * nproma;
  const size_t u3 = bsi ? (size_t)b * bsi : (size_t)b * 5 * klev * nproma;
  const size_t u2o = bso ? (size_t)b * bso : (size_t)b * klev * nproma;
  const size_t uho = bso ? (size_t)b * bso : (size_t)b * (klev + 1) * nproma;
  const size_t u3o = bso ? (size_t)b * bso : (size_t)b * 5 * klev * nproma;"""),
    ("cloudsc_kcache.h",
     """      store_level(A, u2, u3, k, klev, nproma, los, physics, ls, po);
      flux_level(c, A, uh + (size_t)(k + 1) * nproma, los, cur, ls, po, nb.paph_k, nb.paph_n, cs);""",
     """      store_level(A, u2o, u3o, k, klev, nproma, los, physics, ls, po);
      flux_level(c, A, uho + (size_t)(k + 1) * nproma, los, cur, ls, po, nb.paph_k, nb.paph_n, cs);"""),
    ("cloudsc_kcache.h",
     """        flux_top(c, A, (size_t)b * (A.klev + 1) * nproma, lo);""",
     """        flux_top(c, A, A.exp_bso ? (size_t)b * (size_t)A.exp_bso : (size_t)b * (A.klev + 1) * nproma, lo);"""),
    ("cloudsc_gpu.hip",
     """  a.ngptot = ngptot; a.nproma = nproma; a.klev = klev;
  return a;
}""",
     """  a.ngptot = ngptot; a.nproma = nproma; a.klev = klev;
  a.exp_bsi = g_exp_bsi; a.exp_bso = g_exp_bso;
  return a;
}"""),
    ("cloudsc_gpu.hip",
     """namespace {

template <typename real>
KArgs<real> make_args(""",
     """long long g_exp_bsi = 0, g_exp_bso = 0;
extern "C" int cloudsc_exp_set_block_strides(long long bsi, long long bso) {
  g_exp_bsi = bsi;
  g_exp_bso = bso;
  return 0;
}

namespace {

template <typename real>
KArgs<real> make_args("""),
    ("cloudsc_gpu.hip",
     """int cloudsc_gpu_check(int device, void* stream, int variant, void* scratch) {""",
     """int cloudsc_exp_run(int device, void* stream, int precision, int ngptot, int nproma, int klev,
                    const cloudsc_fields_t* f, void* scratch, const void* plude_in) {
  return gpu_run_impl(device, stream, precision, CLOUDSC_VARIANT_KSEG, ngptot, nproma, klev, f, scratch, plude_in,
                      nullptr);
}

int cloudsc_gpu_check(int device, void* stream, int variant, void* scratch) {"""),
]
