/*
 * cloudsc_c_dropin.c -- the reference C kernel's entry point cloudsc_c()
 * (src/cloudsc_c/cloudsc/cloudsc_c.h:18-29), implemented by this library, so
 * that the reference C dwarf links against it UNMODIFIED in place of
 * cloudsc_c.c: dwarf_cloudsc.c, cloudsc_driver.c, load_state.c,
 * cloudsc_validate.c, yomcst_c.c, yoethf_c.c, yoecldp_c.c and mycpu.c as they
 * are, with this file's library on the link line instead of cloudsc_c.o
 * (tests/test_dropin.py).
 *
 * It is built inside the reference's source tree the way a maintainer would
 * add it: against the reference's own parameter-module headers, whose globals
 * (YOMCST rg, rd, ...; YOETHF r2es, ...; struct TECLDP *yrecldp) the driver
 * fills in load_state() (load_state.c:538-690) and this file reads on every
 * call.  Including cloudsc_c.h makes the compiler check the definition below
 * against the reference's declaration.  Make target `dropin`
 * (dwarf-p-cloudsc_amd/Makefile, REF_C = that directory).
 *
 * Two builds of this file:
 *   libcloudsc_c_amd.so      cloudsc_cpu_run on the calling thread (the
 *                            driver's OpenMP loop supplies the threads): the
 *                            library's host build of the kernel
 *   libcloudsc_c_amd_gpu.so  (-DCLOUDSC_DROPIN_GPU) cloudsc_host_run on HIP
 *                            device 0: the block is copied to the MI355X,
 *                            computed by the k-caching kernel and copied back
 * Both give the reference kernel's bits (fp64).  A third build,
 * libcloudsc_c_amd_gpu_prof.so (-DCLOUDSC_DROPIN_PROFILE as well), profiles
 * every call (cloudsc_host_run_profile) and prints where the time went when
 * the dwarf exits (tools/dropin_cost.py).
 *
 * Semantics of the call (cloudsc_c.c:19-2587): one NPROMA block of klon
 * columns, of which columns kidia..kfdia (1-based) are computed; arrays are
 * [klev][klon], [klev+1][klon], [nclv][klev][klon] and [klon].  The columns
 * kidia..kfdia are a block of kfdia-kidia+1 columns with leading dimension
 * klon once every pointer is advanced by kidia-1 elements.  The arguments the
 * reference kernel does not read (tendency_cml_*, pvfa, pdyn*, pccn,
 * plcrit_aer) are not read here either.  The reference returns 0; so does
 * this, or a negative CLOUDSC_E* code with a message on stderr (the driver
 * ignores the value, cloudsc_driver.c:195).
 */
#include <stdio.h>
#ifdef CLOUDSC_DROPIN_PROFILE
#include <pthread.h>
#include <stdlib.h>
#endif

#include "cloudsc_c.h"      /* the reference declaration (and yomcst_c.h, yoethf_c.h, yoecldp_c.h) */
#include "cloudsc_amd.h"

static void params_from_modules(cloudsc_params_t *p, double ptsphy) {
  const struct TECLDP *y = yrecldp;
  p->ptsphy = ptsphy;
  p->rg = rg; p->rd = rd; p->rcpd = rcpd; p->retv = retv; p->rlvtt = rlvtt; p->rlstt = rlstt;
  p->rlmlt = rlmlt; p->rtt = rtt; p->rv = rv;
  p->r2es = r2es; p->r3les = r3les; p->r3ies = r3ies; p->r4les = r4les; p->r4ies = r4ies;
  p->r5les = r5les; p->r5ies = r5ies; p->r5alvcp = r5alvcp; p->r5alscp = r5alscp;
  p->ralvdcp = ralvdcp; p->ralsdcp = ralsdcp; p->ralfdcp = ralfdcp; p->rtwat = rtwat; p->rtice = rtice;
  p->rticecu = rticecu; p->rtwat_rtice_r = rtwat_rtice_r; p->rtwat_rticecu_r = rtwat_rticecu_r;
  p->rkoop1 = rkoop1; p->rkoop2 = rkoop2;
#define T(x) p->x = y->x;
  T(ramid) T(rcldiff) T(rcldiff_convi) T(rclcrit) T(rclcrit_sea) T(rclcrit_land) T(rkconv) T(rprc1) T(rprc2)
  T(rcldmax) T(rpecons) T(rvrfactor) T(rprecrhmax) T(rtaumel) T(ramin) T(rlmin) T(rkooptau) T(rcldtopp)
  T(rlcritsnow) T(rsnowlin1) T(rsnowlin2) T(ricehi1) T(ricehi2) T(riceinit) T(rvice) T(rvrain) T(rvsnow)
  T(rthomo) T(rcovpmin) T(rccn) T(rnice) T(rccnom) T(rccnss) T(rccnsu) T(rcldtopcf) T(rdepliqrefrate)
  T(rdepliqrefdepth) T(rcl_kkaac) T(rcl_kkbac) T(rcl_kkaau) T(rcl_kkbauq) T(rcl_kkbaun)
  T(rcl_kk_cloud_num_sea) T(rcl_kk_cloud_num_land) T(rcl_ai) T(rcl_bi) T(rcl_ci) T(rcl_di)
  T(rcl_x1i) T(rcl_x2i) T(rcl_x3i) T(rcl_x4i) T(rcl_const1i) T(rcl_const2i) T(rcl_const3i) T(rcl_const4i)
  T(rcl_const5i) T(rcl_const6i) T(rcl_apb1) T(rcl_apb2) T(rcl_apb3) T(rcl_as) T(rcl_bs) T(rcl_cs) T(rcl_ds)
  T(rcl_x1s) T(rcl_x2s) T(rcl_x3s) T(rcl_x4s) T(rcl_const1s) T(rcl_const2s) T(rcl_const3s) T(rcl_const4s)
  T(rcl_const5s) T(rcl_const6s) T(rcl_const7s) T(rcl_const8s) T(rdenswat) T(rdensref) T(rcl_ar) T(rcl_br)
  T(rcl_cr) T(rcl_dr) T(rcl_x1r) T(rcl_x2r) T(rcl_x4r) T(rcl_ka273) T(rcl_cdenom1) T(rcl_cdenom2)
  T(rcl_cdenom3) T(rcl_schmidt) T(rcl_dynvisc) T(rcl_const1r) T(rcl_const2r) T(rcl_const3r) T(rcl_const4r)
  T(rcl_fac1) T(rcl_fac2) T(rcl_const5r) T(rcl_const6r) T(rcl_fzrab) T(rcl_fzrbb) T(nshapep) T(nshapeq)
  T(lcldextra) T(lcldbudget) T(nssopt) T(ncldtop) T(naeclbc) T(naecldu) T(naeclom) T(naeclss) T(naeclsu)
  T(nclddiag) T(naercld) T(laerliqautolsp) T(laerliqautocp) T(laerliqautocpb) T(laerliqcoll)
  T(laericesed) T(laericeauto) T(nbeta)
#undef T
}

#ifdef CLOUDSC_DROPIN_PROFILE
/* the sums of every cloudsc_host_run call of the run, on stderr at exit */
static void print_profile(void) {
  cloudsc_host_run_profile_t p;
  if (cloudsc_host_run_profile(-1, &p) != CLOUDSC_OK) return;
  fprintf(stderr,
          "CLOUDSC_C_DROPIN_PROFILE calls=%lld total_ms=%.3f alloc_ms=%.3f setup_ms=%.3f pack_ms=%.3f "
          "enqueue_ms=%.3f h2d_ms=%.3f kernel_ms=%.3f d2h_ms=%.3f wait_ms=%.3f unpack_ms=%.3f max_call_ms=%.3f "
          "first_calls=%lld first_calls_ms=%.3f\n",
          p.calls, p.total_ms, p.alloc_ms, p.setup_ms, p.pack_ms, p.enqueue_ms, p.h2d_ms, p.kernel_ms, p.d2h_ms,
          p.wait_ms, p.unpack_ms, p.max_call_ms, p.first_calls, p.first_calls_ms);
}
static pthread_once_t g_prof_once = PTHREAD_ONCE_INIT;
static void start_profile(void) {
  cloudsc_host_run_profile(1, NULL);
  atexit(print_profile);
}
#endif

int cloudsc_c(int kidia, int kfdia, int klon, int klev, double ptsphy, double * restrict v_pt, double * restrict v_pq,
              double * restrict v_tendency_cml_t, double * restrict v_tendency_cml_q, double * restrict v_tendency_cml_a,
              double * restrict v_tendency_cml_cld,
              double * restrict v_tendency_tmp_t, double * restrict v_tendency_tmp_q, double * restrict v_tendency_tmp_a,
              double * restrict v_tendency_tmp_cld,
              double * restrict v_tendency_loc_t, double * restrict v_tendency_loc_q, double * restrict v_tendency_loc_a,
              double * restrict v_tendency_loc_cld,
              double * restrict v_pvfa, double * restrict v_pvfl, double * restrict v_pvfi, double * restrict v_pdyna,
              double * restrict v_pdynl, double * restrict v_pdyni,
              double * restrict v_phrsw, double * restrict v_phrlw, double * restrict v_pvervel, double * restrict v_pap,
              double * restrict v_paph, double * restrict v_plsm,
              int * restrict v_ktype, double * restrict v_plu, double * restrict v_plude, double * restrict v_psnde,
              double * restrict v_pmfu,
              double * restrict v_pmfd, double * restrict v_pa, double * restrict v_pclv, double * restrict v_psupsat,
              double * restrict v_plcrit_aer, double * restrict v_picrit_aer,
              double * restrict v_pre_ice, double * restrict v_pccn, double * restrict v_pnice,
              double * restrict v_pcovptot, double * restrict v_prainfrac_toprfz, double * restrict v_pfsqlf,
              double * restrict v_pfsqif, double * restrict v_pfcqnng, double * restrict v_pfcqlng,
              double * restrict v_pfsqrf, double * restrict v_pfsqsf, double * restrict v_pfcqrng,
              double * restrict v_pfcqsng, double * restrict v_pfsqltur, double * restrict v_pfsqitur,
              double * restrict v_pfplsl, double * restrict v_pfplsn, double * restrict v_pfhpsl,
              double * restrict v_pfhpsn) {
  (void)v_tendency_cml_t; (void)v_tendency_cml_q; (void)v_tendency_cml_a; (void)v_tendency_cml_cld;
  (void)v_pvfa; (void)v_pdyna; (void)v_pdynl; (void)v_pdyni;
  if (kidia < 1 || kfdia < kidia || kfdia > klon || klev < 2 || !yrecldp) {
    fprintf(stderr, "cloudsc_c (MI355X drop-in): invalid block kidia=%d kfdia=%d klon=%d klev=%d\n", kidia, kfdia,
            klon, klev);
    return CLOUDSC_EINVAL;
  }
  cloudsc_params_t p;
  params_from_modules(&p, ptsphy);
  const long o = kidia - 1;   /* first computed column: every array starts there */
  cloudsc_fields_t f = {
      v_pt + o, v_pq + o, v_tendency_tmp_t + o, v_tendency_tmp_q + o, v_tendency_tmp_a + o, v_tendency_tmp_cld + o,
      v_pvfl + o, v_pvfi + o, v_phrsw + o, v_phrlw + o, v_pvervel + o, v_pap + o, v_paph + o, v_plsm + o,
      v_ktype + o, v_plu + o, v_psnde + o, v_pmfu + o, v_pmfd + o, v_pa + o, v_pclv + o, v_psupsat + o,
      v_plcrit_aer + o, v_picrit_aer + o, v_pre_ice + o, v_pccn + o, v_pnice + o,
      v_plude + o,
      v_tendency_loc_t + o, v_tendency_loc_q + o, v_tendency_loc_a + o, v_tendency_loc_cld + o,
      v_pcovptot + o, v_prainfrac_toprfz + o,
      v_pfsqlf + o, v_pfsqif + o, v_pfcqnng + o, v_pfcqlng + o, v_pfsqrf + o, v_pfsqsf + o, v_pfcqrng + o,
      v_pfcqsng + o, v_pfsqltur + o, v_pfsqitur + o, v_pfplsl + o, v_pfplsn + o, v_pfhpsl + o, v_pfhpsn + o};
  const int ncols = kfdia - kidia + 1;
#ifdef CLOUDSC_DROPIN_PROFILE
  pthread_once(&g_prof_once, start_profile);
#endif
#ifdef CLOUDSC_DROPIN_GPU
  /* one workgroup per block up to 256 columns, else the persistent kernel */
  const int variant = klon <= 256 ? CLOUDSC_VARIANT_KCACHE : CLOUDSC_VARIANT_KSEG;
  const int rc = cloudsc_host_run(0, CLOUDSC_FP64, variant, ncols, klon, klev, &p, &f);
#else
  const int rc = cloudsc_cpu_run(1, ncols, klon, klev, &p, &f, NULL);
#endif
  if (rc != CLOUDSC_OK)
    fprintf(stderr, "cloudsc_c (MI355X drop-in): %s%s%s\n", cloudsc_strerror(rc),
            rc == CLOUDSC_EHIP ? ": " : "", rc == CLOUDSC_EHIP ? cloudsc_last_hip_error() : "");
  return rc;
}
