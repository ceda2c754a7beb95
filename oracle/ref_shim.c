/*
 * ref_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin driver that runs the UNMODIFIED reference C kernel cloudsc_c()
 * (src/cloudsc_c/cloudsc/cloudsc_c.c, compiled from /root/reference by
 * oracle/Makefile into oracle/_ref/libcloudsc_ref.so) on block-layout fields
 * described by cloudsc_amd.h.  It restates what the reference driver does
 * around the kernel (src/cloudsc_c/cloudsc/cloudsc_driver.c:98-217):
 * set the YOMCST/YOETHF globals and the TECLDP struct from the parameter
 * block (load_state.c:538-690), then loop over NPROMA blocks with OpenMP,
 * pre-zero pcovptot and tendency_loc_cld per block (:199-200) and call
 * cloudsc_c(1, bsize, nproma, nlev, ...) (:202-217).
 *
 * No reference source is copied into the repository: this file only includes
 * the reference headers from their original location.
 */
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#include "cloudsc_c.h"     /* from /root/reference/src/cloudsc_c/cloudsc */
#include "cloudsc_amd.h"

static void set_globals(const cloudsc_params_t *p, struct TECLDP *y)
{
  rg = p->rg; rd = p->rd; rcpd = p->rcpd; retv = p->retv; rlvtt = p->rlvtt; rlstt = p->rlstt;
  rlmlt = p->rlmlt; rtt = p->rtt; rv = p->rv;
  r2es = p->r2es; r3les = p->r3les; r3ies = p->r3ies; r4les = p->r4les; r4ies = p->r4ies;
  r5les = p->r5les; r5ies = p->r5ies; r5alvcp = p->r5alvcp; r5alscp = p->r5alscp;
  ralvdcp = p->ralvdcp; ralsdcp = p->ralsdcp; ralfdcp = p->ralfdcp; rtwat = p->rtwat;
  rtice = p->rtice; rticecu = p->rticecu; rtwat_rtice_r = p->rtwat_rtice_r;
  rtwat_rticecu_r = p->rtwat_rticecu_r; rkoop1 = p->rkoop1; rkoop2 = p->rkoop2;
#define T(n) y->n = p->n
  T(ramid); T(rcldiff); T(rcldiff_convi); T(rclcrit); T(rclcrit_sea); T(rclcrit_land); T(rkconv);
  T(rprc1); T(rprc2); T(rcldmax); T(rpecons); T(rvrfactor); T(rprecrhmax); T(rtaumel); T(ramin);
  T(rlmin); T(rkooptau); T(rcldtopp); T(rlcritsnow); T(rsnowlin1); T(rsnowlin2); T(ricehi1);
  T(ricehi2); T(riceinit); T(rvice); T(rvrain); T(rvsnow); T(rthomo); T(rcovpmin); T(rccn);
  T(rnice); T(rccnom); T(rccnss); T(rccnsu); T(rcldtopcf); T(rdepliqrefrate); T(rdepliqrefdepth);
  T(rcl_kkaac); T(rcl_kkbac); T(rcl_kkaau); T(rcl_kkbauq); T(rcl_kkbaun); T(rcl_kk_cloud_num_sea);
  T(rcl_kk_cloud_num_land); T(rcl_ai); T(rcl_bi); T(rcl_ci); T(rcl_di); T(rcl_x1i); T(rcl_x2i);
  T(rcl_x3i); T(rcl_x4i); T(rcl_const1i); T(rcl_const2i); T(rcl_const3i); T(rcl_const4i);
  T(rcl_const5i); T(rcl_const6i); T(rcl_apb1); T(rcl_apb2); T(rcl_apb3); T(rcl_as); T(rcl_bs);
  T(rcl_cs); T(rcl_ds); T(rcl_x1s); T(rcl_x2s); T(rcl_x3s); T(rcl_x4s); T(rcl_const1s);
  T(rcl_const2s); T(rcl_const3s); T(rcl_const4s); T(rcl_const5s); T(rcl_const6s); T(rcl_const7s);
  T(rcl_const8s); T(rdenswat); T(rdensref); T(rcl_ar); T(rcl_br); T(rcl_cr); T(rcl_dr); T(rcl_x1r);
  T(rcl_x2r); T(rcl_x4r); T(rcl_ka273); T(rcl_cdenom1); T(rcl_cdenom2); T(rcl_cdenom3);
  T(rcl_schmidt); T(rcl_dynvisc); T(rcl_const1r); T(rcl_const2r); T(rcl_const3r); T(rcl_const4r);
  T(rcl_fac1); T(rcl_fac2); T(rcl_const5r); T(rcl_const6r); T(rcl_fzrab); T(rcl_fzrbb);
  T(lcldextra); T(lcldbudget); T(nssopt); T(ncldtop); T(naeclbc); T(naecldu); T(naeclom);
  T(naeclss); T(naeclsu); T(nclddiag); T(naercld); T(laerliqautolsp); T(laerliqautocp);
  T(laerliqautocpb); T(laerliqcoll); T(laericesed); T(laericeauto); T(nshapep); T(nshapeq); T(nbeta);
#undef T
  nclv = 5; ncldql = 1; ncldqi = 2; ncldqr = 3; ncldqs = 4; ncldqv = 5;
}

/* The parameter-module globals alone, for callers of cloudsc_c() itself
 * (tests/test_dropin.py calls the reference kernel and the drop-in on one block). */
void cloudsc_ref_set_params(const cloudsc_params_t *p)
{
  static struct TECLDP tecldp;
  yrecldp = &tecldp;
  set_globals(p, yrecldp);
}

/* fp64 only: the reference C kernel is hard-wired to double. */
int cloudsc_ref_run(int nthreads, int ngptot, int nproma, int klev,
                    const cloudsc_params_t *p, const cloudsc_fields_t *f, double *seconds)
{
  if (!p || !f || ngptot <= 0 || nproma <= 0 || klev <= 1) return -1;
  const int nlev = klev;
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  static struct TECLDP tecldp;
  yrecldp = &tecldp;
  set_globals(p, yrecldp);
  const double ptsphy = p->ptsphy;
  /* fields the kernel receives but never reads (tendency_cml_*, pvfa, pdyn*) and
     aerosol fields left NULL by the caller point at one zeroed scratch array */
  double *dummy = calloc((size_t)nblocks * nclv * (nlev + 1) * nproma, sizeof(double));
  if (!dummy) return -5;
#define A(x) ((double *)((x) ? (void *)(x) : (void *)dummy))
  double *pt = A(f->pt), *pq = A(f->pq), *tend_tmp_t = A(f->tendency_tmp_t), *tend_tmp_q = A(f->tendency_tmp_q);
  double *tend_tmp_a = A(f->tendency_tmp_a), *tend_tmp_cld = A(f->tendency_tmp_cld);
  double *pvfl = A(f->pvfl), *pvfi = A(f->pvfi), *phrsw = A(f->phrsw), *phrlw = A(f->phrlw);
  double *pvervel = A(f->pvervel), *pap = A(f->pap), *paph = A(f->paph), *plsm = A(f->plsm);
  int *ktype = (int *)f->ktype;
  double *plu = A(f->plu), *plude = A(f->plude), *psnde = A(f->psnde), *pmfu = A(f->pmfu);
  double *pmfd = A(f->pmfd), *pa = A(f->pa), *pclv = A(f->pclv), *psupsat = A(f->psupsat);
  double *plcrit_aer = A(f->plcrit_aer), *picrit_aer = A(f->picrit_aer), *pre_ice = A(f->pre_ice);
  double *pccn = A(f->pccn), *pnice = A(f->pnice);
  double *tend_loc_t = A(f->tendency_loc_t), *tend_loc_q = A(f->tendency_loc_q);
  double *tend_loc_a = A(f->tendency_loc_a), *tend_loc_cld = A(f->tendency_loc_cld);
  double *pcovptot = A(f->pcovptot), *prainfrac_toprfz = A(f->prainfrac_toprfz);
  double *pfsqlf = A(f->pfsqlf), *pfsqif = A(f->pfsqif), *pfcqnng = A(f->pfcqnng), *pfcqlng = A(f->pfcqlng);
  double *pfsqrf = A(f->pfsqrf), *pfsqsf = A(f->pfsqsf), *pfcqrng = A(f->pfcqrng), *pfcqsng = A(f->pfcqsng);
  double *pfsqltur = A(f->pfsqltur), *pfsqitur = A(f->pfsqitur), *pfplsl = A(f->pfplsl), *pfplsn = A(f->pfplsn);
  double *pfhpsl = A(f->pfhpsl), *pfhpsn = A(f->pfhpsn);
#undef A
  if (nthreads <= 0) nthreads = omp_get_max_threads();
  double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(nthreads) schedule(runtime)
  for (int b = 0; b < nblocks; b++) {
    const int idx = b * nlev * nproma, idxp1 = b * (nlev + 1) * nproma, idx1d = b * nproma;
    const int idx3d = b * nclv * nlev * nproma;
    const int bsize = (ngptot - b * nproma) < nproma ? (ngptot - b * nproma) : nproma;
    for (int i = 0; i < nlev * nproma; i++) pcovptot[idx + i] = 0.0;
    for (int i = 0; i < nclv * nlev * nproma; i++) tend_loc_cld[idx3d + i] = 0.0;
    cloudsc_c(1, bsize, nproma, nlev, ptsphy, &pt[idx], &pq[idx],
              &dummy[idx], &dummy[idx], &dummy[idx], &dummy[idx3d],
              &tend_tmp_t[idx], &tend_tmp_q[idx], &tend_tmp_a[idx], &tend_tmp_cld[idx3d],
              &tend_loc_t[idx], &tend_loc_q[idx], &tend_loc_a[idx], &tend_loc_cld[idx3d],
              &dummy[idx], &pvfl[idx], &pvfi[idx], &dummy[idx], &dummy[idx], &dummy[idx],
              &phrsw[idx], &phrlw[idx], &pvervel[idx], &pap[idx], &paph[idxp1], &plsm[idx1d],
              &ktype[idx1d], &plu[idx], &plude[idx], &psnde[idx], &pmfu[idx], &pmfd[idx],
              &pa[idx], &pclv[idx3d], &psupsat[idx],
              f->plcrit_aer ? &plcrit_aer[idx] : &dummy[idx], f->picrit_aer ? &picrit_aer[idx] : &dummy[idx],
              f->pre_ice ? &pre_ice[idx] : &dummy[idx], f->pccn ? &pccn[idx] : &dummy[idx],
              f->pnice ? &pnice[idx] : &dummy[idx],
              &pcovptot[idx], &prainfrac_toprfz[idx1d], &pfsqlf[idxp1], &pfsqif[idxp1],
              &pfcqnng[idxp1], &pfcqlng[idxp1], &pfsqrf[idxp1], &pfsqsf[idxp1], &pfcqrng[idxp1],
              &pfcqsng[idxp1], &pfsqltur[idxp1], &pfsqitur[idxp1], &pfplsl[idxp1], &pfplsn[idxp1],
              &pfhpsl[idxp1], &pfhpsn[idxp1]);
  }
  double t1 = omp_get_wtime();
  if (seconds) *seconds = t1 - t0;
  free(dummy);
  return 0;
}
