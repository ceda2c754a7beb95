/*
 * cloudsc_oracle.c -- TEST INFRASTRUCTURE ONLY (see cloudsc_oracle.h).
 *
 * CPU restatement of the reference CLOUDSC kernel,
 * src/cloudsc_c/cloudsc/cloudsc_c.c:19-2587 (lukasm91/dwarf-p-cloudsc).
 * The reference sweeps phase by phase over a block of columns with
 * level-sized temporaries; this restatement walks ONE column at a time through
 * one fused level loop (the k-caching order of
 * src/cloudsc_gpu/cloudsc_gpu_scc_k_caching_mod.F90), carrying only the state
 * that crosses levels.  Every floating-point expression keeps the reference's
 * operand order and parenthesisation so that, compiled with
 * -ffp-contract=off against the same libm, results are bit-identical to the
 * reference build (checked by tests/test_oracle.py).
 *
 * Compiled twice: as-is for fp64 (cloudsc_oracle_block_dp) and with
 * -DORACLE_SP for the fp32 path (cloudsc_oracle_block_sp: float storage,
 * float constants, expf/powf -- the JPRB=sp semantics of parkind1.F90:40-43).
 *
 * Hard-wired physics switches of the reference (cloudsc_c.c:367-382):
 * IWARMRAIN=2, IEVAPRAIN=2, IEVAPSNOW=1, IDEPICE=1.  The alternative branches
 * are unreachable in the reference and are not restated.  Data-driven switches
 * (NSSOPT 0-3, NCLDTOP, LAERICESED, LAERICEAUTO) are honoured.
 */
#include "cloudsc_oracle.h"

#include <float.h>
#include <math.h>
#include <stddef.h>
#include <omp.h>

/* Sensitivity probe (fp32 only, off by default): with a non-zero seed every
 * expf/powf result is moved by -1, 0 or +1 ulp, chosen by a hash of its
 * arguments and the seed -- a libm that is faithful but not glibc's.  The
 * outputs' response to it is the noise floor against which a different
 * single-precision exp/pow (the GPU's float-internal forms) is gated
 * (tests/test_gpu_parity.py, SURVEY.md §8c "±1-ulp emulation"). */
extern unsigned cloudsc_oracle_libm_nudge_seed;

#ifdef ORACLE_SP
typedef float real;
static inline float nudge_f(float r, unsigned a, unsigned b)
{
  const unsigned seed = cloudsc_oracle_libm_nudge_seed;
  if (!seed || !(r == r) || r == 0.0f || fabsf(r) > FLT_MAX) return r;
  unsigned h = (a * 2654435761u) ^ (b * 2246822519u) ^ (seed * 3266489917u);
  h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
  const int d = (int)(h % 3u) - 1;
  return d == 0 ? r : nextafterf(r, d > 0 ? INFINITY : -INFINITY);
}
static inline unsigned fbits(float x) { union { float f; unsigned u; } v = {x}; return v.u; }
static inline float expf_probe(float x) { return nudge_f(expf(x), fbits(x), 0x9e3779b9u); }
static inline float powf_probe(float x, float y) { return nudge_f(powf(x, y), fbits(x), fbits(y)); }
#define L(x) x##f
#define EXP expf_probe
#define POW powf_probe
#define SQRT sqrtf
#define FMIN fminf
#define FMAX fmaxf
#define FABS fabsf
#define COPYSIGN copysignf
#define REAL_EPSILON FLT_EPSILON
#define BLOCK_FN cloudsc_oracle_block_sp
#else
typedef double real;
#define L(x) x
#define EXP exp
#define POW pow
#define SQRT sqrt
#define FMIN fmin
#define FMAX fmax
#define FABS fabs
#define COPYSIGN copysign
#define REAL_EPSILON DBL_EPSILON
#define BLOCK_FN cloudsc_oracle_block_dp
#endif

/* species indices (NCLDQL..NCLDQV, 0-based) */
enum { QL = 0, QI = 1, QR = 2, QS = 3, QV = 4, NCLV = 5 };

/* iphase (cloudsc_c.c:400-404): 0 vapour, 1 liquid, 2 ice */
static const int IPHASE[NCLV] = {1, 2, 1, 2, 0};
/* imelt (cloudsc_c.c:408-412), 0-based target species */
static const int IMELT[NCLV] = {QI, QR, QS, QR, -99};

/* Parameters cast to the working precision once. */
typedef struct {
  real ptsphy, rg, rd, rcpd, retv, rlvtt, rlstt, rlmlt, rtt, rv;
  real r2es, r3les, r3ies, r4les, r4ies, r5les, r5ies, r5alvcp, r5alscp;
  real ralvdcp, ralsdcp, ralfdcp, rtwat, rtice, rtwat_rtice_r, rkoop1, rkoop2;
  real ramid, rcldiff, rcldiff_convi, rclcrit_sea, rclcrit_land, rprecrhmax, rtaumel, ramin, rlmin;
  real rkooptau, rlcritsnow, rsnowlin1, rsnowlin2, riceinit, rvice, rvrain, rvsnow, rthomo;
  real rcovpmin, rnice, rcldtopcf, rdepliqrefrate, rdepliqrefdepth, rvrfactor, rpecons;
  real rcl_kkaac, rcl_kkbac, rcl_kkaau, rcl_kkbauq, rcl_kkbaun, rcl_kk_cloud_num_sea, rcl_kk_cloud_num_land;
  real rcl_const1s, rcl_const7s, rcl_const8s, rdensref, rcl_ka273, rcl_cdenom1, rcl_cdenom2, rcl_cdenom3;
  real rcl_const1r, rcl_const2r, rcl_const3r, rcl_const4r, rcl_fac1, rcl_fac2, rcl_const5r, rcl_const6r;
  real rcl_fzrab;
  int nssopt, ncldtop, laericesed, laericeauto;
} prm_t;

static void load_params(const cloudsc_params_t *p, prm_t *q)
{
#define CP(n) q->n = (real)p->n
  CP(ptsphy); CP(rg); CP(rd); CP(rcpd); CP(retv); CP(rlvtt); CP(rlstt); CP(rlmlt); CP(rtt); CP(rv);
  CP(r2es); CP(r3les); CP(r3ies); CP(r4les); CP(r4ies); CP(r5les); CP(r5ies); CP(r5alvcp); CP(r5alscp);
  CP(ralvdcp); CP(ralsdcp); CP(ralfdcp); CP(rtwat); CP(rtice); CP(rtwat_rtice_r); CP(rkoop1); CP(rkoop2);
  CP(ramid); CP(rcldiff); CP(rcldiff_convi); CP(rclcrit_sea); CP(rclcrit_land); CP(rprecrhmax);
  CP(rtaumel); CP(ramin); CP(rlmin); CP(rkooptau); CP(rlcritsnow); CP(rsnowlin1); CP(rsnowlin2);
  CP(riceinit); CP(rvice); CP(rvrain); CP(rvsnow); CP(rthomo); CP(rcovpmin); CP(rnice); CP(rcldtopcf);
  CP(rdepliqrefrate); CP(rdepliqrefdepth); CP(rvrfactor); CP(rpecons);
  CP(rcl_kkaac); CP(rcl_kkbac); CP(rcl_kkaau); CP(rcl_kkbauq); CP(rcl_kkbaun);
  CP(rcl_kk_cloud_num_sea); CP(rcl_kk_cloud_num_land); CP(rcl_const1s); CP(rcl_const7s); CP(rcl_const8s);
  CP(rdensref); CP(rcl_ka273); CP(rcl_cdenom1); CP(rcl_cdenom2); CP(rcl_cdenom3); CP(rcl_const1r);
  CP(rcl_const2r); CP(rcl_const3r); CP(rcl_const4r); CP(rcl_fac1); CP(rcl_fac2); CP(rcl_const5r);
  CP(rcl_const6r); CP(rcl_fzrab);
#undef CP
  q->nssopt = p->nssopt; q->ncldtop = p->ncldtop;
  q->laericesed = p->laericesed; q->laericeauto = p->laericeauto;
}

/* FOEALFA (fcttre.func.h; inlined at cloudsc_c.c:588 etc.); pow(x,2) == x*x */
static inline real foealfa(const prm_t *c, real t)
{
  real x = (FMAX(c->rtice, FMIN(c->rtwat, t)) - c->rtice) * c->rtwat_rtice_r;
  return FMIN(L(1.0), x * x);
}
/* the two saturation exponentials, FOEELIQ/FOEEICE without the R2ES factor */
static inline real exp_liq(const prm_t *c, real t) { return EXP((c->r3les * (t - c->rtt)) / (t - c->r4les)); }
static inline real exp_ice(const prm_t *c, real t) { return EXP((c->r3ies * (t - c->rtt)) / (t - c->r4ies)); }
/* FOEDEM-like term of the condensation limiter (cloudsc_c.c:1166) */
static inline real foedem_term(const prm_t *c, real t, real alfa)
{
  real dl = t - c->r4les, di = t - c->r4ies;
  return ((alfa * c->r5alvcp) * (L(1.0) / (dl * dl))) + (((L(1.0) - alfa) * c->r5alscp) * (L(1.0) / (di * di)));
}
/* mixed-phase saturation vapour pressure * r2es (FOEEWM, cloudsc_c.c:1162) */
static inline real foeewm(const prm_t *c, real t)
{
  real a = foealfa(c, t);
  return c->r2es * (a * exp_liq(c, t) + (L(1.0) - a) * exp_ice(c, t));
}

#define IX2(k)    ((size_t)(k) * klon + jl)                     /* [lev][klon]        */
#define IX3(m, k) (((size_t)(m) * klev + (k)) * klon + jl)      /* [nclv][lev][klon]  */

int BLOCK_FN(const cloudsc_params_t *p, int kidia, int kfdia, int klon, int klev,
             const cloudsc_fields_t *f)
{
  prm_t cc, *c = &cc;
  load_params(p, c);

  const real *pt = f->pt, *pq = f->pq, *ttt = f->tendency_tmp_t, *ttq = f->tendency_tmp_q;
  const real *tta = f->tendency_tmp_a, *ttcld = f->tendency_tmp_cld, *pvfl = f->pvfl, *pvfi = f->pvfi;
  const real *phrsw = f->phrsw, *phrlw = f->phrlw, *pvervel = f->pvervel, *pap = f->pap;
  const real *paph = f->paph, *plsm = f->plsm, *plu = f->plu, *psnde = f->psnde;
  const real *pmfu = f->pmfu, *pmfd = f->pmfd, *pa = f->pa, *pclv = f->pclv, *psupsat = f->psupsat;
  const real *picrit_aer = f->picrit_aer, *pre_ice = f->pre_ice, *pnice = f->pnice;
  const int *ktype = f->ktype;
  real *plude = f->plude;
  real *tlt = f->tendency_loc_t, *tlq = f->tendency_loc_q, *tla = f->tendency_loc_a;
  real *tlcld = f->tendency_loc_cld, *pcovptot = f->pcovptot, *prainfrac = f->prainfrac_toprfz;
  real *pfsqlf = f->pfsqlf, *pfsqif = f->pfsqif, *pfcqnng = f->pfcqnng, *pfcqlng = f->pfcqlng;
  real *pfsqrf = f->pfsqrf, *pfsqsf = f->pfsqsf, *pfcqrng = f->pfcqrng, *pfcqsng = f->pfcqsng;
  real *pfsqltur = f->pfsqltur, *pfsqitur = f->pfsqitur, *pfplsl = f->pfplsl, *pfplsn = f->pfplsn;
  real *pfhpsl = f->pfhpsl, *pfhpsn = f->pfhpsn;

  /* 0. constants (cloudsc_c.c:360-456) */
  const real zepsilon = L(100.0) * REAL_EPSILON;
  const real zqtmst = L(1.0) / c->ptsphy;
  const real zrdcp = c->rd / c->rcpd;
  const real zepsec = L(1.0e-14);
  const real zrg_r = L(1.0) / c->rg;
  const real zrldcp = L(1.0) / (c->ralsdcp - c->ralvdcp);
  const real ztw1 = L(1329.31000000000), ztw2 = L(0.00746150000000000), ztw3 = L(85000.0000000000);
  const real ztw4 = L(40.6370000000000), ztw5 = L(275.000000000000);
  real zvqx[NCLV] = {L(0.0), c->rvice, c->rvrain, c->rvsnow, L(0.0)};
  int llfall[NCLV];
  for (int m = 0; m < NCLV; m++) llfall[m] = zvqx[m] > L(0.0);
  llfall[QI] = 0;                        /* ice still sediments (cloudsc_c.c:456) */
  const int ncldtop0 = c->ncldtop - 1;   /* first physics level, 0-based */

  for (int jl = kidia - 1; jl <= kfdia - 1; jl++) {
    /* ---- state carried from level to level (one column) ---- */
    real t_prev = L(0.0), a_prev = L(0.0), pap_prev = L(0.0);   /* ztp1, za, pap at k-1 */
    real zanewm1 = L(0.0), zcovptot = L(0.0), zcovpmax = L(0.0), zcldtopdist = L(0.0);
    real zqxnm1[NCLV] = {0};
    real zpfplsx[NCLV] = {0};              /* precip fluxes arriving at level k (zpfplsx[:][k]) */
    real fl_lf = 0, fl_if = 0, fl_lng = 0, fl_nng = 0, fl_ltur = 0, fl_itur = 0; /* running flux sums */
    real rainfrac = L(0.0);
    const real paph_sfc = paph[IX2(klev)];
    const real zpaphd = L(1.0) / paph_sfc; (void)zpaphd;  /* ztrpaus (cloudsc_c.c:697-712) is unused */

    /* level 0 of the half-level fluxes (cloudsc_c.c:2532-2543) */
    pfsqlf[IX2(0)] = 0; pfsqif[IX2(0)] = 0; pfsqrf[IX2(0)] = 0; pfsqsf[IX2(0)] = 0;
    pfcqlng[IX2(0)] = 0; pfcqnng[IX2(0)] = 0; pfcqrng[IX2(0)] = 0; pfcqsng[IX2(0)] = 0;
    pfsqltur[IX2(0)] = 0; pfsqitur[IX2(0)] = 0;
    pfplsl[IX2(0)] = zpfplsx[QR] + zpfplsx[QL];
    pfplsn[IX2(0)] = zpfplsx[QS] + zpfplsx[QI];
    pfhpsl[IX2(0)] = -c->rlvtt * pfplsl[IX2(0)];
    pfhpsn[IX2(0)] = -c->rlstt * pfplsn[IX2(0)];

    for (int k = 0; k < klev; k++) {
      /* ===== 1. initial values at this level (cloudsc_c.c:462-485) ===== */
      real ztp1 = pt[IX2(k)] + c->ptsphy * ttt[IX2(k)];
      real zqx[NCLV], zqx0[NCLV], zlneg[NCLV] = {0};
      zqx[QV] = pq[IX2(k)] + c->ptsphy * ttq[IX2(k)];
      zqx0[QV] = pq[IX2(k)] + c->ptsphy * ttq[IX2(k)];
      real za = pa[IX2(k)] + c->ptsphy * tta[IX2(k)];
      const real zaorig = pa[IX2(k)] + c->ptsphy * tta[IX2(k)];
      for (int m = 0; m < 4; m++) {
        zqx[m] = pclv[IX3(m, k)] + c->ptsphy * ttcld[IX3(m, k)];
        zqx0[m] = pclv[IX3(m, k)] + c->ptsphy * ttcld[IX3(m, k)];
      }
      real ttend = L(0.0), qtend = L(0.0);     /* tendency_loc_t/q, zero-initialised (:415-421) */
      real ctend[4] = {0, 0, 0, 0};

      /* tidy up very small cloud cover or total cloud water (:519-541) */
      if (zqx[QL] + zqx[QI] < c->rlmin || za < c->ramin) {
        real zqadj;
        zlneg[QL] = zlneg[QL] + zqx[QL];
        zqadj = zqx[QL] * zqtmst;
        qtend = qtend + zqadj;
        ttend = ttend - c->ralvdcp * zqadj;
        zqx[QV] = zqx[QV] + zqx[QL];
        zqx[QL] = L(0.0);
        zlneg[QI] = zlneg[QI] + zqx[QI];
        zqadj = zqx[QI] * zqtmst;
        qtend = qtend + zqadj;
        ttend = ttend - c->ralsdcp * zqadj;
        zqx[QV] = zqx[QV] + zqx[QI];
        zqx[QI] = L(0.0);
        za = L(0.0);
      }
      /* tidy up small CLV variables (:547-575) */
      for (int m = 0; m < 4; m++) {
        if (zqx[m] < c->rlmin) {
          zlneg[m] = zlneg[m] + zqx[m];
          real zqadj = zqx[m] * zqtmst;
          qtend = qtend + zqadj;
          if (IPHASE[m] == 1) ttend = ttend - c->ralvdcp * zqadj;
          if (IPHASE[m] == 2) ttend = ttend - c->ralsdcp * zqadj;
          zqx[QV] = zqx[QV] + zqx[m];
          zqx[m] = L(0.0);
        }
      }
      /* saturation values (:583-609) */
      const real e_liq = exp_liq(c, ztp1), e_ice = exp_ice(c, ztp1);
      const real zfoealfa = foealfa(c, ztp1);
      const real zfoeewmt = FMIN((c->r2es * (zfoealfa * e_liq + (L(1.0) - zfoealfa) * e_ice)) / pap[IX2(k)], L(0.5));
      real zqsmix = zfoeewmt;
      zqsmix = zqsmix / (L(1.0) - c->retv * zqsmix);
      const real zalfa_d = FMAX(L(0.0), COPYSIGN(L(1.0), ztp1 - c->rtt));
      real zfoeew = FMIN((zalfa_d * (c->r2es * e_liq) + (L(1.0) - zalfa_d) * (c->r2es * e_ice)) / pap[IX2(k)], L(0.5));
      zfoeew = FMIN(L(0.5), zfoeew);
      const real zqsice = zfoeew / (L(1.0) - c->retv * zfoeew);
      const real zfoeeliqt = FMIN((c->r2es * e_liq) / pap[IX2(k)], L(0.5));
      real zqsliq = zfoeeliqt;
      zqsliq = zqsliq / (L(1.0) - c->retv * zqsliq);
      /* clip cloud fraction, liquid/ice fractions (:620-640) */
      za = FMAX(L(0.0), FMIN(L(1.0), za));
      const real zli = zqx[QL] + zqx[QI];
      real zliqfrac, zicefrac;
      if (zli > c->rlmin) {
        zliqfrac = zqx[QL] / zli;
        zicefrac = L(1.0) - zliqfrac;
      } else {
        zliqfrac = L(0.0);
        zicefrac = L(0.0);
      }

      real zqxn[NCLV];
      real plude_k = plude[IX2(k)];
      real zcovptot_out = L(0.0);
      real atend = L(0.0);
      int physics = (k >= ncldtop0);

      if (physics) {
        /* ===== 3. physics (cloudsc_c.c:732-2508) ===== */
        const real pap_k = pap[IX2(k)];
        real zqxfg[NCLV];
        for (int m = 0; m < NCLV; m++) zqxfg[m] = zqx[m];
        real zsolqa[NCLV][NCLV] = {{0}}, zsolqb[NCLV][NCLV] = {{0}};
        real zfallsrce[NCLV] = {0}, zfallsink[NCLV] = {0}, zconvsrce[NCLV] = {0}, zconvsink[NCLV] = {0};
        real zpsupsatsrce[NCLV] = {0};
        real zlicld, zqpretot = L(0.0), zlfinalsum = L(0.0), zsolab = L(0.0), zsolac = L(0.0);
        real zldefr = L(0.0);

        /* 3.0 derived variables (:799-841) */
        const real zdp = paph[IX2(k + 1)] - paph[IX2(k)];
        const real zgdp = c->rg / zdp;
        const real zrho = pap_k / (c->rd * ztp1);
        const real zdtgdp = c->ptsphy * zgdp;
        const real zrdtgdp = zdp * (L(1.0) / (c->ptsphy * c->rg));
        real zfacw, zcor, zfaci, zfac;
        {
          real d = ztp1 - c->r4les;
          zfacw = c->r5les / (d * d);
        }
        zcor = L(1.0) / (L(1.0) - c->retv * zfoeeliqt);
        const real zdqsliqdt = (zfacw * zcor) * zqsliq;
        const real zcorqsliq = L(1.0) + c->ralvdcp * zdqsliqdt; (void)zcorqsliq;
        {
          real d = ztp1 - c->r4ies;
          zfaci = c->r5ies / (d * d);
        }
        zcor = L(1.0) / (L(1.0) - c->retv * zfoeew);
        const real zdqsicedt = (zfaci * zcor) * zqsice;
        const real zcorqsice = L(1.0) + c->ralsdcp * zdqsicedt;
        const real zalfaw0 = zfoealfa;
        zfac = zalfaw0 * zfacw + (L(1.0) - zalfaw0) * zfaci;
        zcor = L(1.0) / (L(1.0) - c->retv * zfoeewmt);
        const real zdqsmixdt = (zfac * zcor) * zqsmix;
        const real alfa_t = foealfa(c, ztp1);
        const real zcorqsmix = L(1.0) + (alfa_t * c->ralvdcp + (L(1.0) - alfa_t) * c->ralsdcp) * zdqsmixdt;
        const real zevaplimmix = FMAX((zqsmix - zqx[QV]) / zcorqsmix, L(0.0));
        const real zevaplimice = FMAX((zqsice - zqx[QV]) / zcorqsice, L(0.0)); (void)zevaplimice;
        real ztmpa = L(1.0) * L(1.0) / FMAX(za, zepsec);
        real zliqcld = zqx[QL] * ztmpa;
        real zicecld = zqx[QI] * ztmpa;
        zlicld = zliqcld + zicecld;

        /* evaporate very small amounts of liquid and ice (:846-859) */
        if (zqx[QL] < c->rlmin) {
          zsolqa[QL][QV] = zqx[QL];
          zsolqa[QV][QL] = -zqx[QL];
        }
        if (zqx[QI] < c->rlmin) {
          zsolqa[QI][QV] = zqx[QI];
          zsolqa[QV][QI] = -zqx[QI];
        }

        /* 3.1 ice supersaturation adjustment (:874-954) */
        const real zfokoop = FMIN(c->rkoop1 - c->rkoop2 * ztp1,
                                  (c->r2es * e_liq) * L(1.0) / (c->r2es * e_ice));
        if (c->nssopt == 0 || ztp1 >= c->rtt) {
          zfac = L(1.0);
          zfaci = L(1.0);
        } else {
          zfac = za + zfokoop * (L(1.0) - za);
          zfaci = c->ptsphy / c->rkooptau;
        }
        real zsupsat;
        if (za > L(1.0) - c->ramin) {
          zsupsat = FMAX((zqx[QV] - zfac * zqsice) / zcorqsice, L(0.0));
        } else {
          real zqp1env = (zqx[QV] - za * zqsice) * L(1.0) / FMAX(L(1.0) - za, zepsilon);
          zsupsat = FMAX(((L(1.0) - za) * (zqp1env - zfac * zqsice)) / zcorqsice, L(0.0));
        }
        if (zsupsat > zepsec) {
          if (ztp1 > c->rthomo) {
            zsolqa[QV][QL] = zsolqa[QV][QL] + zsupsat;
            zsolqa[QL][QV] = zsolqa[QL][QV] - zsupsat;
            zqxfg[QL] = zqxfg[QL] + zsupsat;
          } else {
            zsolqa[QV][QI] = zsolqa[QV][QI] + zsupsat;
            zsolqa[QI][QV] = zsolqa[QI][QV] - zsupsat;
            zqxfg[QI] = zqxfg[QI] + zsupsat;
          }
          zsolac = (L(1.0) - za) * zfaci;
        }
        const real psupsat_k = psupsat[IX2(k)];
        if (psupsat_k > zepsec) {
          if (ztp1 > c->rthomo) {
            zsolqa[QL][QL] = zsolqa[QL][QL] + psupsat_k;
            zpsupsatsrce[QL] = psupsat_k;
            zqxfg[QL] = zqxfg[QL] + psupsat_k;
          } else {
            zsolqa[QI][QI] = zsolqa[QI][QI] + psupsat_k;
            zpsupsatsrce[QI] = psupsat_k;
            zqxfg[QI] = zqxfg[QI] + psupsat_k;
          }
          zsolac = (L(1.0) - za) * zfaci;
        }

        /* 3.2 detrainment from convection (:967-987) */
        if (k < klev - 1) {
          plude_k = plude_k * zdtgdp;
          const real plu_kp1 = plu[IX2(k + 1)];
          if (plu_kp1 > zepsec && plude_k > c->rlmin) {
            zsolac = zsolac + plude_k / plu_kp1;
            const real zalfaw = zfoealfa;
            zconvsrce[QL] = zalfaw * plude_k;
            zconvsrce[QI] = (L(1.0) - zalfaw) * plude_k;
            zsolqa[QL][QL] = zsolqa[QL][QL] + zconvsrce[QL];
            zsolqa[QI][QI] = zsolqa[QI][QI] + zconvsrce[QI];
          } else {
            plude_k = L(0.0);
          }
          zsolqa[QS][QS] = zsolqa[QS][QS] + psnde[IX2(k)] * zdtgdp;
        }

        /* 3.3 subsidence source from layer above + evaporation (:1002-1058) */
        if (k > ncldtop0) {
          const real zmf = FMAX(L(0.0), (pmfu[IX2(k)] + pmfd[IX2(k)]) * zdtgdp);
          real zacust = zmf * zanewm1;
          real zlcust[NCLV] = {0};
          for (int m = 0; m < NCLV; m++) {
            if (!llfall[m] && IPHASE[m] > 0) {
              zlcust[m] = zmf * zqxnm1[m];
              zconvsrce[m] = zconvsrce[m] + zlcust[m];
            }
          }
          const real zdtdp = ((zrdcp * L(0.5)) * (t_prev + ztp1)) / paph[IX2(k)];
          const real zdtforc = zdtdp * (pap_k - pap_prev);
          const real zdqs = (zanewm1 * zdtforc) * zdqsmixdt;
          for (int m = 0; m < NCLV; m++) {
            if (!llfall[m] && IPHASE[m] > 0) {
              real zlfinal = FMAX(L(0.0), zlcust[m] - zdqs);
              real zevap = FMIN(zlcust[m] - zlfinal, zevaplimmix);
              zlfinal = zlcust[m] - zevap;
              zlfinalsum = zlfinalsum + zlfinal;
              zsolqa[m][m] = zsolqa[m][m] + zlcust[m];
              zsolqa[m][QV] = zsolqa[m][QV] + zevap;
              zsolqa[QV][m] = zsolqa[QV][m] - zevap;
            }
          }
          if (zlfinalsum < zepsec) zacust = L(0.0);
          zsolac = zsolac + zacust;
        }

        /* subsidence sink of cloud to the layer below (:1064-1075) */
        if (k < klev - 1) {
          const real zmfdn = FMAX(L(0.0), (pmfu[IX2(k + 1)] + pmfd[IX2(k + 1)]) * zdtgdp);
          zsolab = zsolab + zmfdn;
          zsolqb[QL][QL] = zsolqb[QL][QL] + zmfdn;
          zsolqb[QI][QI] = zsolqb[QI][QI] + zmfdn;
          zconvsink[QL] = zmfdn;
          zconvsink[QI] = zmfdn;
        }

        /* 3.4 erosion of clouds by turbulent mixing (:1087-1118) */
        real zldifdt = c->rcldiff * c->ptsphy;
        if (ktype[jl] > 0 && plude_k > zepsec) zldifdt = c->rcldiff_convi * zldifdt;
        if (zli > zepsec) {
          real ze = zldifdt * FMAX(zqsmix - zqx[QV], L(0.0));
          real zleros = za * ze;
          zleros = FMIN(zleros, zevaplimmix);
          zleros = FMIN(zleros, zli);
          real zaeros = zleros / zlicld;
          zsolac = zsolac - zaeros;
          zsolqa[QL][QV] = zsolqa[QL][QV] + zliqfrac * zleros;
          zsolqa[QV][QL] = zsolqa[QV][QL] - zliqfrac * zleros;
          zsolqa[QI][QV] = zsolqa[QI][QV] + zicefrac * zleros;
          zsolqa[QV][QI] = zsolqa[QV][QI] - zicefrac * zleros;
        }

        /* 3.4 condensation/evaporation due to dqsat/dt (:1137-1182) */
        real zdqs;
        {
          const real zdtdp = (zrdcp * ztp1) / pap_k;
          const real zdpmxdt = zdp * zqtmst;
          real zmfdn = L(0.0);
          if (k < klev - 1) zmfdn = pmfu[IX2(k + 1)] + pmfd[IX2(k + 1)];
          real zwtot = pvervel[IX2(k)] + (L(0.5) * c->rg) * (pmfu[IX2(k)] + pmfd[IX2(k)] + zmfdn);
          zwtot = FMIN(zdpmxdt, FMAX(-zdpmxdt, zwtot));
          const real zzzdt = phrsw[IX2(k)] + phrlw[IX2(k)];
          const real zdtdiab = FMIN(zdpmxdt * zdtdp, FMAX(-zdpmxdt * zdtdp, zzzdt)) * c->ptsphy + c->ralfdcp * zldefr;
          const real zdtforc = (zdtdp * zwtot) * c->ptsphy + zdtdiab;
          const real zqold = zqsmix;
          real tt = ztp1 + zdtforc;
          tt = FMAX(tt, L(160.0));
          real qsm = zqsmix;
          const real zqp = L(1.0) / pap_k;
          for (int it = 0; it < 2; it++) {         /* two Newton steps (:1162-1175) */
            real zqsat = foeewm(c, tt) * zqp;
            zqsat = FMIN(L(0.5), zqsat);
            real zcor2 = L(1.0) / (L(1.0) - c->retv * zqsat);
            zqsat = zqsat * zcor2;
            const real zcond = (qsm - zqsat) * L(1.0) / (L(1.0) + (zqsat * zcor2) * foedem_term(c, tt, foealfa(c, tt)));
            const real a2 = foealfa(c, tt);
            tt = tt + (a2 * c->ralvdcp + (L(1.0) - a2) * c->ralsdcp) * zcond;
            qsm = qsm - zcond;
          }
          zdqs = qsm - zqold;
        }

        /* 3.4a evaporation of clouds (:1189-1207) */
        if (zdqs > L(0.0)) {
          real zlevap = za * FMIN(zdqs, zlicld);
          zlevap = FMIN(zlevap, zevaplimmix);
          zlevap = FMIN(zlevap, FMAX(zqsmix - zqx[QV], L(0.0)));
          zsolqa[QL][QV] = zsolqa[QL][QV] + zliqfrac * zlevap;
          zsolqa[QV][QL] = zsolqa[QV][QL] - zliqfrac * zlevap;
          zsolqa[QI][QV] = zsolqa[QI][QV] + zicefrac * zlevap;
          zsolqa[QV][QI] = zsolqa[QV][QI] - zicefrac * zlevap;
        }

        /* 3.4b(1) increase of cloud water in existing clouds (:1213-1250) */
        if (zdqs <= -c->rlmin && za > zepsec) {
          real zlcond1 = FMAX(-zdqs, L(0.0));
          real zcdmax;
          if (za > L(0.99)) {
            real zcor3 = L(1.0) / (L(1.0) - c->retv * zqsmix);
            zcdmax = (zqx[QV] - zqsmix) * L(1.0) / (L(1.0) + (zcor3 * zqsmix) * foedem_term(c, ztp1, foealfa(c, ztp1)));
          } else {
            zcdmax = (zqx[QV] - za * zqsmix) / za;
          }
          zlcond1 = FMAX(FMIN(zlcond1, zcdmax), L(0.0));
          zlcond1 = za * zlcond1;
          if (zlcond1 < c->rlmin) zlcond1 = L(0.0);
          if (ztp1 > c->rthomo) {
            zsolqa[QV][QL] = zsolqa[QV][QL] + zlcond1;
            zsolqa[QL][QV] = zsolqa[QL][QV] - zlcond1;
            zqxfg[QL] = zqxfg[QL] + zlcond1;
          } else {
            zsolqa[QV][QI] = zsolqa[QV][QI] + zlcond1;
            zsolqa[QI][QV] = zsolqa[QI][QV] - zlcond1;
            zqxfg[QI] = zqxfg[QI] + zlcond1;
          }
        }

        /* 3.4b(2) generation of new clouds (:1253-1363) */
        if (zdqs <= -c->rlmin && za < L(1.0) - zepsec) {
          real zrhc = c->ramid;
          const real zsigk = pap_k / paph_sfc;
          if (zsigk > L(0.8)) {
            real s = (zsigk - L(0.8)) / L(0.2);
            zrhc = c->ramid + (L(1.0) - c->ramid) * (s * s);
          }
          real zqe = L(0.0);
          if (c->nssopt == 0) {
            zqe = (zqx[QV] - za * zqsice) * L(1.0) / FMAX(zepsec, L(1.0) - za);
            zqe = FMAX(L(0.0), zqe);
          } else if (c->nssopt == 1) {
            zqe = (zqx[QV] - za * zqsice) * L(1.0) / FMAX(zepsec, L(1.0) - za);
            zqe = FMAX(L(0.0), zqe);
          } else if (c->nssopt == 2) {
            zqe = zqx[QV];
          } else if (c->nssopt == 3) {
            zqe = zqx[QV] + zli;
          }
          real zfacn;
          if (c->nssopt == 0 || ztp1 >= c->rtt) zfacn = L(1.0);
          else zfacn = zfokoop;
          if (zqe >= zqsice * zfacn * zrhc && zqe < zqsice * zfacn) {
            real zacond = -((L(1.0) - za) * zfacn) * zdqs * L(1.0) / FMAX(L(2.0) * (zfacn * zqsice - zqe), zepsec);
            zacond = FMIN(zacond, L(1.0) - za);
            real zlcond2 = -(zfacn * zdqs) * L(0.5) * zacond;
            const real zzdl = (L(2.0) * (zfacn * zqsice - zqe)) * L(1.0) / FMAX(zepsec, L(1.0) - za);
            if (zdqs * zfacn < -zzdl) {
              real zlcondlim = ((za - L(1.0)) * zfacn) * zdqs - zfacn * zqsice + zqx[QV];
              zlcond2 = FMIN(zlcond2, zlcondlim);
            }
            zlcond2 = FMAX(zlcond2, L(0.0));
            if (L(1.0) - za < zepsec || zlcond2 < c->rlmin) {
              zlcond2 = L(0.0);
              zacond = L(0.0);
            }
            if (zlcond2 == L(0.0)) zacond = L(0.0);
            zsolac = zsolac + zacond;
            if (ztp1 > c->rthomo) {
              zsolqa[QV][QL] = zsolqa[QV][QL] + zlcond2;
              zsolqa[QL][QV] = zsolqa[QL][QV] - zlcond2;
              zqxfg[QL] = zqxfg[QL] + zlcond2;
            } else {
              zsolqa[QV][QI] = zsolqa[QV][QI] + zlcond2;
              zsolqa[QI][QV] = zsolqa[QI][QV] - zlcond2;
              zqxfg[QI] = zqxfg[QI] + zlcond2;
            }
          }
        }

        /* 3.7 growth of ice by vapour deposition, Rotstayn (:1382-1447) */
        if (za >= c->rcldtopcf && a_prev < c->rcldtopcf) {
          zcldtopdist = L(0.0);
        } else {
          zcldtopdist = zcldtopdist + zdp / (zrho * c->rg);
        }
        if (zqxfg[QL] > c->rlmin && ztp1 < c->rtt) {
          const real zvpice = ((c->r2es * e_ice) * c->rv) / c->rd;
          const real zvpliq = zvpice * zfokoop;
          const real zicenuclei = L(1000.0) * EXP((L(12.96) * (zvpliq - zvpice)) / zvpliq - L(0.639));
          const real zadd = (c->rlstt * (c->rlstt / (c->rv * ztp1) - L(1.0))) / (L(0.024) * ztp1);
          const real zbdd = ((c->rv * ztp1) * pap_k) / (L(2.21) * zvpice);
          const real zcvds = ((L(7.8) * POW(zicenuclei / zrho, L(0.666))) * (zvpliq - zvpice)) / ((L(8.87) * (zadd + zbdd)) * zvpice);
          const real zice0 = FMAX(zicecld, (zicenuclei * c->riceinit) / zrho);
          const real zinew = POW((L(0.666) * zcvds) * c->ptsphy + POW(zice0, L(0.666)), L(1.5));
          real zdepos = FMAX(za * (zinew - zice0), L(0.0));
          zdepos = FMIN(zdepos, zqxfg[QL]);
          const real zinfactor = FMIN(zicenuclei / L(15000.0), L(1.0));
          zdepos = zdepos * FMIN(zinfactor + (L(1.0) - zinfactor) * (c->rdepliqrefrate + zcldtopdist / c->rdepliqrefdepth), L(1.0));
          zsolqa[QL][QI] = zsolqa[QL][QI] + zdepos;
          zsolqa[QI][QL] = zsolqa[QI][QL] - zdepos;
          zqxfg[QI] = zqxfg[QI] + zdepos;
          zqxfg[QL] = zqxfg[QL] - zdepos;
        }

        /* 4. revise in-cloud condensate (:1528-1533) */
        ztmpa = L(1.0) * L(1.0) / FMAX(za, zepsec);
        zliqcld = zqxfg[QL] * ztmpa;
        zicecld = zqxfg[QI] * ztmpa;
        zlicld = zliqcld + zicecld;

        /* 4.2 sedimentation (:1541-1576) */
        for (int m = 0; m < NCLV; m++) {
          if (llfall[m] || m == QI) {
            if (k > ncldtop0) {
              zfallsrce[m] = zpfplsx[m] * zdtgdp;
              zsolqa[m][m] = zsolqa[m][m] + zfallsrce[m];
              zqxfg[m] = zqxfg[m] + zfallsrce[m];
              zqpretot = zqpretot + zqxfg[m];
            }
            if (c->laericesed && m == QI) zvqx[QI] = L(0.002) * pre_ice[IX2(k)];   /* pow(x,1.0) == x */
            const real zfall = zvqx[m] * zrho;
            zfallsink[m] = zdtgdp * zfall;
          }
        }

        /* precip cover overlap, MAX-RAN (:1594-1611) */
        real zcovpclr, zraincld, zsnowcld;
        if (zqpretot > zepsec) {
          zcovptot = L(1.0) - (L(1.0) - zcovptot) * (L(1.0) - FMAX(za, a_prev)) * L(1.0) / (L(1.0) - FMIN(a_prev, L(1.0) - L(1.0e-6)));
          zcovptot = FMAX(zcovptot, c->rcovpmin);
          zcovpclr = FMAX(L(0.0), zcovptot - za);
          zraincld = zqxfg[QR] / zcovptot;
          zsnowcld = zqxfg[QS] / zcovptot;
          zcovpmax = FMAX(zcovptot, zcovpmax);
        } else {
          zraincld = L(0.0);
          zsnowcld = L(0.0);
          zcovptot = L(0.0);
          zcovpclr = L(0.0);
          zcovpmax = L(0.0);
        }

        /* 4.3a autoconversion to snow (:1616-1637) */
        if (ztp1 <= c->rtt) {
          if (zicecld > zepsec) {
            real zzco = (c->ptsphy * c->rsnowlin1) * EXP(c->rsnowlin2 * (ztp1 - c->rtt));
            real zlcrit;
            if (c->laericeauto) {
              zlcrit = picrit_aer[IX2(k)];
              zzco = zzco * POW(c->rnice / pnice[IX2(k)], L(0.333));
            } else {
              zlcrit = c->rlcritsnow;
            }
            const real r = zicecld / zlcrit;
            const real zsnowaut = zzco * (L(1.0) - EXP(-(r * r)));
            zsolqb[QI][QS] = zsolqb[QI][QS] + zsnowaut;
          }
        }
        /* 4.3b warm-rain autoconversion, Khairoutdinov and Kogan (:1644-1761) */
        if (zliqcld > zepsec) {
          real zconst, zlcrit, zrainaut, zrainacc;
          if (plsm[jl] > L(0.5)) {
            zconst = c->rcl_kk_cloud_num_land;
            zlcrit = c->rclcrit_land;
          } else {
            zconst = c->rcl_kk_cloud_num_sea;
            zlcrit = c->rclcrit_sea;
          }
          if (zliqcld > zlcrit) {
            zrainaut = ((((L(1.5) * za) * c->ptsphy) * c->rcl_kkaau) * POW(zliqcld, c->rcl_kkbauq)) * POW(zconst, c->rcl_kkbaun);
            zrainaut = FMIN(zrainaut, zqxfg[QL]);
            if (zrainaut < zepsec) zrainaut = L(0.0);
            zrainacc = (((L(2.0) * za) * c->ptsphy) * c->rcl_kkaac) * POW(zliqcld * zraincld, c->rcl_kkbac);
            zrainacc = FMIN(zrainacc, zqxfg[QL]);
            if (zrainacc < zepsec) zrainacc = L(0.0);
          } else {
            zrainaut = L(0.0);
            zrainacc = L(0.0);
          }
          if (ztp1 <= c->rtt) {
            zsolqa[QL][QS] = zsolqa[QL][QS] + zrainaut;
            zsolqa[QL][QS] = zsolqa[QL][QS] + zrainacc;
            zsolqa[QS][QL] = zsolqa[QS][QL] - zrainaut;
            zsolqa[QS][QL] = zsolqa[QS][QL] - zrainacc;
          } else {
            zsolqa[QL][QR] = zsolqa[QL][QR] + zrainaut;
            zsolqa[QL][QR] = zsolqa[QL][QR] + zrainacc;
            zsolqa[QR][QL] = zsolqa[QR][QL] - zrainaut;
            zsolqa[QR][QL] = zsolqa[QR][QL] - zrainacc;
          }
        }

        /* riming of snow by cloud water (:1768-1808) */
        if (ztp1 <= c->rtt && zliqcld > zepsec) {
          const real zfallcorr = POW(c->rdensref / zrho, L(0.4));
          if (zcovptot > L(0.01) && zsnowcld > zepsec) {
            real zsnowrime = ((((L(0.3) * zcovptot) * c->ptsphy) * c->rcl_const7s) * zfallcorr) * POW((zrho * zsnowcld) * c->rcl_const1s, c->rcl_const8s);
            zsnowrime = FMIN(zsnowrime, L(1.0));
            zsolqb[QL][QS] = zsolqb[QL][QS] + zsnowrime;
          }
        }

        /* 4.4a melting of snow and ice (:1817-1859) */
        const real zicetot = zqxfg[QI] + zqxfg[QS];
        real zmeltmax = L(0.0);
        if (zicetot > zepsec && ztp1 > c->rtt) {
          const real zsubsat = FMAX(zqsice - zqx[QV], L(0.0));
          const real ztdmtw0 = ztp1 - c->rtt - zsubsat * (ztw1 + ztw2 * (pap_k - ztw3) - ztw4 * (ztp1 - ztw5));
          const real zcons1 = FABS((c->ptsphy * (L(1.0) + L(0.5) * ztdmtw0)) / c->rtaumel);
          zmeltmax = FMAX((ztdmtw0 * zcons1) * zrldcp, L(0.0));
        }
        for (int m = 0; m < NCLV; m++) {
          if (IPHASE[m] == 2) {
            const int n = IMELT[m];
            if (zicetot > zepsec && zmeltmax > zepsec) {
              const real zalfa = zqxfg[m] / zicetot;
              const real zmelt = FMIN(zqxfg[m], zalfa * zmeltmax);
              zqxfg[m] = zqxfg[m] - zmelt;
              zqxfg[n] = zqxfg[n] + zmelt;
              zsolqa[m][n] = zsolqa[m][n] + zmelt;
              zsolqa[n][m] = zsolqa[n][m] - zmelt;
            }
          }
        }

        /* 4.4b freezing of rain (:1864-1908) */
        if (zqx[QR] > zepsec) {
          if (ztp1 <= c->rtt && t_prev > c->rtt) {
            zqpretot = FMAX(zqx[QS] + zqx[QR], zepsec);
            rainfrac = zqx[QR] / zqpretot;
          }
          if (ztp1 < c->rtt) {
            real zfrzmax;
            if (rainfrac > L(0.8)) {
              const real zlambda = POW(c->rcl_fac1 / (zrho * zqx[QR]), c->rcl_fac2);
              const real ztemp = c->rcl_fzrab * (ztp1 - c->rtt);
              const real zfrz = ((c->ptsphy * (c->rcl_const5r / zrho)) * (EXP(ztemp) - L(1.0))) * POW(zlambda, c->rcl_const6r);
              zfrzmax = FMAX(zfrz, L(0.0));
            } else {
              const real zcons1 = FABS((c->ptsphy * (L(1.0) + L(0.5) * (c->rtt - ztp1))) / c->rtaumel);
              zfrzmax = FMAX(((c->rtt - ztp1) * zcons1) * zrldcp, L(0.0));
            }
            if (zfrzmax > zepsec) {
              const real zfrz = FMIN(zqx[QR], zfrzmax);
              zsolqa[QR][QS] = zsolqa[QR][QS] + zfrz;
              zsolqa[QS][QR] = zsolqa[QS][QR] - zfrz;
            }
          }
        }

        /* 4.4c freezing of liquid (:1913-1928) */
        {
          const real zfrzmax = FMAX((c->rthomo - ztp1) * zrldcp, L(0.0));
          if (zfrzmax > zepsec && zqxfg[QL] > zepsec) {
            const real zfrz = FMIN(zqxfg[QL], zfrzmax);
            zsolqa[QL][QI] = zsolqa[QL][QI] + zfrz;
            zsolqa[QI][QL] = zsolqa[QI][QL] - zfrz;
          }
        }

        /* 4.5 evaporation of rain, Abel and Boutle (:1982-2040) */
        {
          real zzrh = c->rprecrhmax + ((L(1.0) - c->rprecrhmax) * zcovpmax) * L(1.0) / FMAX(zepsec, L(1.0) - za);
          zzrh = FMIN(FMAX(zzrh, c->rprecrhmax), L(1.0));
          zzrh = FMIN(L(0.8), zzrh);
          const real zqe = FMAX(L(0.0), FMIN(zqx[QV], zqsliq));
          const int llo1 = zcovpclr > zepsec && zqxfg[QR] > zepsec && zqe < zzrh * zqsliq;
          if (llo1) {
            const real zpreclr = zqxfg[QR] / zcovptot;
            const real zfallcorr = POW(c->rdensref / zrho, L(0.4));
            const real zesatliq = (c->rv / c->rd) * (c->r2es * e_liq);
            const real zlambda = POW(c->rcl_fac1 / (zrho * zpreclr), c->rcl_fac2);
            const real zevap_denom = c->rcl_cdenom1 * zesatliq - c->rcl_cdenom2 * ztp1 * zesatliq + (c->rcl_cdenom3 * POW(ztp1, L(3.0))) * pap_k;
            const real zcorr2 = (POW(ztp1 / L(273.0), L(1.5)) * L(393.0)) / (ztp1 + L(120.0));
            const real zsubsat = FMAX(zzrh * zqsliq - zqe, L(0.0));
            const real zbeta = ((((L(0.5) / zqsliq) * (ztp1 * ztp1)) * zesatliq) * c->rcl_const1r) * (zcorr2 / zevap_denom) *
                               (L(0.78) / POW(zlambda, c->rcl_const4r) + (c->rcl_const2r * SQRT(zrho * zfallcorr)) / (SQRT(zcorr2) * POW(zlambda, c->rcl_const3r)));
            const real zdenom = L(1.0) + zbeta * c->ptsphy;
            const real zdpevap = (((zcovpclr * zbeta) * c->ptsphy) * zsubsat) / zdenom;
            const real zevap = FMIN(zdpevap, zqxfg[QR]);
            zsolqa[QR][QV] = zsolqa[QR][QV] + zevap;
            zsolqa[QV][QR] = zsolqa[QV][QR] - zevap;
            zcovptot = FMAX(c->rcovpmin, zcovptot - FMAX(L(0.0), ((zcovptot - za) * zevap) / zqxfg[QR]));
            zqxfg[QR] = zqxfg[QR] - zevap;
          }
        }

        /* 4.5 evaporation of snow, Sundqvist (:2048-2087) */
        {
          real zzrh = c->rprecrhmax + ((L(1.0) - c->rprecrhmax) * zcovpmax) * L(1.0) / FMAX(zepsec, L(1.0) - za);
          zzrh = FMIN(FMAX(zzrh, c->rprecrhmax), L(1.0));
          real zqe = (zqx[QV] - za * zqsice) * L(1.0) / FMAX(zepsec, L(1.0) - za);
          zqe = FMAX(L(0.0), FMIN(zqe, zqsice));
          const int llo1 = zcovpclr > zepsec && zqxfg[QS] > zepsec && zqe < zzrh * zqsice;
          if (llo1) {
            const real x = zcovptot * zdtgdp;
            const real zpreclr = (zqxfg[QS] * zcovpclr) * L(1.0) / COPYSIGN(FMAX(FABS(x), zepsilon), x);
            const real zbeta1 = ((SQRT(pap_k / paph_sfc) / c->rvrfactor) * zpreclr) * L(1.0) / FMAX(zcovpclr, zepsec);
            const real zbeta = (c->rg * c->rpecons) * POW(zbeta1, L(0.5777));
            const real zdenom = L(1.0) + (zbeta * c->ptsphy) * zcorqsice;
            const real zdpr = ((((zcovpclr * zbeta) * (zqsice - zqe)) / zdenom) * zdp) * zrg_r;
            const real zdpevap = zdpr * zdtgdp;
            const real zevap = FMIN(zdpevap, zqxfg[QS]);
            zsolqa[QS][QV] = zsolqa[QS][QV] + zevap;
            zsolqa[QV][QS] = zsolqa[QV][QS] - zevap;
            zcovptot = FMAX(c->rcovpmin, zcovptot - FMAX(L(0.0), ((zcovptot - za) * zevap) / zqxfg[QS]));
            zqxfg[QS] = zqxfg[QS] - zevap;
          }
        }

        /* evaporate small precipitation amounts (:2144-2158) */
        for (int m = 0; m < NCLV; m++) {
          if (llfall[m]) {
            if (zqxfg[m] < c->rlmin) {
              zsolqa[m][QV] = zsolqa[m][QV] + zqxfg[m];
              zsolqa[QV][m] = zsolqa[QV][m] - zqxfg[m];
            }
          }
        }

        /* 5.1 solver for cloud cover (:2168-2180) */
        real zanew = (za + zsolac) / (L(1.0) + zsolab);
        zanew = FMIN(zanew, L(1.0));
        if (zanew < c->ramin) zanew = L(0.0);
        const real zda = zanew - zaorig;
        zanewm1 = zanew;

        /* 5.2 truncate explicit sinks (:2190-2286); the first zratio pass of
           :2220-2227 is overwritten before use and is not restated */
        for (int m = 0; m < NCLV; m++) {
          real psum = L(0.0);
          for (int n = 0; n < NCLV; n++) psum = psum + zsolqa[n][m];
          const real zsinksum = L(0.0) - psum;
          const real zmm = FMAX(zqx[m], zepsec);
          const real zrr = FMAX(zsinksum, zmm);
          const real zzratio = zmm / zrr;
          for (int n = 0; n < NCLV; n++) {
            if (zsolqa[n][m] < L(0.0)) {
              zsolqa[n][m] = zsolqa[n][m] * zzratio;
              zsolqa[m][n] = zsolqa[m][n] * zzratio;
            }
          }
        }

        /* 5.2.2 implicit solver: LHS, RHS, unpivoted LU (:2294-2397) */
        real zqlhs[NCLV][NCLV];
        for (int m = 0; m < NCLV; m++) {
          for (int n = 0; n < NCLV; n++) {
            if (n == m) {
              zqlhs[m][n] = L(1.0) + zfallsink[m];
              for (int o = 0; o < NCLV; o++) zqlhs[m][n] = zqlhs[m][n] + zsolqb[n][o];
            } else {
              zqlhs[m][n] = -zsolqb[m][n];
            }
          }
        }
        for (int m = 0; m < NCLV; m++) {
          real zexplicit = L(0.0);
          for (int n = 0; n < NCLV; n++) zexplicit = zexplicit + zsolqa[n][m];
          zqxn[m] = zqx[m] + zexplicit;
        }
        for (int n = 0; n < 4; n++) {
          for (int m = n + 1; m < NCLV; m++) {
            zqlhs[n][m] = zqlhs[n][m] / zqlhs[n][n];
            for (int ik = n + 1; ik < NCLV; ik++) zqlhs[ik][m] = zqlhs[ik][m] - zqlhs[n][m] * zqlhs[ik][n];
          }
        }
        for (int n = 1; n < NCLV; n++)
          for (int m = 0; m < n; m++) zqxn[n] = zqxn[n] - zqlhs[m][n] * zqxn[m];
        zqxn[QV] = zqxn[QV] / zqlhs[QV][QV];
        for (int n = 3; n >= 0; n--) {
          for (int m = n + 1; m < NCLV; m++) zqxn[n] = zqxn[n] - zqlhs[m][n] * zqxn[m];
          zqxn[n] = zqxn[n] / zqlhs[n][n];
        }
        /* no small values (:2402-2412) */
        for (int n = 0; n < 4; n++) {
          if (zqxn[n] < zepsec) {
            zqxn[QV] = zqxn[QV] + zqxn[n];
            zqxn[n] = L(0.0);
          }
        }
        for (int m = 0; m < NCLV; m++) zqxnm1[m] = zqxn[m];

        /* 5.3 fluxes to the next level (:2430-2448) */
        for (int m = 0; m < NCLV; m++) zpfplsx[m] = (zfallsink[m] * zqxn[m]) * zrdtgdp;
        zqpretot = zpfplsx[QS] + zpfplsx[QR];
        if (zqpretot < zepsec) zcovptot = L(0.0);

        /* 6. tendencies (:2456-2506) */
        for (int m = 0; m < 4; m++) {
          const real zfluxq = zpsupsatsrce[m] + zconvsrce[m] + zfallsrce[m] - (zfallsink[m] + zconvsink[m]) * zqxn[m];
          if (IPHASE[m] == 1) ttend = ttend + (c->ralvdcp * (zqxn[m] - zqx[m] - zfluxq)) * zqtmst;
          if (IPHASE[m] == 2) ttend = ttend + (c->ralsdcp * (zqxn[m] - zqx[m] - zfluxq)) * zqtmst;
          ctend[m] = ctend[m] + (zqxn[m] - zqx0[m]) * zqtmst;
        }
        qtend = qtend + (zqxn[QV] - zqx[QV]) * zqtmst;
        atend = atend + zda * zqtmst;
        zcovptot_out = zcovptot;
      } else {
        for (int m = 0; m < NCLV; m++) zqxn[m] = L(0.0);   /* zqxn2d stays zero above NCLDTOP */
      }

      /* ---- outputs of level k ---- */
      tlt[IX2(k)] = ttend;
      tlq[IX2(k)] = qtend;
      tla[IX2(k)] = atend;
      for (int m = 0; m < 4; m++) tlcld[IX3(m, k)] = ctend[m];
      tlcld[IX3(QV, k)] = L(0.0);
      pcovptot[IX2(k)] = zcovptot_out;
      plude[IX2(k)] = plude_k;

      /* ===== 8. flux diagnostics, fused (cloudsc_c.c:2521-2582) ===== */
      {
        const real zgdph_r = -zrg_r * (paph[IX2(k + 1)] - paph[IX2(k)]) * zqtmst;
        const real zalfaw = zfoealfa;
        const real lf = fl_lf, fi = fl_if, lng = fl_lng, nng = fl_nng;
        fl_lf = lf + (zqxn[QL] - zqx0[QL] + pvfl[IX2(k)] * c->ptsphy - zalfaw * plude_k) * zgdph_r;
        fl_lng = lng + zlneg[QL] * zgdph_r;
        fl_ltur = fl_ltur + (pvfl[IX2(k)] * c->ptsphy) * zgdph_r;
        const real rf = lf + (zqxn[QR] - zqx0[QR]) * zgdph_r;
        const real rng = lng + zlneg[QR] * zgdph_r;
        fl_if = fi + (zqxn[QI] - zqx0[QI] + pvfi[IX2(k)] * c->ptsphy - (L(1.0) - zalfaw) * plude_k) * zgdph_r;
        fl_nng = nng + zlneg[QI] * zgdph_r;
        fl_itur = fl_itur + (pvfi[IX2(k)] * c->ptsphy) * zgdph_r;
        const real sf = fi + (zqxn[QS] - zqx0[QS]) * zgdph_r;
        const real sng = nng + zlneg[QS] * zgdph_r;
        pfsqlf[IX2(k + 1)] = fl_lf;   pfsqif[IX2(k + 1)] = fl_if;
        pfcqlng[IX2(k + 1)] = fl_lng; pfcqnng[IX2(k + 1)] = fl_nng;
        pfsqltur[IX2(k + 1)] = fl_ltur; pfsqitur[IX2(k + 1)] = fl_itur;
        pfsqrf[IX2(k + 1)] = rf; pfcqrng[IX2(k + 1)] = rng;
        pfsqsf[IX2(k + 1)] = sf; pfcqsng[IX2(k + 1)] = sng;
        const real plsl = zpfplsx[QR] + zpfplsx[QL];
        const real plsn = zpfplsx[QS] + zpfplsx[QI];
        pfplsl[IX2(k + 1)] = plsl;
        pfplsn[IX2(k + 1)] = plsn;
        pfhpsl[IX2(k + 1)] = -c->rlvtt * plsl;
        pfhpsn[IX2(k + 1)] = -c->rlstt * plsn;
      }

      t_prev = ztp1;
      a_prev = za;
      pap_prev = pap[IX2(k)];
    }
    prainfrac[jl] = rainfrac;
  }
  return 0;
}

#ifndef ORACLE_SP
unsigned cloudsc_oracle_libm_nudge_seed = 0;
void cloudsc_oracle_set_libm_nudge(unsigned seed) { cloudsc_oracle_libm_nudge_seed = seed; }

/* The driver entry is compiled once (in the fp64 object). */
int cloudsc_oracle_run(int nthreads, int precision, int ngptot, int nproma, int klev,
                       const cloudsc_params_t *p, const cloudsc_fields_t *f, double *seconds)
{
  if (!p || !f || ngptot <= 0 || nproma <= 0 || klev <= 1) return CLOUDSC_EINVAL;
  if (precision != CLOUDSC_FP64 && precision != CLOUDSC_FP32) return CLOUDSC_EINVAL;
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  const size_t es = precision == CLOUDSC_FP64 ? sizeof(double) : sizeof(float);
  const size_t s2 = (size_t)klev * nproma, s2h = (size_t)(klev + 1) * nproma, s3 = (size_t)NCLV * klev * nproma;
  if (nthreads <= 0) nthreads = omp_get_max_threads();
  double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(nthreads) schedule(runtime)
  for (int b = 0; b < nblocks; b++) {
    const int bsize = (ngptot - b * nproma) < nproma ? (ngptot - b * nproma) : nproma;
    cloudsc_fields_t g;
#define B2(x) g.x = f->x ? (const char *)f->x + b * s2 * es : NULL
#define B2H(x) g.x = (char *)f->x + b * s2h * es
#define B3(x) g.x = (const char *)f->x + b * s3 * es
#define B1(x) g.x = (char *)f->x + (size_t)b * nproma * es
    B2(pt); B2(pq); B2(tendency_tmp_t); B2(tendency_tmp_q); B2(tendency_tmp_a); B3(tendency_tmp_cld);
    B2(pvfl); B2(pvfi); B2(phrsw); B2(phrlw); B2(pvervel); B2(pap); g.paph = (const char *)f->paph + b * s2h * es;
    g.plsm = (const char *)f->plsm + (size_t)b * nproma * es; g.ktype = f->ktype + (size_t)b * nproma;
    B2(plu); B2(psnde); B2(pmfu); B2(pmfd); B2(pa); B3(pclv); B2(psupsat);
    B2(plcrit_aer); B2(picrit_aer); B2(pre_ice); B2(pccn); B2(pnice);
    g.plude = (char *)f->plude + b * s2 * es;
    g.tendency_loc_t = (char *)f->tendency_loc_t + b * s2 * es;
    g.tendency_loc_q = (char *)f->tendency_loc_q + b * s2 * es;
    g.tendency_loc_a = (char *)f->tendency_loc_a + b * s2 * es;
    g.tendency_loc_cld = (char *)f->tendency_loc_cld + b * s3 * es;
    g.pcovptot = (char *)f->pcovptot + b * s2 * es;
    B1(prainfrac_toprfz);
    B2H(pfsqlf); B2H(pfsqif); B2H(pfcqnng); B2H(pfcqlng); B2H(pfsqrf); B2H(pfsqsf); B2H(pfcqrng);
    B2H(pfcqsng); B2H(pfsqltur); B2H(pfsqitur); B2H(pfplsl); B2H(pfplsn); B2H(pfhpsl); B2H(pfhpsn);
#undef B2
#undef B2H
#undef B3
#undef B1
    if (precision == CLOUDSC_FP64) cloudsc_oracle_block_dp(p, 1, bsize, nproma, klev, &g);
    else cloudsc_oracle_block_sp(p, 1, bsize, nproma, klev, &g);
  }
  double t1 = omp_get_wtime();
  if (seconds) *seconds = t1 - t0;
  return 0;
}
#endif
