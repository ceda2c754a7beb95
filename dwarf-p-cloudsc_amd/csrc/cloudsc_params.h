// cloudsc_params.h -- the host-side folding of cloudsc_params_t into the
// kernels' DevParams<real> block (shared by the GPU launch path and the CPU
// variant).  Products and reciprocals the reference evaluates per point are
// computed once here with the SAME single IEEE operation, so results do not
// change (each member of DevParams cites the reference line it replaces).
#pragma once
#include <cstring>

#include "cloudsc_amd.h"
#include "cloudsc_dev.h"

namespace cloudsc {

template <typename real>
inline DevParams<real> fold_params(const cloudsc_params_t& p) {
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
  d.rd_rcp = one / rd;
  d.rtaumel_rcp = one / (real)p.rtaumel;
  d.rdepliqrefdepth_rcp = one / (real)p.rdepliqrefdepth;
  d.rvrfactor_rcp = one / (real)p.rvrfactor;
  d.nssopt = p.nssopt;
  d.ncldtop = p.ncldtop;
  d.laericesed = p.laericesed;
  d.laericeauto = p.laericeauto;
  return d;
}

}  // namespace cloudsc
