# fp32 FAST: v_sqrt_f32 for sqrt, and known-divisor divisions as one multiply by RN(1/d)
EDITS = [
 ("cloudsc_dev.h", '''template <typename real, typename P>
CLOUDSC_HD real cl_div_known_p(const P& c, typename std::common_type<real>::type n, real d, real rcp_d) {
  return cl_div_p<real>(c, n, Recip<real>{d, rcp_d});
}''', '''template <typename real, typename P>
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
}'''),
 ("cloudsc_dev.h", '''template <typename real, typename P>
CLOUDSC_HD real cl_div_lit_p(const P& c, typename std::common_type<real>::type n, real d) {
  return cl_div_p<real>(c, n, Recip<real>{d, real(1) / d});
}''', '''template <typename real, typename P>
CLOUDSC_HD real cl_div_lit_p(const P& c, typename std::common_type<real>::type n, real d) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LibmFast<P>::value) return n * (real(1) / d);
#endif
  return cl_div_p<real>(c, n, Recip<real>{d, real(1) / d});
}'''),
 ("cloudsc_kcache.h", "(c.rcl_const2r * sqrt(zrho * zfallcorr)), (sqrt(zcorr2) *", "(c.rcl_const2r * cl_sqrt_p<real>(c, zrho * zfallcorr)), (cl_sqrt_p<real>(c, zcorr2) *"),
 ("cloudsc_kcache.h", "cl_div_known_p<real>(c, sqrt(cl_div_p<real>(c, pap_k, cc.paph_sfc))", "cl_div_known_p<real>(c, cl_sqrt_p<real>(c, cl_div_p<real>(c, pap_k, cc.paph_sfc))"),
]
