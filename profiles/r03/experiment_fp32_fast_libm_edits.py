# experiment: fp32 exp/pow computed in float with the hardware exp2/log2 (v_exp_f32/v_log_f32)
FAST = r'''
__device__ __forceinline__ float cl_expf_fast(float x) {
  const float L2E = 0x1.715476p+0f, L2E_LO = 0x1.4ae0bep-26f;
  const float ph = x * L2E;
  float pl = __builtin_fmaf(x, L2E, -ph);
  pl = __builtin_fmaf(x, L2E_LO, pl);
  const float e = __builtin_rintf(ph);
  const float a = (ph - e) + pl;
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(a), (int)e);
}
__device__ __forceinline__ float cl_powf_fast(float x, float y) {
  const float m = __builtin_amdgcn_frexp_mantf(x);
  const float E = (float)__builtin_amdgcn_frexp_expf(x);
  const float l = __builtin_amdgcn_logf(m);
  const float a = y * E, a_lo = __builtin_fmaf(y, E, -a);
  const float b = y * l, b_lo = __builtin_fmaf(y, l, -b);
  const float hi = a + b;
  const float bb = hi - a;
  const float lo = ((a - (hi - bb)) + (b - bb)) + (a_lo + b_lo);
  const float k = __builtin_rintf(hi);
  const float f = (hi - k) + lo;
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f), (int)k);
}
__device__ __forceinline__ float cl_powr(float x, float y) {
  const uint32_t ix = __builtin_bit_cast(uint32_t, x), iy = __builtin_bit_cast(uint32_t, y);
  if (__builtin_expect(ix - 0x00800000u >= 0x7f800000u - 0x00800000u || 2 * iy - 1 >= 2u * 0x7f800000u - 1, 0))
    return cl_powf_cold(x, y);
  return cl_powf_fast(x, y);
}'''
EDITS = [
    ("cloudsc_dev.h", '''__device__ __forceinline__ float cl_powr(float x, float y) {
  return cloudsc_libm::powf_split(x, y, LdsLibmTabsF{}, DevLibmCold{});
}''', FAST),
    ("cloudsc_dev.h", '''__device__ __forceinline__ float cl_exp_impl(float x) { return cloudsc_libm::expf_split(x, LdsLibmTabsF{}, DevLibmCold{}); }''',
     '''__device__ __forceinline__ float cl_exp_impl(float x) {
  if (__builtin_expect(!(__builtin_fabsf(x) < 88.0f), 0)) return cl_expf_cold(x);
  return cl_expf_fast(x);
}'''),
]
