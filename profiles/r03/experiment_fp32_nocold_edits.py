# fp32 FAST exp/pow without the out-of-line cold calls: branch-free special cases
EDITS = [
    ("cloudsc_dev.h", '''__device__ __forceinline__ float cl_expf_fast(float x) {
  if (__builtin_expect(!(__builtin_fabsf(x) < 88.0f), 0)) return cl_expf_cold(x);
  const float kL2e''', '''__device__ __forceinline__ float cl_expf_fast(float x0) {
  // |x| clamped: e^89 overflows to +inf and e^-104 underflows to 0 through ldexp as they should
  const float x = __builtin_fminf(__builtin_fmaxf(x0, -104.0f), 89.0f);
  const float kL2e'''),
    ("cloudsc_dev.h", '''  const float f = (ph - e) + pl;                                    // |f| <= 1/2 + tiny
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f), (int)e);''', '''  const float f = (ph - e) + pl;                                    // |f| <= 1/2 + tiny
  const float r = __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f), (int)e);
  return x0 != x0 ? x0 : r;                                         // NaN stays NaN'''),
    ("cloudsc_dev.h", '''  // hot range: x a positive normal number, y finite and non-zero (else the complete function)
  if (__builtin_expect(ix - 0x00800000u >= 0x7f800000u - 0x00800000u || 2 * iy - 1 >= 2u * 0x7f800000u - 1, 0))
    return cl_powf_cold(x, y);''', '''  (void)ix; (void)iy;'''),
    ("cloudsc_dev.h", '''  if (__builtin_expect(!(__builtin_fabsf(hi) < 126.0f), 0)) return cl_powf_cold(x, y);
  const float k = __builtin_rintf(hi);
  const float f = (hi - k) + lo;
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f), (int)k);''', '''  const float hc = __builtin_fminf(__builtin_fmaxf(hi, -160.0f), 160.0f);   // ldexp over/underflows from here
  const float k = __builtin_rintf(hc);
  const float f = (hc - k) + (hc == hi ? lo : 0.0f);
  const float r = __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f), (int)k);
  // x == 0: log2 is -inf; pow(0, y) = 0 for y > 0, +inf for y < 0 (CLOUDSC: bases >= 0)
  return x == 0.0f ? (y > 0.0f ? 0.0f : __builtin_inff()) : r;'''),
]
