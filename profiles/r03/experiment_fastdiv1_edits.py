# fp32: division as v_rcp_f32, q = n*r, one residual correction
EDITS = [
    ("cloudsc_dev.h", '''  float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  r = __builtin_fmaf(e, r, r);
  float q = n * r;
  float rem = __builtin_fmaf(-d, q, n);
  q = __builtin_fmaf(rem, r, q);
  rem = __builtin_fmaf(-d, q, n);
  return __builtin_fmaf(rem, r, q);''', '''  const float r = __builtin_amdgcn_rcpf(d);
  const float q = n * r;
  return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);'''),
    ("cloudsc_dev.h", '''  float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  r = __builtin_fmaf(e, r, r);
  return {d, r};''', '''  return {d, __builtin_amdgcn_rcpf(d)};'''),
    ("cloudsc_dev.h", '''  float q = n * rd.r;
  float rem = __builtin_fmaf(-rd.d, q, n);
  q = __builtin_fmaf(rem, rd.r, q);
  rem = __builtin_fmaf(-rd.d, q, n);
  return __builtin_fmaf(rem, rd.r, q);''', '''  const float q = n * rd.r;
  return __builtin_fmaf(__builtin_fmaf(-rd.d, q, n), rd.r, q);'''),
]
