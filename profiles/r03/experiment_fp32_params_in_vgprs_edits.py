# experiment: fp32 parameters held in VGPRs for the whole level loop (one bulk load per call),
# instead of a scalar load + lgkmcnt(0) wait at each use
EDITS = [
    ("cloudsc_kcache.h", '''  for (int kloop = lev0; kloop < lev1; kloop++) {
    // the level index is laundered too, so no per-field induction pointers are formed''',
     '''  // the parameters in VGPRs (fp32): opaque per-lane copies, read by every use without a wait
  PT pv = *(const PT*)cpar;
  if constexpr (sizeof(real) == 4) {
    float* pa = (float*)&pv;
#pragma unroll
    for (int q = 0; q < (int)(sizeof(PT) / 4) - 4; q++) asm volatile("" : "+v"(pa[q]));
  }
  for (int kloop = lev0; kloop < lev1; kloop++) {
    // the level index is laundered too, so no per-field induction pointers are formed'''),
    ("cloudsc_kcache.h", '''    LevelState<real> ls;
    PhysOut<real> po;
    {
      CLOUDSC_PARAMS_HERE;
      init_level(c, cur, ls);''', '''    LevelState<real> ls;
    PhysOut<real> po;
    {
      const PT& c = sizeof(real) == 4 ? pv : *(const PT*)launder_uniform(cpar);
      init_level(c, cur, ls);'''),
    ("cloudsc_kcache.h", '''      const KArgs<real>& A = *(const KArgs<real>*)launder_uniform(ka);
      CLOUDSC_PARAMS_HERE;
      store_level(A, u2, u3, k, klev, nproma, lo, physics, ls, po);''', '''      const KArgs<real>& A = *(const KArgs<real>*)launder_uniform(ka);
      const PT& c = sizeof(real) == 4 ? pv : *(const PT*)launder_uniform(cpar);
      store_level(A, u2, u3, k, klev, nproma, lo, physics, ls, po);'''),
]
EDITS.append(("cloudsc_dev.h", '''template <typename T>
CLOUDSC_HD T sval(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(v));
#endif
  return v;
}''', '''template <typename T>
CLOUDSC_HD T sval(T v) {
  return v;
}'''))
