EDITS = [("cloudsc_kcache.h",
"""      const real zqp = cl_div_p<real>(c, R(1.0), r_pap);
  #pragma unroll
      for (int it = 0; it < 2; it++) {""",
"""      const real zqp = cl_div_p<real>(c, R(1.0), r_pap);
#ifdef __HIP_DEVICE_COMPILE__
      __builtin_amdgcn_s_setprio(2);
#endif
  #pragma unroll
      for (int it = 0; it < 2; it++) {"""),
("cloudsc_kcache.h",
"""      zdqs = qsm - zqsmix;
    }
""",
"""      zdqs = qsm - zqsmix;
#ifdef __HIP_DEVICE_COMPILE__
      __builtin_amdgcn_s_setprio(0);
#endif
    }
""")]
