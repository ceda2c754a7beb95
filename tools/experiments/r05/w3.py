EDITS = [("cloudsc_gpu.hip",
"""  static constexpr int code = 20 + CLOUDSC_FP32_PF, waves = 2, pf = CLOUDSC_FP32_PF;""",
"""  static constexpr int code = 30 + CLOUDSC_FP32_PF, waves = 3, pf = CLOUDSC_FP32_PF;"""),
("cloudsc_gpu.hip", """  if (w > per_simd) w = per_simd;""", """  w = per_simd;"""),
("cloudsc_kcache.h", """  constexpr bool PVR = sizeof(real) == 4;""", """  constexpr bool PVR = false;"""),
]
