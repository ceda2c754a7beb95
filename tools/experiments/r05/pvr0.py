EDITS = [("cloudsc_kcache.h", """  constexpr bool PVR = sizeof(real) == 4;""", """  constexpr bool PVR = false;""")]
