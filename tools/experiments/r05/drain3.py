# PF 3 (the fp64 default) also drains the prologue's loads before the level loop, like PF 1: the waitcnt pass
# then no longer waits at every level top for the previous level's stores (s_waitcnt vmcnt(9) before the
# neighbour rotation)
EDITS = [("cloudsc_kcache.h",
          "  if constexpr (PFX) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt(7), lgkmcnt(15)",
          "  if constexpr (PFX || PFM) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt(7), lgkmcnt(15)")]
