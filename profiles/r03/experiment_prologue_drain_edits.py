# drain the prologue's loads once before the level loop, so the loop header's merge of
# (prologue, latch) states does not make every level wait for the previous level's stores
EDITS = [("cloudsc_kcache.h", '''    if (PFA) load_level<real, AER>(nxt, A, u2, u3, lev0, klev, nproma, lo);
  }''', '''    if (PFA) load_level<real, AER>(nxt, A, u2, u3, lev0, klev, nproma, lo);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the prologue's loads, once per segment
#endif''')]
