# PF 1: the level loop unrolled by two with the prefetch buffers swapping roles
# (cur/nxt), so the level-(k+1) prefetch needs no cur = nxt register copies
EDITS = [
 ("cloudsc_kcache.h", '''  for (int kloop = lev0; kloop < lev1; kloop++) {
    // the level index is laundered too, so no per-field induction pointers are formed''',
  '''  const auto level = [&](const int kloop, LevelIn<real>& cur, LevelIn<real>& nxt) {
    // the level index is laundered too, so no per-field induction pointers are formed'''),
 ("cloudsc_kcache.h", '''    if (PFX) cur = nxt;
  }
}''', '''  };
  if constexpr (PFX) {
    for (int kloop = lev0; kloop < lev1; kloop += 2) {
      level(kloop, cur, nxt);
      if (kloop + 1 < lev1) level(kloop + 1, nxt, cur);
    }
  } else {
    for (int kloop = lev0; kloop < lev1; kloop++) level(kloop, cur, nxt);
  }
}'''),
]
