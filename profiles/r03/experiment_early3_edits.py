# PF 3: psupsat, plude and psnde (read by sections 3.1 / 3.2, early in the physics) join the
# mid-level-prefetched early group; the late group keeps pvfl, pvfi, phrsw, phrlw, pvervel (3.4, 8)
EDITS = [
 ("cloudsc_kcache.h", '''template <typename real>
struct EarlyIn {
  real pt, pq, ttt, ttq, tta, pa, pap;
  real pclv[4], ttcld[4];
};''', '''template <typename real>
struct EarlyIn {
  real pt, pq, ttt, ttq, tta, pa, pap, psupsat, plude, psnde;
  real pclv[4], ttcld[4];
};'''),
 ("cloudsc_kcache.h", '''  E.tta = ldg1(A.tta, i, lo); E.pa = ldg1(A.pa, i, lo); E.pap = ldg1(A.pap, i, lo);
#pragma unroll''', '''  E.tta = ldg1(A.tta, i, lo); E.pa = ldg1(A.pa, i, lo); E.pap = ldg1(A.pap, i, lo);
  E.psupsat = ldg1(A.psupsat, i, lo); E.plude = ldg1(A.plude_in, i, lo); E.psnde = ldg1(A.psnde, i, lo);
#pragma unroll'''),
 ("cloudsc_kcache.h", '''  L.plude = ldg1(A.plude_in, i, lo); L.pvfl = ldg1(A.pvfl, i, lo); L.pvfi = ldg1(A.pvfi, i, lo);
  L.phrsw = ldg1(A.phrsw, i, lo); L.phrlw = ldg1(A.phrlw, i, lo); L.pvervel = ldg1(A.pvervel, i, lo);
  L.psnde = ldg1(A.psnde, i, lo); L.psupsat = ldg1(A.psupsat, i, lo);
  if (AER) {''', '''  L.pvfl = ldg1(A.pvfl, i, lo); L.pvfi = ldg1(A.pvfi, i, lo);
  L.phrsw = ldg1(A.phrsw, i, lo); L.phrlw = ldg1(A.phrlw, i, lo); L.pvervel = ldg1(A.pvervel, i, lo);
  if (AER) {'''),
 ("cloudsc_kcache.h", '''  L.pt = E.pt; L.pq = E.pq; L.ttt = E.ttt; L.ttq = E.ttq; L.tta = E.tta; L.pa = E.pa; L.pap = E.pap;''',
  '''  L.pt = E.pt; L.pq = E.pq; L.ttt = E.ttt; L.ttq = E.ttq; L.tta = E.tta; L.pa = E.pa; L.pap = E.pap;
  L.psupsat = E.psupsat; L.plude = E.plude; L.psnde = E.psnde;'''),
]
