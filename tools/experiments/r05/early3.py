EDITS = [("cloudsc_kcache.h",
"""struct EarlyIn {
  real pt, pq, ttt, ttq, tta, pa, pap;""",
"""struct EarlyIn {
  real pt, pq, ttt, ttq, tta, pa, pap, psupsat, plude, psnde;"""),
("cloudsc_kcache.h",
"""  E.tta = ldg1(A.tta, i, lo); E.pa = ldg1(A.pa, i, lo); E.pap = ldg1(A.pap, i, lo);
""",
"""  E.tta = ldg1(A.tta, i, lo); E.pa = ldg1(A.pa, i, lo); E.pap = ldg1(A.pap, i, lo);
  E.psupsat = ldg1(A.psupsat, i, lo); E.plude = ldg1(A.plude_in, i, lo); E.psnde = ldg1(A.psnde, i, lo);
"""),
("cloudsc_kcache.h",
"""  L.plude = ldg1(A.plude_in, i, lo); L.pvfl = ldg1(A.pvfl, i, lo); L.pvfi = ldg1(A.pvfi, i, lo);""",
"""  L.pvfl = ldg1(A.pvfl, i, lo); L.pvfi = ldg1(A.pvfi, i, lo);"""),
("cloudsc_kcache.h",
"""  L.psnde = ldg1(A.psnde, i, lo); L.psupsat = ldg1(A.psupsat, i, lo);
  if (AER) {""",
"""  if (AER) {"""),
("cloudsc_kcache.h",
"""  L.pt = E.pt; L.pq = E.pq; L.ttt = E.ttt; L.ttq = E.ttq; L.tta = E.tta; L.pa = E.pa; L.pap = E.pap;
""",
"""  L.pt = E.pt; L.pq = E.pq; L.ttt = E.ttt; L.ttq = E.ttq; L.tta = E.tta; L.pa = E.pa; L.pap = E.pap;
  L.psupsat = E.psupsat; L.plude = E.plude; L.psnde = E.psnde;
""")]
