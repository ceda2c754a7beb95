EDITS = [("cloudsc_kcache.h",
"""struct EarlyIn {
  real pt, pq, ttt, ttq, tta, pa, pap;""",
"""struct EarlyIn {
  real pt, pq, ttt, ttq, tta, pa, pap, psupsat;"""),
("cloudsc_kcache.h",
"""  E.tta = ldg1(A.tta, i, lo); E.pa = ldg1(A.pa, i, lo); E.pap = ldg1(A.pap, i, lo);
""",
"""  E.tta = ldg1(A.tta, i, lo); E.pa = ldg1(A.pa, i, lo); E.pap = ldg1(A.pap, i, lo);
  E.psupsat = ldg1(A.psupsat, i, lo);
"""),
("cloudsc_kcache.h",
"""  L.psnde = ldg1(A.psnde, i, lo); L.psupsat = ldg1(A.psupsat, i, lo);
  if (AER) {""",
"""  L.psnde = ldg1(A.psnde, i, lo);
  if (AER) {"""),
("cloudsc_kcache.h",
"""  L.pt = E.pt; L.pq = E.pq; L.ttt = E.ttt; L.ttq = E.ttq; L.tta = E.tta; L.pa = E.pa; L.pap = E.pap;
""",
"""  L.pt = E.pt; L.pq = E.pq; L.ttt = E.ttt; L.ttq = E.ttq; L.tta = E.tta; L.pa = E.pa; L.pap = E.pap;
  L.psupsat = E.psupsat;
""")]
