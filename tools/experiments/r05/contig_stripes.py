# dequeue stripes as contiguous block ranges instead of b = lb * S + st (blocks 8 apart): the 256 workgroups of an
# XCD then work on neighbouring blocks (fewer distinct pages in flight per XCD)
EDITS = [("cloudsc_kcache.h",
          "    const int b = lb * S + st;",
          "    const int b = st * (P.nblocks / S) + (st < P.nblocks % S ? st : P.nblocks % S) + lb;")]
