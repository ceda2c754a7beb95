# Experiment build (round 6): the compute floor -- every KSEG item reads and writes block (b & 31), so the
# data stays in the memory-side cache; profiles/r06/compute_memory_floors.txt.
#   python tools/exp_variant.py cmponly32 tools/exp_compute_floor_edits.py -DCLOUDSC_ONLY_KSEG=8
EDITS = [
("cloudsc_kcache.h", """  const size_t u1 = (size_t)b * nproma;                            // [nblocks][nproma]
  const size_t u2 = (size_t)b * klev * nproma;                     // [nblocks][klev][nproma]
  const size_t uh = (size_t)b * (klev + 1) * nproma;               // [nblocks][klev+1][nproma]
  const size_t u3 = (size_t)b * 5 * klev * nproma;                 // [nblocks][5][klev][nproma]""",
"""  const size_t b0 = (size_t)(b & 31);
  const size_t u1 = b0 * nproma;
  const size_t u2 = b0 * klev * nproma;
  const size_t uh = b0 * (klev + 1) * nproma;
  const size_t u3 = b0 * 5 * klev * nproma;"""),
("cloudsc_kcache.h", """        flux_top(c, A, (size_t)b * (A.klev + 1) * nproma, lo);""", """        flux_top(c, A, (size_t)(b & 31) * (A.klev + 1) * nproma, lo);"""),
("cloudsc_kcache.h", """      stg(((const KArgs<real>*)launder_uniform(ka))->prainfrac, (size_t)b * nproma, lo, cs.rainfrac);
    }
#ifdef CLOUDSC_KSEG_TRACE""", """      stg(((const KArgs<real>*)launder_uniform(ka))->prainfrac, (size_t)(b & 31) * nproma, lo, cs.rainfrac);
    }
#ifdef CLOUDSC_KSEG_TRACE"""),
]
