EDITS = [("cloudsc_kcache.h",
"""    real paph_nn, pmfu_nn, pmfd_nn, plu_nn;
    {
      const KArgs<real>& A = *(const KArgs<real>*)launder_uniform(ka);""",
"""    real paph_nn, pmfu_nn, pmfd_nn, plu_nn;
    __builtin_amdgcn_s_setprio(3);
    {
      const KArgs<real>& A = *(const KArgs<real>*)launder_uniform(ka);"""),
("cloudsc_kcache.h",
"""        pmfu_nn = ldg1(A.pmfu, i2, lo); pmfd_nn = ldg1(A.pmfd, i2, lo); plu_nn = ldg1(A.plu, i2, lo);
      }
    }
""",
"""        pmfu_nn = ldg1(A.pmfu, i2, lo); pmfd_nn = ldg1(A.pmfd, i2, lo); plu_nn = ldg1(A.plu, i2, lo);
      }
    }
    __builtin_amdgcn_s_setprio(0);
""")]
