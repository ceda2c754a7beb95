# the mid hook (next level's early loads) issued at high priority
EDITS = [("cloudsc_kcache.h",
"""      const auto mid = [&]() {
        if (PFM || PFA) {""",
"""      const auto mid = [&]() {
        __builtin_amdgcn_s_setprio(3);
        if (PFM || PFA) {"""),
("cloudsc_kcache.h",
"""            load_level<real, AER>(nxt, *(const KArgs<real>*)launder_uniform(ka), u2, u3, k1, klev, nproma,
                                  launder_vgpr(lo0));
        }
      };""",
"""            load_level<real, AER>(nxt, *(const KArgs<real>*)launder_uniform(ka), u2, u3, k1, klev, nproma,
                                  launder_vgpr(lo0));
        }
        __builtin_amdgcn_s_setprio(0);
      };""")]
