KERNEL = r'''
// experiment: the same traffic with two levels per step -- each plane's level
// k and k+1 stored (and, READ, loaded) back to back: 2 x 64 lanes contiguous
template <typename real, bool READ>
__global__ void __launch_bounds__(64) place_probe_pair_kernel(const ProbeArgs a) {
  constexpr int NL = READ ? kProbeInLevel + 9 : 1;
  const int lane = threadIdx.x;
  for (int it = blockIdx.x; it < a.nitems; it += gridDim.x) {
    const long long b = it / a.nsub;
    const int sub = it - (int)(b * a.nsub);
    const int jl = sub * 64 + lane;
    const long long col = b * a.nproma + jl;
    if (jl >= a.nproma || col >= a.ngptot) continue;
    const size_t np = (size_t)a.nproma, kl = (size_t)a.klev;
    const size_t lvl0 = (size_t)b * kl * np + jl, half0 = (size_t)b * (kl + 1) * np + jl;
    const size_t spc0 = (size_t)b * 5 * kl * np + jl;
    real acc = (real)0, nxt[2][NL];
    auto load = [&](int k, int h) {
      if constexpr (READ) {
        const size_t il = lvl0 + (size_t)k * np;
#pragma unroll
        for (int q = 0; q < kProbeInLevel; q++) nxt[h][q] = a.in_level[q] ? ldnt<real>(a.in_level[q], il) : (real)0;
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
          for (int s = 0; s < 4; s++)
            nxt[h][kProbeInLevel + 4 * q + s] =
                a.in_species[q] ? ldnt<real>(a.in_species[q], spc0 + ((size_t)s * kl + k) * np) : (real)0;
        nxt[h][NL - 1] = a.paph ? ldnt<real>(a.paph, half0 + (size_t)(k + 1) * np) : (real)0;
      }
    };
    auto load2 = [&](int k) {   // planes of k and k+1 interleaved per field
      if constexpr (READ) {
        const int k1 = k + 1 < a.klev ? k + 1 : k;
        const size_t il = lvl0 + (size_t)k * np, il1 = lvl0 + (size_t)k1 * np;
#pragma unroll
        for (int q = 0; q < kProbeInLevel; q++) {
          nxt[0][q] = a.in_level[q] ? ldnt<real>(a.in_level[q], il) : (real)0;
          nxt[1][q] = a.in_level[q] ? ldnt<real>(a.in_level[q], il1) : (real)0;
        }
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
          for (int s = 0; s < 4; s++) {
            nxt[0][kProbeInLevel + 4 * q + s] =
                a.in_species[q] ? ldnt<real>(a.in_species[q], spc0 + ((size_t)s * kl + k) * np) : (real)0;
            nxt[1][kProbeInLevel + 4 * q + s] =
                a.in_species[q] ? ldnt<real>(a.in_species[q], spc0 + ((size_t)s * kl + k1) * np) : (real)0;
          }
        nxt[0][NL - 1] = a.paph ? ldnt<real>(a.paph, half0 + (size_t)(k + 1) * np) : (real)0;
        nxt[1][NL - 1] = a.paph ? ldnt<real>(a.paph, half0 + (size_t)(k1 + 1) * np) : (real)0;
      }
    };
    (void)load;
    load2(0);
    const real v0 = (real)b;
#pragma unroll
    for (int q = 0; q < kProbeOutHalf; q++)
      if (a.out_half[q]) stnt<real>(a.out_half[q], half0, v0);
    for (int k = 0; k < a.klev; k += 2) {
      real cur[2][NL];
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int q = 0; q < NL; q++) cur[h][q] = nxt[h][q];
      if (k + 2 < a.klev) load2(k + 2);
      const bool two = k + 1 < a.klev;
      const size_t il = lvl0 + (size_t)k * np;
      const real v = v0 + (real)k;
#pragma unroll
      for (int q = 0; q < kProbeOutLevel; q++)
        if (a.out_level[q]) { stnt<real>(a.out_level[q], il, v); if (two) stnt<real>(a.out_level[q], il + np, v); }
      if (a.out_species)
#pragma unroll
        for (int s = 0; s < 5; s++) {
          const size_t i = spc0 + ((size_t)s * kl + k) * np;
          stnt<real>(a.out_species, i, v);
          if (two) stnt<real>(a.out_species, i + np, v);
        }
#pragma unroll
      for (int q = 0; q < kProbeOutHalf; q++)
        if (a.out_half[q]) {
          stnt<real>(a.out_half[q], half0 + (size_t)(k + 1) * np, v);
          if (two) stnt<real>(a.out_half[q], half0 + (size_t)(k + 2) * np, v);
        }
      if constexpr (READ) {
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int q = 0; q < NL; q++) acc += cur[h][q];
      }
    }
    if (a.out_surf) stnt<real>(a.out_surf, (size_t)b * np + jl, acc);
  }
}
'''
EDITS = [("cloudsc_place.hip",
"""ProbeArgs probe_args(const cloudsc_fields_t* f, int ngptot, int nproma, int klev, bool read) {""",
KERNEL + """
ProbeArgs probe_args(const cloudsc_fields_t* f, int ngptot, int nproma, int klev, bool read) {"""),
("cloudsc_place.hip",
"""  const ProbeArgs a = probe_args(f, ngptot, nproma, klev, mode == 1);""",
"""  const ProbeArgs a = probe_args(f, ngptot, nproma, klev, mode == 1 || mode == 3);"""),
("cloudsc_place.hip",
"""    if (precision == CLOUDSC_FP64) {
      if (mode == 1) hipLaunchKernelGGL((place_probe_kernel<double, true>), grid, dim3(64), 0, stream, a);""",
"""    if (mode >= 2) {
      if (precision == CLOUDSC_FP64) {
        if (mode == 3) hipLaunchKernelGGL((place_probe_pair_kernel<double, true>), grid, dim3(64), 0, stream, a);
        else hipLaunchKernelGGL((place_probe_pair_kernel<double, false>), grid, dim3(64), 0, stream, a);
      } else {
        if (mode == 3) hipLaunchKernelGGL((place_probe_pair_kernel<float, true>), grid, dim3(64), 0, stream, a);
        else hipLaunchKernelGGL((place_probe_pair_kernel<float, false>), grid, dim3(64), 0, stream, a);
      }
    } else if (precision == CLOUDSC_FP64) {
      if (mode == 1) hipLaunchKernelGGL((place_probe_kernel<double, true>), grid, dim3(64), 0, stream, a);"""),
("cloudsc_place.hip",
"""  if (!f || !ms || reps <= 0 || (mode != 0 && mode != 1)) return CLOUDSC_EINVAL;""",
"""  if (!f || !ms || reps <= 0 || mode < 0 || mode > 3) return CLOUDSC_EINVAL;"""),
]
