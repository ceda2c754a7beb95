// libm_check.cc -- bit-for-bit check of cloudsc_libm.h's exp/pow (host build of
// the device code) against the host C library's exp/pow, over random inputs in
// the ranges CLOUDSC uses and over wide random ranges.
//   g++ -O2 -mfma -ffp-contract=off -std=c++20 -I../dwarf-p-cloudsc_amd/csrc libm_check.cc -o libm_check
//   ./libm_check [millions of samples per case] [seed]
// Prints one line per case: samples, mismatches, worst ulp difference; exit 1 on
// any mismatch.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "cloudsc_libm.h"

using cloudsc_libm::HostTabs;

// the split (device) forms, with the complete functions as their cold path
struct HostCold {
  double exp(double x) const { return cloudsc_libm::exp(x, HostTabs{}); }
  double pow(double x, double y) const { return cloudsc_libm::pow(x, y, HostTabs{}); }
};
struct HostColdF {
  float expf(float x) const { return cloudsc_libm::expf(x, cloudsc_libm::HostTabsF{}); }
  float powf(float x, float y) const { return cloudsc_libm::powf(x, y, cloudsc_libm::HostTabsF{}); }
};
static float split_expf(float x) { return cloudsc_libm::expf_split(x, cloudsc_libm::HostTabsF{}, HostColdF{}); }
static float split_powf(float x, float y) {
  return cloudsc_libm::powf_split(x, y, cloudsc_libm::HostTabsF{}, HostColdF{});
}
static double split_exp(double x) { return cloudsc_libm::exp_split(x, HostTabs{}, HostCold{}); }
static double split_pow(double x, double y) { return cloudsc_libm::pow_split(x, y, HostTabs{}, HostCold{}); }

static long long ulpdiff(double a, double b) {
  long long ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  if (ia < 0) ia = (long long)0x8000000000000000ULL - ia;
  if (ib < 0) ib = (long long)0x8000000000000000ULL - ib;
  return ia > ib ? ia - ib : ib - ia;
}

struct Tally {
  const char* name;
  long long n = 0, bad = 0, worst = 0;
  double bx = 0, by = 0;
  void addf(float got, float want, float x, float y) {
    ++n;
    if (std::memcmp(&got, &want, 4) != 0 && !(std::isnan(got) && std::isnan(want))) {
      if (bad++ < 3) std::fprintf(stderr, "  %s(%a, %a): got %a want %a\n", name, x, y, got, want);
      worst = 1;
    }
  }
  void add(double got, double want, double x, double y) {
    ++n;
    if (std::memcmp(&got, &want, 8) != 0 && !(std::isnan(got) && std::isnan(want))) {
      long long u = ulpdiff(got, want);
      if (bad++ < 3) std::fprintf(stderr, "  %s(%a, %a): got %a want %a\n", name, x, y, got, want);
      if (u > worst) { worst = u; bx = x; by = y; }
    }
  }
  int report() const {
    std::printf("%-28s samples %12lld  mismatches %8lld  worst %lld ulp\n", name, n, bad, worst);
    return bad != 0;
  }
};

int main(int argc, char** argv) {
  const long long M = (argc > 1 ? std::atoll(argv[1]) : 4) * 1000000LL;
  const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 20250227u;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  HostTabs tabs;
  int fail = 0;

  {  // exp of the Tetens saturation arguments (|x| < 30) and the CLOUDSC range
    Tally t{"exp x in [-30,30]"};
    for (long long s = 0; s < M; ++s) {
      double x = -30.0 + 60.0 * u01(rng);
      t.add(cloudsc_libm::exp(x, tabs), std::exp(x), x, 0);
      t.add(split_exp(x), std::exp(x), x, 0);
    }
    fail |= t.report();
  }
  {
    Tally t{"exp x in [-745,710]"};
    for (long long s = 0; s < M; ++s) {
      double x = -745.0 + 1455.0 * u01(rng);
      t.add(cloudsc_libm::exp(x, tabs), std::exp(x), x, 0);
      t.add(split_exp(x), std::exp(x), x, 0);
    }
    fail |= t.report();
  }
  {  // the scaled paths: result overflow-near (k > 0) and subnormal-near (k < 0)
    Tally t{"exp |x| in [512,745]"};
    for (long long s = 0; s < M; ++s) {
      double x = (s & 1) ? 512.0 + 197.78 * u01(rng) : -512.0 - 233.2 * u01(rng);
      t.add(cloudsc_libm::exp(x, tabs), std::exp(x), x, 0);
      t.add(split_exp(x), std::exp(x), x, 0);
    }
    fail |= t.report();
  }
  {  // the tiny range the split form runs through its hot path (|x| < 2^-54 incl. subnormals)
    Tally t{"exp |x| < 2^-54"};
    for (long long s = 0; s < M; ++s) {
      const double x = ((s & 1) ? -1.0 : 1.0) * std::exp2(-1074.0 + 1020.0 * u01(rng));
      t.add(split_exp(x), std::exp(x), x, 0);
    }
    for (double x : {0x1p-54, -0x1p-54, 0x1.fffffffffffffp-55, -0x1.fffffffffffffp-55, 0x1p-1074, -0x1p-1074})
      t.add(split_exp(x), std::exp(x), x, 0);
    fail |= t.report();
  }
  {  // pow with y*log(x) tiny (x next to 1, small y)
    Tally t{"pow tiny y*log(x)"};
    for (long long s = 0; s < M; ++s) {
      const double x = 1.0 + (u01(rng) - 0.5) * std::exp2(-30.0 * u01(rng) - 20.0);
      const double y = ((s & 1) ? -1.0 : 1.0) * std::exp2(-60.0 * u01(rng));
      t.add(split_pow(x, y), std::pow(x, y), x, y);
    }
    fail |= t.report();
  }
  {  // tiny and special arguments
    Tally t{"exp special"};
    const double xs[] = {0.0, -0.0, 1e-300, -1e-300, 0x1p-60, 709.78, 709.79, -708.4, -745.13, -745.14, 1e4, -1e4,
                         INFINITY, -INFINITY, NAN, 1.0, -1.0, 0x1p-54, -0x1p-54, 512.0, -512.0, 1024.0, -1024.0};
    for (double x : xs) t.add(cloudsc_libm::exp(x, tabs), std::exp(x), x, 0);
    for (double x : xs) t.add(split_exp(x), std::exp(x), x, 0);
    for (long long s = 0; s < M / 8; ++s) {   // random bit patterns
      uint64_t b = rng();
      double x;
      std::memcpy(&x, &b, 8);
      t.add(cloudsc_libm::exp(x, tabs), std::exp(x), x, 0);
      t.add(split_exp(x), std::exp(x), x, 0);
    }
    fail |= t.report();
  }
  {  // pow with the exponents the kernel uses, over a log-uniform base
    const double ys[] = {0.666, 1.5, 0.333, 0.4, 0.5777, 3.0, 2.47, -1.79, 1.15, 2.47 * 1.0, -0.3, 0.25, 0.11, 0.5};
    Tally t{"pow kernel exponents"};
    for (long long s = 0; s < M; ++s) {
      double x = std::exp2(-60.0 + 80.0 * u01(rng));
      double y = ys[s % (sizeof(ys) / sizeof(ys[0]))];
      t.add(cloudsc_libm::pow(x, y, tabs), std::pow(x, y), x, y);
      t.add(split_pow(x, y), std::pow(x, y), x, y);
    }
    fail |= t.report();
  }
  {
    Tally t{"pow x in (0,1e3), |y|<8"};
    for (long long s = 0; s < M; ++s) {
      double x = 1e3 * u01(rng), y = -8.0 + 16.0 * u01(rng);
      t.add(cloudsc_libm::pow(x, y, tabs), std::pow(x, y), x, y);
      t.add(split_pow(x, y), std::pow(x, y), x, y);
    }
    fail |= t.report();
  }
  {
    Tally t{"pow x near 1"};
    for (long long s = 0; s < M; ++s) {
      double x = 1.0 + (u01(rng) - 0.5) * 1e-3, y = -50.0 + 100.0 * u01(rng);
      t.add(cloudsc_libm::pow(x, y, tabs), std::pow(x, y), x, y);
      t.add(split_pow(x, y), std::pow(x, y), x, y);
    }
    fail |= t.report();
  }
  {
    Tally t{"pow random bits"};
    for (long long s = 0; s < M / 4; ++s) {
      uint64_t bx = rng(), by = rng();
      double x, y;
      std::memcpy(&x, &bx, 8);
      std::memcpy(&y, &by, 8);
      if (s & 1) y = std::ldexp(y, -1000) ;   // moderate exponents too
      t.add(cloudsc_libm::pow(x, y, tabs), std::pow(x, y), x, y);
      t.add(split_pow(x, y), std::pow(x, y), x, y);
    }
    const double sp[][2] = {{0.0, 0.666}, {0.0, -1.0}, {-0.0, 3.0}, {-2.0, 3.0}, {-2.0, 0.5}, {1.0, NAN},
                            {NAN, 0.0}, {INFINITY, 0.5}, {0x1p-1070, 0.666}, {4.9e-324, 1.5}, {2.0, 1e300}};
    for (auto& p : sp) {
      t.add(cloudsc_libm::pow(p[0], p[1], tabs), std::pow(p[0], p[1]), p[0], p[1]);
      t.add(split_pow(p[0], p[1]), std::pow(p[0], p[1]), p[0], p[1]);
    }
    fail |= t.report();
  }
  // ---------------- single precision ----------------
  cloudsc_libm::HostTabsF tf;
  std::uniform_real_distribution<float> uf(0.0f, 1.0f);
  {
    Tally t{"expf x in [-110,90]"};
    for (long long s = 0; s < M; ++s) {
      const float x = -110.0f + 200.0f * uf(rng);
      t.addf(cloudsc_libm::expf(x, tf), ::expf(x), x, 0);
      t.addf(split_expf(x), ::expf(x), x, 0);
    }
    fail |= t.report();
  }
  {
    Tally t{"expf bit patterns (stride)"};
    for (uint64_t b = 0; b < (1ULL << 32); b += (M < 4000000 ? 128 : 8) + (rng() & 7)) {
      float x;
      const uint32_t u = (uint32_t)b;
      std::memcpy(&x, &u, 4);
      t.addf(cloudsc_libm::expf(x, tf), ::expf(x), x, 0);
    }
    fail |= t.report();
  }
  {
    const float ys[] = {0.666f, 1.5f, 0.333f, 0.4f, 0.5777f, 3.0f, 2.47f, -1.79f, 1.15f, -0.3f, 0.25f, 0.11f, 0.5f};
    Tally t{"powf kernel exponents"};
    for (long long s = 0; s < M; ++s) {
      const float x = std::exp2(-60.0f + 80.0f * uf(rng));
      const float y = ys[s % (sizeof(ys) / sizeof(ys[0]))];
      t.addf(cloudsc_libm::powf(x, y, tf), ::powf(x, y), x, y);
      t.addf(split_powf(x, y), ::powf(x, y), x, y);
    }
    fail |= t.report();
  }
  {
    Tally t{"powf random bits"};
    for (long long s = 0; s < M; ++s) {
      uint32_t bx = (uint32_t)rng(), by = (uint32_t)rng();
      float x, y;
      std::memcpy(&x, &bx, 4);
      std::memcpy(&y, &by, 4);
      if (s & 1) y = std::ldexp(y, -(int)(by % 120));
      t.addf(cloudsc_libm::powf(x, y, tf), ::powf(x, y), x, y);
      t.addf(split_powf(x, y), ::powf(x, y), x, y);
    }
    const float sp[][2] = {{0.0f, 0.666f}, {0.0f, -1.0f}, {-0.0f, 3.0f}, {-2.0f, 3.0f}, {-2.0f, 0.5f}, {1.0f, NAN},
                           {NAN, 0.0f}, {INFINITY, 0.5f}, {1e-40f, 0.666f}, {2.0f, 200.0f}, {2.0f, -149.5f}};
    for (auto& p : sp) t.addf(cloudsc_libm::powf(p[0], p[1], tf), ::powf(p[0], p[1]), p[0], p[1]);
    fail |= t.report();
  }
  return fail;
}
