// div_const_check.c -- host check that a division by a run-time-constant
// divisor d, computed with the host's correctly rounded reciprocal
// r = RN(1/d) and cl_div's correction steps (cloudsc_dev.h, cl_div(n, Recip)),
//   fp64:  q = n*r; q += fma(-d, q, n)*r                  (one correction)
//   fp32:  two corrections
// returns the IEEE quotient n/d.  Divisors: the ones CLOUDSC divides by
// (literals and the cloudsc100 parameters), plus random divisors.
//   gcc -O2 -ffp-contract=off tools/div_const_check.c -lm -o /tmp/dcc && /tmp/dcc [millions]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9e3779b97f4a7c15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

static double rand_double(void) {   // random sign/mantissa, exponent in [-300, 300]
  uint64_t m = rnd() & ((1ull << 52) - 1), e = (uint64_t)(1023 - 300 + rnd() % 601), sg = rnd() & 1;
  uint64_t b = (sg << 63) | (e << 52) | m; double x; memcpy(&x, &b, 8); return x;
}
static float rand_float(void) {     // exponent in [-60, 60]
  uint32_t m = (uint32_t)rnd() & ((1u << 23) - 1), e = (uint32_t)(127 - 60 + rnd() % 121), sg = rnd() & 1;
  uint32_t b = (sg << 31) | (e << 23) | m; float x; memcpy(&x, &b, 4); return x;
}

static long check_d(double d, long n_iter) {
  volatile double one = 1.0;
  const double r = one / d;
  long bad = 0;
  for (long i = 0; i < n_iter; ++i) {
    double n = rand_double();
    double q = n * r;
    double rem = fma(-d, q, n);
    double q2 = fma(rem, r, q);
    if (q2 != n / d) { if (bad < 3) printf("  fp64 d=%.17g n=%.17g got %.17g want %.17g\n", d, n, q2, n / d); ++bad; }
  }
  return bad;
}
static long check_f(float d, long n_iter) {
  volatile float one = 1.0f;
  const float r = one / d;
  long bad = 0;
  for (long i = 0; i < n_iter; ++i) {
    float n = rand_float();
    float q = n * r;
    float rem = fmaf(-d, q, n);
    q = fmaf(rem, r, q);
    rem = fmaf(-d, q, n);
    q = fmaf(rem, r, q);
    if (q != n / d) { if (bad < 3) printf("  fp32 d=%.9g n=%.9g got %.9g want %.9g\n", d, n, q, n / d); ++bad; }
  }
  return bad;
}

int main(int argc, char** argv) {
  const long m = (argc > 1 ? atol(argv[1]) : 10) * 1000000L;
  const double ds[] = {0.2, 15000.0, 273.0, 287.0596736665907, 7200.0, 500.0, 0.0050899999999999999};
  long total = 0;
  for (unsigned i = 0; i < sizeof(ds) / sizeof(ds[0]); ++i) {
    long b64 = check_d(ds[i], m), b32 = check_f((float)ds[i], m);
    printf("d=%-22.17g fp64 mismatches %ld / %ld, fp32 %ld / %ld\n", ds[i], b64, m, b32, m);
    total += b64 + b32;
  }
  long rb = 0;
  for (int i = 0; i < 1000; ++i) {
    double d = fabs(rand_double());
    rb += check_d(d, m / 1000) + check_f((float)fabs(rand_float()), m / 1000);
  }
  printf("1000 random divisors: %ld mismatches / %ld\n", rb, 2 * m);
  total += rb;
  printf("total mismatches %ld\n", total);
  return total != 0;
}
