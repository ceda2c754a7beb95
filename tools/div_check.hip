// div_check.hip -- diagnostic: accuracy of v_rcp_f64 on this device, and how
// often shorter correctly-rounded-division sequences differ from the IEEE
// quotient n / d (the compiler's div_scale/div_fmas/div_fixup sequence).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/div_check.hip -o build/div_check
//   build/div_check [billions of samples]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}
// random double with exponent in [-e, e] and a random mantissa (some all-ones / all-zero mantissas)
__device__ __forceinline__ double rnd(unsigned long long s, int e) {
  unsigned long long m = mix(s);
  const int ex = (int)(mix(s + 0x9e3779b97f4a7c15ULL) % (unsigned long long)(2 * e + 1)) - e;
  unsigned long long mant = m & 0xfffffffffffffULL;
  const unsigned sel = (unsigned)(m >> 60);
  if (sel == 0) mant = 0xfffffffffffffULL;              // all-ones mantissa
  else if (sel == 1) mant = 0;                          // power of two
  else if (sel == 2) mant |= 0xffffffff00000ULL;        // many leading ones
  const unsigned long long bits = ((unsigned long long)(ex + 1023) << 52) | mant;
  return __longlong_as_double((long long)bits) * ((m >> 59) & 1 ? -1.0 : 1.0);
}
__device__ __forceinline__ double div2(double n, double d) {   // the kernels' cl_div
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0); r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0); r = __builtin_fma(r, e, r);
  const double q = n * r, rem = __builtin_fma(-d, q, n);
  return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ double div1(double n, double d) {   // one Newton step
  double r = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, r, 1.0); r = __builtin_fma(r, e, r);
  const double q = n * r, rem = __builtin_fma(-d, q, n);
  return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ double div0(double n, double d) {   // no Newton step
  const double r = __builtin_amdgcn_rcp(d);
  const double q = n * r, rem = __builtin_fma(-d, q, n);
  return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ double div1b(double n, double d) {  // one step, then two quotient corrections
  double r = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, r, 1.0); r = __builtin_fma(r, e, r);
  double q = n * r, rem = __builtin_fma(-d, q, n);
  q = __builtin_fma(rem, r, q);
  rem = __builtin_fma(-d, q, n);
  return __builtin_fma(rem, r, q);
}

__global__ void check(unsigned long long seed, long long n, int e, unsigned long long* cnt) {
  unsigned long long c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const double d = rnd(seed + 2 * i, e), x = rnd(seed + 2 * i + 1, e);
    const double ref = x / d;
    const double rr = 1.0 / d;
    const double r0 = __builtin_amdgcn_rcp(d);
    const long long ulp = __double_as_longlong(r0) - __double_as_longlong(rr);
    const long long a = ulp < 0 ? -ulp : ulp;
    if (a == 0) c[0]++; else if (a <= 1) c[1]++; else if (a <= 4) c[2]++; else c[3]++;
    if (__double_as_longlong(div2(x, d)) != __double_as_longlong(ref)) c[4]++;
    if (__double_as_longlong(div1(x, d)) != __double_as_longlong(ref)) c[5]++;
    if (__double_as_longlong(div0(x, d)) != __double_as_longlong(ref)) c[6]++;
    if (__double_as_longlong(div1b(x, d)) != __double_as_longlong(ref)) c[7]++;
  }
  for (int k = 0; k < 8; k++) if (c[k]) atomicAdd(&cnt[k], c[k]);
}

int main(int argc, char** argv) {
  const double billions = argc > 1 ? atof(argv[1]) : 1.0;
  const long long n = (long long)(billions * 1e9);
  unsigned long long* d = nullptr;
  hipMalloc(&d, 8 * sizeof(unsigned long long));
  const char* names[8] = {"rcp exact (= RN(1/d))", "rcp 1 ulp", "rcp 2-4 ulp", "rcp > 4 ulp",
                          "div 2 Newton (cl_div) != IEEE", "div 1 Newton != IEEE", "div 0 Newton != IEEE",
                          "div 1 Newton + 2 corrections != IEEE"};
  for (int e : {20, 300}) {
    hipMemset(d, 0, 8 * sizeof(unsigned long long));
    check<<<4096, 256>>>(12345 + e, n, e, d);
    unsigned long long h[8];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("exponents in [-%d, %d], %lld samples\n", e, e, n);
    for (int k = 0; k < 8; k++) printf("  %-40s %llu\n", names[k], h[k]);
  }
  return 0;
}
