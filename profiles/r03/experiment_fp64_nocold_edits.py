# experiment only (NOT exact outside the hot range): fp64 exp/pow without the out-of-line cold calls
EDITS = [
    ("cloudsc_dev.h", '''struct DevLibmCold {
  __device__ __forceinline__ double exp(double x) const { return cl_exp_cold(x); }
  __device__ __forceinline__ double pow(double x, double y) const { return cl_pow_cold(x, y); }''',
     '''struct DevLibmCold {
  __device__ __forceinline__ double exp(double x) const { return x > 0.0 ? __builtin_inf() : (x != x ? x : 0.0); }
  __device__ __forceinline__ double pow(double x, double y) const { return x == 0.0 ? (y > 0.0 ? 0.0 : __builtin_inf()) : __builtin_nan(""); }'''),
]
