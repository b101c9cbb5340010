// Checks that HIP's sincos(x) returns bit for bit what sin(x) and cos(x)
// return (ocml) on fp64 inputs of the ranges the kernels use and beyond, so
// that the kernels may fuse their sin / cos pairs (one range reduction each).
// sin / cos and sincos run in separate kernels (no fusing by the compiler).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/sincos_check.hip -o tools/sincos_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ double arg(unsigned long long i, unsigned long long seed) {
  unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
  z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 27; z *= 0x94D049BB133111EBull; z ^= z >> 31;
  const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);  // [0, 1)
  switch ((int)(i % 4)) {
    case 0: return (u - 0.5) * 7.0;                                  // |angle| < 200 deg, radians
    case 1: return (u - 0.5) * 800.0 * 0.017453292519943295;         // degrees * d2r, wide
    case 2: return (u - 0.5) * 1e6;                                  // large arguments
    default: return __longlong_as_double((long long)(z & 0x7fefffffffffffffull)) * ((z >> 63) ? -1.0 : 1.0);
  }
}
__global__ void k_sep(unsigned long long n, unsigned long long seed, double2 *o) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const double x = arg(i, seed);
    o[i] = make_double2(sin(x), cos(x));
  }
}
__global__ void k_fused(unsigned long long n, unsigned long long seed, double2 *o) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    double s, c;
    sincos(arg(i, seed), &s, &c);
    o[i] = make_double2(s, c);
  }
}
__global__ void k_cmp(unsigned long long n, const double2 *a, const double2 *b, unsigned long long *bad) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x)
    if (__double_as_longlong(a[i].x) != __double_as_longlong(b[i].x) ||
        __double_as_longlong(a[i].y) != __double_as_longlong(b[i].y))
      atomicAdd(bad, 1ull);
}

int main() {
  const unsigned long long n = 1ull << 26;
  double2 *a, *b;
  unsigned long long *bad, hb = 0, tot = 0;
  if (hipMalloc(&a, n * 16) || hipMalloc(&b, n * 16) || hipMalloc(&bad, 8)) return 2;
  for (unsigned long long seed = 1; seed <= 4; ++seed) {
    if (hipMemset(bad, 0, 8)) return 2;
    hipLaunchKernelGGL(k_sep, dim3(4096), dim3(256), 0, 0, n, seed, a);
    hipLaunchKernelGGL(k_fused, dim3(4096), dim3(256), 0, 0, n, seed, b);
    hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, n, a, b, bad);
    if (hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost)) return 2;
    tot += hb;
  }
  printf("sincos vs sin / cos: %llu of %llu inputs differ\n", tot, 4 * n);
  return tot != 0;
}
