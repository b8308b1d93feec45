// Probe: is 1 / RN(sqrt(d)) computed from the square root's own reciprocal estimate (one Newton
// step... two steps, then the division's final correction) bit-identical to div_core(1, sqrt_core(d)) (the
// kernel's correctly rounded pair)? Counts mismatches over random and targeted operands.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/fused_inv_probe.hip -o tools/fused_inv_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double sqrt_core(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double div_core(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = a * r;
  const double rem = __builtin_fma(-b, q, a);
  return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ double inv_fused(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  const double s = __builtin_fma(d, h, g);
  double q = h + h;
  double f = __builtin_fma(-s, q, 1.0);
  q = __builtin_fma(q, f, q);
  f = __builtin_fma(-s, q, 1.0);  // a second step, as the division's own sequence takes
  q = __builtin_fma(q, f, q);
  const double rem = __builtin_fma(-s, q, 1.0);
  return __builtin_fma(rem, q, q);
}
__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// mode 0: random d in [2^-40, 2^40]; mode 1: d = s*s rounded for s with an all-ones-ish significand;
// mode 2: d within a few ulps of 1 and of powers of 4
__global__ void k(uint64_t base, int mode, unsigned long long* bad, double* ex) {
  const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t z = mix(i);
  double d;
  if (mode == 0) {
    const uint64_t e = 1023 - 40 + (z >> 56) % 81;
    d = __builtin_bit_cast(double, (e << 52) | (mix(z) & ((1ull << 52) - 1)));
  } else if (mode == 1) {
    const uint64_t e = 1023 - 20 + (z >> 58) % 41;
    const uint64_t m = ((1ull << 52) - 1) - (z & 0xFFFF);  // significands near all ones
    const double s = __builtin_bit_cast(double, (e << 52) | m);
    d = s * s;
  } else {
    const int64_t k = (int64_t)(z % 4096) - 2048;
    const uint64_t e = 1023 - 30 + 2 * ((z >> 40) % 31);
    d = __builtin_bit_cast(double, (uint64_t)((int64_t)(e << 52) + k));
  }
  const double a = div_core(1.0, sqrt_core(d));
  const double b = inv_fused(d);
  if (__builtin_bit_cast(uint64_t, a) != __builtin_bit_cast(uint64_t, b)) {
    const unsigned long long n = atomicAdd(bad, 1ull);
    if (n < 8) { ex[3 * n] = d; ex[3 * n + 1] = a; ex[3 * n + 2] = b; }
  }
}
int main() {
  unsigned long long* bad;
  double* ex;
  hipMalloc(&bad, 8);
  hipMalloc(&ex, 24 * 8);
  const int threads = 256, blocks = 1 << 16;
  const uint64_t per = (uint64_t)threads * blocks;
  for (int mode = 0; mode < 3; ++mode) {
    hipMemset(bad, 0, 8);
    const int reps = mode == 0 ? 600 : 200;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, (uint64_t)r * per + ((uint64_t)mode << 60), mode, bad, ex);
    unsigned long long h = 0;
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    double e[24];
    hipMemcpy(e, ex, sizeof(e), hipMemcpyDeviceToHost);
    printf("mode %d: %llu operands, %llu mismatches\n", mode, (unsigned long long)reps * per, h);
    for (unsigned long long j = 0; j < h && j < 8; ++j) printf("  d=%a div=%a fused=%a\n", e[3 * j], e[3 * j + 1], e[3 * j + 2]);
    fflush(stdout);
  }
  return 0;
}
