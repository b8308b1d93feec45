// Accuracy of the hardware f64 reciprocal / reciprocal square root and of short Newton sequences
// built on them, against the correctly rounded results (the compiler's full expansions).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/approx_probe tools/approx_probe.hip && tools/approx_probe
// Prints the largest error in ulps of the correctly rounded value for random operands over
// [2^-20, 2^20] (the range of the specular's denominators and square-root arguments).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

__global__ void k(const double* x, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double b = x[i];
  double* o = out + (size_t)i * 10;
  o[0] = 1.0 / b;                       // reference: correctly rounded
  o[1] = __builtin_amdgcn_rcp(b);       // hardware rcp
  double r = __builtin_amdgcn_rcp(b);   // one Newton step
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  o[2] = r;
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);  // two steps
  o[3] = r;
  o[4] = __builtin_sqrt(b);             // reference sqrt
  o[5] = __builtin_amdgcn_rsq(b);       // hardware rsq (compare with 1/sqrt)
  // Goldschmidt step + one correction (the library's sqrt_core without its last correction)
  const double y = __builtin_amdgcn_rsq(b);
  double g = b * y, h = y * 0.5;
  const double rr = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, rr, g);
  h = __builtin_fma(h, rr, h);
  o[6] = g;  // after the Goldschmidt step
  const double d = __builtin_fma(-g, g, b);
  o[7] = __builtin_fma(d, h, g);  // + one correction
  o[8] = 1.0 / __builtin_sqrt(b);  // reference 1/sqrt (two roundings, as norm() computes it)
  double z = __builtin_amdgcn_rsq(b);  // rsq + one Newton step
  z = __builtin_fma(z * 0.5, __builtin_fma(-b * z, z, 1.0), z);
  o[9] = z;
}

static double ulps(double got, double want) {
  if (got == want) return 0.0;
  int64_t a, b;
  memcpy(&a, &got, 8);
  memcpy(&b, &want, 8);
  return (double)llabs(a - b);
}

int main() {
  const int n = 1 << 22;
  double* hx = new double[n];
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;  // [0, 1)
    hx[i] = std::exp2(-20.0 + 40.0 * u);
  }
  double *dx, *dout;
  (void)hipMalloc(&dx, n * 8);
  (void)hipMalloc(&dout, (size_t)n * 80);
  (void)hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, n, dout);
  double* ho = new double[(size_t)n * 10];
  (void)hipMemcpy(ho, dout, (size_t)n * 80, hipMemcpyDeviceToHost);
  double m[10] = {0};
  for (int i = 0; i < n; ++i) {
    const double* o = ho + (size_t)i * 10;
    m[1] = fmax(m[1], ulps(o[1], o[0]));
    m[2] = fmax(m[2], ulps(o[2], o[0]));
    m[3] = fmax(m[3], ulps(o[3], o[0]));
    m[5] = fmax(m[5], ulps(o[5], o[8]));
    m[6] = fmax(m[6], ulps(o[6], o[4]));
    m[7] = fmax(m[7], ulps(o[7], o[4]));
    m[9] = fmax(m[9], ulps(o[9], o[8]));
  }
  printf("max ulps over %d operands in [2^-20, 2^20]:\n", n);
  printf("  v_rcp_f64 vs 1/b                  %.0f\n", m[1]);
  printf("  rcp + 1 Newton step               %.0f\n", m[2]);
  printf("  rcp + 2 Newton steps              %.0f\n", m[3]);
  printf("  v_rsq_f64 vs 1/sqrt(b)            %.0f\n", m[5]);
  printf("  sqrt: rsq + Goldschmidt           %.0f\n", m[6]);
  printf("  sqrt: + one correction            %.0f\n", m[7]);
  printf("  1/sqrt: rsq + 1 Newton step       %.0f\n", m[9]);
  return 0;
}
