// Issue rate of f64 VALU ops on one MI355X: 8 independent chains per lane, many waves.
// hipcc --offload-arch=gfx950 -O3 tools/trans_rate.hip -o tools/trans_rate && tools/trans_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void k(double* out, double seed, int iters) {
  double v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = seed + threadIdx.x * 1e-3 + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) v[j] = __builtin_amdgcn_rcp(v[j]);
      if (OP == 1) v[j] = __builtin_amdgcn_rsq(v[j]);
      if (OP == 2) v[j] = v[j] + 1.0000001;
      if (OP == 3) v[j] = __builtin_fma(v[j], 0.999999, 1e-9);
      if (OP == 4) v[j] = __builtin_fmax(v[j], 0.5);
    }
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += v[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
double run(const char* name, double* d, int blocks, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1.5, iters);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1.5, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double insts = (double)blocks * 4 * iters * 8;  // wave instructions
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
  const double simd_cycles = ms * 1e-3 * clk * 1e3;
  printf("%-10s %8.3f ms  %.2f cycles per wave-instruction per SIMD (%d CUs, %.0f MHz)\n", name, ms,
         simd_cycles * cus * 4 / insts, cus, clk / 1e3);
  return ms;
}

int main() {
  double* d;
  const int blocks = 256 * 8 * 4;
  (void)hipMalloc(&d, (size_t)blocks * 256 * sizeof(double));
  const int iters = 2000;
  run<2>("v_add_f64", d, blocks, iters);
  run<3>("v_fma_f64", d, blocks, iters);
  run<4>("v_max_f64", d, blocks, iters);
  run<0>("v_rcp_f64", d, blocks, iters);
  run<1>("v_rsq_f64", d, blocks, iters);
  (void)hipFree(d);
  return 0;
}
