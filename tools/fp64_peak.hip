// fp64_peak.hip — measures the MI355X float64 vector rate this kernel family can reach, to anchor
// the roofline "peak" of bench.py (datasheet: 78.6 TFLOP/s FP64 vector = 2 flops per FMA).
// Build: hipcc --offload-arch=gfx950 -O3 -o fp64_peak tools/fp64_peak.hip
// Runs: FMA chains (v_fma_f64) and, separately, non-fused mul+add pairs (what -ffp-contract=off
// code issues), 8 independent chains per lane, 2048 blocks x 256 threads.
#include <hip/hip_runtime.h>

#include <cstdio>

template <bool FUSED>
__global__ __launch_bounds__(256) void k_peak(double* out, double a, double b, int iters) {
  double x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3 + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (FUSED) {
        x[j] = __builtin_fma(x[j], a, b);
      } else {
        x[j] = x[j] * a;
        asm volatile("" : "+v"(x[j]));
        x[j] = x[j] + b;
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j];
  if (s == 12345.678) out[0] = s;  // keep live
}

int main() {
  double* d;
  hipMalloc(&d, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 2048 * 4, threads = 256, iters = 4096;
  for (int fused = 1; fused >= 0; --fused) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (fused)
        hipLaunchKernelGGL(k_peak<true>, dim3(blocks), dim3(threads), 0, 0, d, 0.999999, 1e-7, iters);
      else
        hipLaunchKernelGGL(k_peak<false>, dim3(blocks), dim3(threads), 0, 0, d, 0.999999, 1e-7, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double ops = (double)blocks * threads * iters * 8 * 2;  // 2 flops per fma or per mul+add pair
      printf("%s rep %d: %.3f ms  %.2f TFLOP/s\n", fused ? "fma    " : "mul+add", rep, ms, ops / (ms * 1e-3) / 1e12);
    }
  }
  hipFree(d);
  return 0;
}
