// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access patterns of k_render_fast
// (MI355X_MICROARCH.md §HBM: only 16-byte-per-lane streaming accesses are calibrated).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/traffic_calib tools/traffic_calib.hip
//   rocprofv3 --pmc WRITE_SIZE -- tools/traffic_calib      (and a separate --pmc FETCH_SIZE run)
//
// Each kernel moves a known byte count (printed); compare with the counter per dispatch:
//   k_tile_f32   the render kernel's frame write: 256-thread blocks of 2x2 waves, each wave an 8x8
//                pixel tile, one 4-byte nontemporal store per lane and colour plane, 1920x1080 x 3
//                planes = 24,883,200 bytes
//   k_stream16   16 bytes per lane, consecutive lanes consecutive (the guide's calibrated case), same
//                byte count
//   k_read_f64   8-byte loads per lane of a 24,883,200-byte buffer (summed into one word per block)
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int W = 1920, H = 1080;

__global__ __launch_bounds__(256) void k_tile_f32(float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 16 + (w % 2) * 8 + (lane % 8);
  const int row = blockIdx.y * 16 + (w / 2) * 8 + (lane / 8);
  if (col >= W || row >= H) return;
  const long long i = (long long)row * W + col, n = (long long)W * H;
  __builtin_nontemporal_store(1.0f, out + i);
  __builtin_nontemporal_store(2.0f, out + n + i);
  __builtin_nontemporal_store(3.0f, out + 2 * n + i);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream16(u32x4* out, long long n16) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(u32x4{1u, 2u, 3u, 4u}, out + i);
}

__global__ __launch_bounds__(256) void k_read_f64(const double* in, long long n, double* sink) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  double v = i < n ? in[i] : 0.0;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0 && v == 12345.678) sink[0] = v;  // never true: keeps the loads alive
}

int main() {
  const long long bytes = 3LL * W * H * 4;
  void *a = nullptr, *b = nullptr, *s = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&s, 64) != hipSuccess) {
    fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  (void)hipMemset(b, 0, bytes);
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(k_tile_f32, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, 0, (float*)a);
    hipLaunchKernelGGL(k_stream16, dim3((unsigned)((bytes / 16 + 255) / 256)), dim3(256), 0, 0, (u32x4*)a,
                       bytes / 16);
    hipLaunchKernelGGL(k_read_f64, dim3((unsigned)((bytes / 8 + 255) / 256)), dim3(256), 0, 0, (const double*)b,
                       bytes / 8, (double*)s);
  }
  if (hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "kernel failed\n");
    return 1;
  }
  printf("bytes per dispatch: k_tile_f32 writes %lld, k_stream16 writes %lld, k_read_f64 reads %lld\n", bytes, bytes,
         bytes);
  return 0;
}
