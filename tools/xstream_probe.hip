// What does a second kernel per frame cost, and would a side-stream poller be cheaper?
//   hipcc --offload-arch=gfx950 -O3 -o tools/xstream_probe tools/xstream_probe.hip && tools/xstream_probe
// Per iteration, on stream A, a "frame" kernel busy for ~70 us on every CU, then:
//   mode 0: nothing else                                   (the floor)
//   mode 1: a tiny kernel on A (k_render_general's place)
//   mode 3/4: the frame kernel uses scratch (alone / + the tiny kernel)
//   mode 5/6: the frame kernel writes a 25 MB frame with nontemporal stores (alone / + tiny)
//   mode 2: a tiny kernel on side stream B that spins until the frame kernel's blocks have all
//           finished (non-returning atomics), A waits for B's event (the poller design); B first
//           waits for an event recorded on A before the frame kernel (graph-capture shape)
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_busy(unsigned long long ticks, unsigned* done) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (done && threadIdx.x == 0) atomicAdd(done, 1u);
}

// the same, with a private array the compiler must place in scratch (like the render kernel's spills)
__global__ __launch_bounds__(256) void k_busy_scratch(unsigned long long ticks, unsigned* w) {
  volatile double a[32];
  for (int i = 0; i < 32; ++i) a[i] = i * 1.5 + threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (a[(threadIdx.x + w[2]) & 31] == -1.0) w[3] = 1;
}

// a frame-like write: every lane stores 12 bytes of a 25 MB frame (nontemporal), then ends
__global__ __launch_bounds__(256) void k_busy_write(unsigned long long ticks, float* out, long long n) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    __builtin_nontemporal_store(1.0f, out + i);
    __builtin_nontemporal_store(2.0f, out + n + i);
    __builtin_nontemporal_store(3.0f, out + 2 * n + i);
  }
}

__global__ void k_tiny(unsigned* w) {
  if (threadIdx.x == 0 && w[0] == 0xFFFFFFFFu) w[1] = 1;
}

__global__ void k_poll(unsigned* done, unsigned target) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) break;  // 5 s: never expected
    }
    done[0] = 0;
  }
}

int main() {
  hipStream_t A, B;
  (void)hipStreamCreateWithFlags(&A, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&B, hipStreamNonBlocking);
  unsigned* w;
  (void)hipMalloc(&w, 256);
  (void)hipMemset(w, 0, 256);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const unsigned blocks = (unsigned)cus * 4;
  hipEvent_t e0, e1, ea[64], eb[64];
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 64; ++i) {
    (void)hipEventCreateWithFlags(&ea[i], hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&eb[i], hipEventDisableTiming);
  }
  const int N = 200;
  float* frame;
  const long long npx = 1920LL * 1080;
  (void)hipMalloc(&frame, npx * 12);
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 7; ++mode) {
      (void)hipStreamSynchronize(A);
      (void)hipEventRecord(e0, A);
      for (int i = 0; i < N; ++i) {
        if (mode == 2) {
          (void)hipEventRecord(ea[i % 64], A);
          (void)hipStreamWaitEvent(B, ea[i % 64], 0);
          hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, A, 7000ull, w + 8);
          hipLaunchKernelGGL(k_poll, dim3(1), dim3(64), 0, B, w + 8, blocks);
          (void)hipEventRecord(eb[i % 64], B);
          (void)hipStreamWaitEvent(A, eb[i % 64], 0);
        } else if (mode <= 1) {
          hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, A, 7000ull, (unsigned*)nullptr);
          if (mode == 1) hipLaunchKernelGGL(k_tiny, dim3(64), dim3(64), 0, A, w);
        } else if (mode <= 4) {  // 3: scratch frame kernel alone, 4: + tiny kernel
          hipLaunchKernelGGL(k_busy_scratch, dim3(blocks), dim3(256), 0, A, 7000ull, w);
          if (mode == 4) hipLaunchKernelGGL(k_tiny, dim3(64), dim3(64), 0, A, w);
        } else {  // 5: frame-writing kernel alone, 6: + tiny kernel
          hipLaunchKernelGGL(k_busy_write, dim3(blocks), dim3(256), 0, A, 7000ull, frame, npx);
          if (mode == 6) hipLaunchKernelGGL(k_tiny, dim3(64), dim3(64), 0, A, w);
        }
      }
      (void)hipEventRecord(e1, A);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("rep %d mode %d: %.2f us per frame\n", rep, mode, ms * 1e3 / N);
    }
  }
  return 0;
}
