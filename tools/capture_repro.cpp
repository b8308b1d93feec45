// capture_repro.cpp — minimal reproducer for the round-5 crash (session r5a): a loopback RCCL
// send/receive pair captured into a HIP graph, the way rtx_tiles_submit/finish enqueue it
// (python_ray_tracer_amd/csrc/rtx_tiles.hip). No torch, no renderer: one process, one GPU, a one-rank
// communicator over the librccl given on the command line (torch's own, as in the crash).
//
//   hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -o tools/capture_repro tools/capture_repro.cpp -ldl
//   tools/capture_repro VARIANT LIBRCCL [BYTES]        (BYTES: the transfer's size, default 1 MiB)
//
// VARIANT (each step is printed before it runs, so a crash names its call):
//   memcpy  fork/join of a side stream by events inside the capture, a device copy on it (no RCCL)
//   plain   ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd on the capturing stream itself
//   fork    the same group on a side stream forked from the capturing stream by an event and joined
//           back by another (rtx_tiles_submit + rtx_tiles_finish)
//   stale   fork, plus, first, a wait of the capturing stream on an event recorded before the capture
//           began (a reused slot's `done` event: rtx_tiles_submit's first call)
//   kbefore fork, plus a kernel on the capturing stream before the fork (the render)
//   kafter  fork, plus a kernel on the side stream after the RCCL group (the root's assembly)
//   kboth   both kernels: the whole shape of rtx_tiles_submit + rtx_tiles_finish
//   extk    kboth, the kernel before the fork launched by hipExtLaunchKernelGGL (null events), as
//           the library launches k_render_fast
//   samevent  kboth; the capture begins with a wait on the join event as recorded before the capture
//           (the eager frame's), and the join records and waits that same event again: rtx_tiles_submit's
//           `done` event of a reused slot
//   nulleager  eager, with the eager frame on the null stream (torch's default current stream)
//   eager   kboth, and before the capture one eager frame of the same shape (fork to the side stream
//           by an event, RCCL, join back by another), as TileGather's first, eager submit does
#include <dlfcn.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// a stand-in for the render (before the fork) and the assembly (after the RCCL group): one pass over
// the buffer
__global__ void touch(unsigned char* p, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i];
}

#define STEP(what, call)                                                \
  do {                                                                  \
    printf("step: %s\n", what);                                         \
    fflush(stdout);                                                     \
    const int rc_ = (int)(call);                                        \
    printf("  -> %d\n", rc_);                                           \
    fflush(stdout);                                                     \
    if (rc_) {                                                          \
      printf("FAILED at %s\n", what);                                   \
      return 2;                                                         \
    }                                                                   \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s memcpy|plain|fork|stale|kbefore|kafter|kboth LIBRCCL\n", argv[0]);
    return 1;
  }
  const char* v = argv[1];
  void* lib = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
  if (!lib) {
    printf("dlopen: %s\n", dlerror());
    return 1;
  }
  auto get_id = (decltype(&ncclGetUniqueId))dlsym(lib, "ncclGetUniqueId");
  auto init = (decltype(&ncclCommInitRank))dlsym(lib, "ncclCommInitRank");
  auto destroy = (decltype(&ncclCommDestroy))dlsym(lib, "ncclCommDestroy");
  auto gstart = (decltype(&ncclGroupStart))dlsym(lib, "ncclGroupStart");
  auto gend = (decltype(&ncclGroupEnd))dlsym(lib, "ncclGroupEnd");
  auto send = (decltype(&ncclSend))dlsym(lib, "ncclSend");
  auto recv = (decltype(&ncclRecv))dlsym(lib, "ncclRecv");
  const size_t n = argc > 3 ? (size_t)strtoull(argv[3], nullptr, 10) : (size_t)1 << 20;
  printf("transfer of %zu bytes\n", n);
  std::vector<unsigned char> host(n), back(n);
  for (size_t i = 0; i < n; ++i) host[i] = (unsigned char)(i * 131 + 7);
  void *sb = nullptr, *rb = nullptr;
  hipStream_t s, cs;
  hipEvent_t fork_ev, join_ev, stale_ev;
  ncclUniqueId id;
  ncclComm_t comm = nullptr;
  STEP("hipSetDevice", hipSetDevice(0));
  STEP("hipMalloc", hipMalloc(&sb, n));
  STEP("hipMalloc", hipMalloc(&rb, n));
  STEP("hipMemcpy H2D", hipMemcpy(sb, host.data(), n, hipMemcpyHostToDevice));
  STEP("hipStreamCreate", hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  STEP("hipStreamCreate (side)", hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  STEP("hipEventCreate", hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
  STEP("hipEventCreate", hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
  STEP("hipEventCreate", hipEventCreateWithFlags(&stale_ev, hipEventDisableTiming));
  STEP("ncclGetUniqueId", get_id(&id));
  STEP("ncclCommInitRank (world 1)", init(&comm, 1, id, 0));
  // eager first, like the renderer's first frame (RCCL's own lazy set-up happens here)
  const bool nulleager = !strcmp(v, "nulleager");
  hipStream_t es = nulleager ? nullptr : s;  // the eager frame's stream
  if (!strcmp(v, "eager") || nulleager) {  // the eager frame's fork and join, outside any capture
    STEP("eager fork: record on s", hipEventRecord(fork_ev, es));
    STEP("eager fork: side stream waits", hipStreamWaitEvent(cs, fork_ev, 0));
  }
  STEP("eager ncclGroupStart", gstart());
  STEP("eager ncclSend", send(sb, n, ncclUint8, 0, comm, cs));
  STEP("eager ncclRecv", recv(rb, n, ncclUint8, 0, comm, cs));
  STEP("eager ncclGroupEnd", gend());
  STEP("eager stale event record", hipEventRecord(stale_ev, cs));
  if (!strcmp(v, "eager") || nulleager) STEP("eager join: s waits", hipStreamWaitEvent(es, stale_ev, 0));
  STEP("eager sync", hipStreamSynchronize(cs));
  STEP("hipMemset", hipMemset(rb, 0, n));
  STEP("hipDeviceSynchronize", hipDeviceSynchronize());

  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  if (!strcmp(v, "samevent")) {
    STEP("eager: record the join event on the side stream", hipEventRecord(join_ev, cs));
    STEP("eager: sync", hipStreamSynchronize(cs));
  }
  STEP("hipStreamBeginCapture (global)", hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  if (!strcmp(v, "stale")) STEP("wait on the pre-capture event", hipStreamWaitEvent(s, stale_ev, 0));
  const bool same = !strcmp(v, "samevent");
  if (same) STEP("wait on the join event as recorded before the capture", hipStreamWaitEvent(s, join_ev, 0));
  if (!strcmp(v, "plain")) {
    STEP("ncclGroupStart", gstart());
    STEP("ncclSend (capturing stream)", send(sb, n, ncclUint8, 0, comm, s));
    STEP("ncclRecv (capturing stream)", recv(rb, n, ncclUint8, 0, comm, s));
    STEP("ncclGroupEnd", gend());
  } else {
    const bool ext = !strcmp(v, "extk");
    const bool eg = !strcmp(v, "eager") || nulleager;
    const bool kb = !strcmp(v, "kbefore") || !strcmp(v, "kboth") || ext || eg || same;
    const bool ka = !strcmp(v, "kafter") || !strcmp(v, "kboth") || ext || eg || same;
    if (kb) {
      printf("step: kernel on the capturing stream%s\n", ext ? " (hipExtLaunchKernelGGL)" : "");
      fflush(stdout);
      if (ext) {
        hipExtLaunchKernelGGL(touch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nullptr, nullptr, 0u,
                              (unsigned char*)sb, n);
      } else {
        hipLaunchKernelGGL(touch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (unsigned char*)sb, n);
      }
      STEP("hipGetLastError", hipGetLastError());
    }
    STEP("fork: record on the capturing stream", hipEventRecord(fork_ev, s));
    STEP("fork: side stream waits", hipStreamWaitEvent(cs, fork_ev, 0));
    if (!strcmp(v, "memcpy")) {
      STEP("hipMemcpyAsync (side stream)", hipMemcpyAsync(rb, sb, n, hipMemcpyDeviceToDevice, cs));
    } else {
      STEP("ncclGroupStart", gstart());
      STEP("ncclSend (side stream)", send(sb, n, ncclUint8, 0, comm, cs));
      STEP("ncclRecv (side stream)", recv(rb, n, ncclUint8, 0, comm, cs));
      STEP("ncclGroupEnd", gend());
    }
    if (ka) {
      printf("step: kernel on the side stream after the group\n");
      fflush(stdout);
      hipLaunchKernelGGL(touch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, cs, (unsigned char*)rb, n);
      STEP("hipGetLastError", hipGetLastError());
    }
    STEP("join: record on the side stream", hipEventRecord(join_ev, cs));
    STEP("join: capturing stream waits", hipStreamWaitEvent(s, join_ev, 0));
  }
  STEP("hipStreamEndCapture", hipStreamEndCapture(s, &g));
  size_t nodes = 0;
  STEP("hipGraphGetNodes", hipGraphGetNodes(g, nullptr, &nodes));
  printf("graph nodes: %zu\n", nodes);
  STEP("hipGraphInstantiate", hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int k = 0; k < 2; ++k) {
    STEP("hipMemsetAsync", hipMemsetAsync(rb, 0, n, s));  // (on s: the graph's stream is non-blocking)
    STEP("hipGraphLaunch", hipGraphLaunch(ge, s));
    STEP("hipStreamSynchronize", hipStreamSynchronize(s));
    STEP("hipMemcpy D2H", hipMemcpy(back.data(), rb, n, hipMemcpyDeviceToHost));
    const bool ok = !memcmp(back.data(), host.data(), n);
    printf("replay %d: %s\n", k, ok ? "received bytes equal" : "MISMATCH");
    if (!ok) return 3;
  }
  STEP("hipGraphExecDestroy", hipGraphExecDestroy(ge));
  STEP("hipGraphDestroy", hipGraphDestroy(g));
  STEP("ncclCommDestroy", destroy(comm));
  printf("variant %s: ok\n", v);
  return 0;
}
