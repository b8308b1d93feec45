// rtx_tiles.hip — the row-tiled multi-GPU frame driven natively (the north star's
// "framebuffer row-tiles across the GPUs of one node with an RCCL gather over xGMI"). The reference
// renders a frame in one process (render_image_pipeline, application.py:43-52); here every rank
// renders its interleaved row tile (rtx_render_camera_ex), the root receives the peers' tiles over
// RCCL point-to-point (one ncclRecv per peer inside one group: each peer's bytes arrive over its own
// xGMI link at once, where a ring would be bound by one link) and un-permutes the rows on the device
// (rtx_assemble_rows). One call per frame and rank submits all of it — no Python between the render,
// the collective and the assembly (distributed.TileGather drives it).
//
// Streams: the render runs on the caller's stream; the collective and the assembly on the plan's
// own stream, after an event, so frame k's gather runs while frame k+1 renders (two slots). A slot's
// buffers are reused only after its previous frame's gather and assembly have completed (event).
//
// RCCL is the process's own librccl (the one torch loaded: the same library instance must create
// and drive a communicator), resolved at run time with dlopen/dlsym; <rccl/rccl.h> supplies types
// only. The library has no link-time RCCL dependency, so the single-GPU entry points load without it.
// Host code only: no kernels in this unit.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "../../include/rtx_hip.h"

// rtx_kernels.hip: the library's thread-local error message
__attribute__((visibility("hidden"))) int rtx_set_error(int code, const char* msg);

namespace {

struct Rccl {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommInitRankConfig) comm_init_rank_config = nullptr;  // optional (max_ctas)
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};
Rccl g_rccl;
std::mutex g_rccl_mu;

int err(int code, const char* fmt, const char* a = "", long long b = 0) {
  char m[512];
  snprintf(m, sizeof(m), fmt, a, b);
  return rtx_set_error(code, m);
}

int nccl_err(const char* what, ncclResult_t r) {
  char m[512];
  snprintf(m, sizeof(m), "%s: %s", what, g_rccl.error_string ? g_rccl.error_string(r) : "RCCL error");
  return rtx_set_error(RTX_E_COMM, m);
}

bool rccl_ready() { return g_rccl.send != nullptr; }

template <typename F>
bool sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g_rccl.lib, name));
  return f != nullptr;
}

// A row-tiled frame plan: one rank's view of the frame (its tile, the communicator, the slots'
// buffers and events). Buffers are caller-owned device memory registered once.
struct Tiles {
  ncclComm_t comm;
  int world, rank, root;
  int width, height, row_block, out_kind;
  int root_run, run;  // rank 0 renders parts [0, root_run), rank i parts [root_run + (i-1) run, + run)
  int n_parts, first, my_run;  // the interleave (root_run + (world - 1) run parts) and this rank's run
  int slots;
  int64_t part_bytes;
  int local_rows;
  int device;
  bool loop;  // RTX_TILES_LOOPBACK: a one-rank plan whose tile still goes through RCCL (send to itself)
  bool rows;  // RTX_TILES_ROWS: each row block travels on its own and lands in the frame (no assembly)
  bool timed;  // RTX_TILES_TIMED: timing events around each slot's gather and assembly (rtx_tiles_timing)
  unsigned reserve;  // RTX_F_RESERVE bits passed to every render (plans that gather)
  hipStream_t cs;  // collective + assembly stream
  void* send[RTX_TILES_MAX_SLOTS];
  void* recv[RTX_TILES_MAX_SLOTS];
  hipEvent_t rendered[RTX_TILES_MAX_SLOTS];
  hipEvent_t done[RTX_TILES_MAX_SLOTS];
  // RTX_TILES_TIMED, on the plan's stream: g0 when the gather may start (this rank's tile rendered,
  // the slot's previous frame gone), g1 when the group's transfers are complete, a1 after the
  // root's assembly (or the root's own row blocks under RTX_TILES_ROWS)
  hipEvent_t g0[RTX_TILES_MAX_SLOTS], g1[RTX_TILES_MAX_SLOTS], a1[RTX_TILES_MAX_SLOTS];
  bool used[RTX_TILES_MAX_SLOTS];
};

int local_rows(int height, int row_block, int n_parts, int p, int run = 1) {  // tiling.n_local_rows
  const int cycle = row_block * n_parts, own = row_block * run;
  const int q = height / cycle, rem = height % cycle - p * row_block;
  return q * own + (rem < 0 ? 0 : rem > own ? own : rem);
}

int64_t bytes_per_pixel(int kind) { return kind == RTX_OUT_F32_SOA ? 12 : kind == RTX_OUT_F64_SOA ? 24 : 3; }

// RTX_TILES_ROWS: the gather moves every row block of a part on its own, straight into its rows of
// the root's frame (a uint8 row block is contiguous there), so the root never assembles: per peer,
// one ncclSend per block of its tile (local rows in order), and at the root one ncclRecv per block
// into frame row ((j * P + p) * rb); the root's own blocks are one strided device copy. Sends and
// receives between a pair match in order. On the plan's stream after the render; records done.
int gather_rows(Tiles* t, int slot, bool root, uint8_t* frame) {
  const int P = t->world, rb = t->row_block;
  const int64_t rowb = (int64_t)t->width * 3;
  ncclResult_t r = g_rccl.group_start();
  if (r != ncclSuccess) return nccl_err("ncclGroupStart", r);
  const bool sender = t->loop || !root;
  const int dest = t->loop ? 0 : t->root;
  if (sender) {
    const int n = local_rows(t->height, rb, P, t->rank);
    for (int j = 0; j * rb < n && r == ncclSuccess; ++j) {
      const int rows = n - j * rb < rb ? n - j * rb : rb;
      r = g_rccl.send((const uint8_t*)t->send[slot] + (int64_t)j * rb * rowb, (size_t)(rows * rowb), ncclUint8, dest,
                      t->comm, t->cs);
    }
  }
  if (root) {
    for (int p = 0; p < P && r == ncclSuccess; ++p) {
      if (p == t->root && !t->loop) continue;
      const int n = local_rows(t->height, rb, P, p);
      for (int j = 0; j * rb < n && r == ncclSuccess; ++j) {
        const int rows = n - j * rb < rb ? n - j * rb : rb;
        r = g_rccl.recv(frame + (int64_t)(j * P + p) * rb * rowb, (size_t)(rows * rowb), ncclUint8, p, t->comm, t->cs);
      }
    }
  }
  const ncclResult_t r2 = g_rccl.group_end();
  if (r != ncclSuccess) return nccl_err(root ? "ncclRecv" : "ncclSend", r);
  if (r2 != ncclSuccess) return nccl_err("ncclGroupEnd", r2);
  hipError_t e = t->timed ? hipEventRecord(t->g1[slot], t->cs) : hipSuccess;
  if (e == hipSuccess && root && !t->loop) {  // the root's own blocks: rows (j P + root) rb .. + rb of the frame
    const int n = t->local_rows, full = n / rb, tail = n % rb;
    const uint8_t* own = (const uint8_t*)t->recv[slot];
    uint8_t* dst0 = frame + (int64_t)t->root * rb * rowb;
    if (full > 0)
      e = hipMemcpy2DAsync(dst0, (size_t)(P * rb * rowb), own, (size_t)(rb * rowb), (size_t)(rb * rowb), (size_t)full,
                           hipMemcpyDeviceToDevice, t->cs);
    if (e == hipSuccess && tail > 0)
      e = hipMemcpyAsync(dst0 + (int64_t)full * P * rb * rowb, own + (int64_t)full * rb * rowb, (size_t)(tail * rowb),
                         hipMemcpyDeviceToDevice, t->cs);
  }
  if (e == hipSuccess && t->timed) e = hipEventRecord(t->a1[slot], t->cs);
  if (e == hipSuccess) e = hipEventRecord(t->done[slot], t->cs);
  if (e != hipSuccess) return err(RTX_E_LAUNCH, "gather_rows: %s", hipGetErrorString(e));
  return RTX_OK;
}

}  // namespace

extern "C" {

int rtx_rccl_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (rccl_ready()) return RTX_OK;
  // the library torch (or the caller) already loaded, if any: RTLD_NOLOAD returns its handle
  void* h = dlopen(path && *path ? path : "librccl.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen(path && *path ? path : "librccl.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char* why = dlerror();
    return err(RTX_E_COMM, "cannot load RCCL (%s)", why ? why : "dlopen failed");
  }
  g_rccl = Rccl{};
  g_rccl.lib = h;
  bool ok = sym(g_rccl.get_unique_id, "ncclGetUniqueId") && sym(g_rccl.comm_init_rank, "ncclCommInitRank") &&
            sym(g_rccl.comm_destroy, "ncclCommDestroy") && sym(g_rccl.recv, "ncclRecv") &&
            sym(g_rccl.group_start, "ncclGroupStart") && sym(g_rccl.group_end, "ncclGroupEnd") &&
            sym(g_rccl.error_string, "ncclGetErrorString") && sym(g_rccl.send, "ncclSend");
  if (!ok) {
    g_rccl = Rccl{};
    return err(RTX_E_COMM, "RCCL library lacks a required symbol%s", "");
  }
  sym(g_rccl.comm_init_rank_config, "ncclCommInitRankConfig");
  return RTX_OK;
}

int rtx_comm_unique_id(void* id_out) {
  if (!id_out) return err(RTX_E_ARG, "null pointer argument%s", "");
  if (!rccl_ready()) return err(RTX_E_COMM, "RCCL not loaded (rtx_rccl_load)%s", "");
  ncclUniqueId id;
  if (ncclResult_t r = g_rccl.get_unique_id(&id)) return nccl_err("ncclGetUniqueId", r);
  memcpy(id_out, &id, sizeof(id));
  return RTX_OK;
}

int rtx_comm_init(const void* id, int world, int rank, int max_ctas, void** comm_out) {
  if (!id || !comm_out) return err(RTX_E_ARG, "null pointer argument%s", "");
  if (world < 1 || rank < 0 || rank >= world) return err(RTX_E_ARG, "bad world/rank%s (%lld)", "", world);
  if (!rccl_ready()) return err(RTX_E_COMM, "RCCL not loaded (rtx_rccl_load)%s", "");
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  if (max_ctas > 0) {  // cap the CTAs (blocks) of the communicator's kernels: the gather runs beside a render
    if (!g_rccl.comm_init_rank_config) return err(RTX_E_COMM, "RCCL lacks ncclCommInitRankConfig%s", "");
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.minCTAs = 1;
    cfg.maxCTAs = max_ctas;
    if (ncclResult_t r = g_rccl.comm_init_rank_config(&c, world, uid, rank, &cfg))
      return nccl_err("ncclCommInitRankConfig", r);
  } else if (ncclResult_t r = g_rccl.comm_init_rank(&c, world, uid, rank)) {
    return nccl_err("ncclCommInitRank", r);
  }
  *comm_out = c;
  return RTX_OK;
}

int rtx_comm_destroy(void* comm) {
  if (!comm) return RTX_OK;
  if (!rccl_ready()) return err(RTX_E_COMM, "RCCL not loaded%s", "");
  if (ncclResult_t r = g_rccl.comm_destroy((ncclComm_t)comm)) return nccl_err("ncclCommDestroy", r);
  return RTX_OK;
}

int rtx_tiles_create(void* comm, int world, int rank, int root, int width, int height, int row_block, int out_kind,
                     int slots, void* const* send, void* const* recv, int64_t part_bytes, int root_run, int run,
                     unsigned flags, void** plan_out) {
  if (!plan_out) return err(RTX_E_ARG, "null plan pointer%s", "");
  *plan_out = nullptr;
  if (world < 1 || rank < 0 || rank >= world || root < 0 || root >= world)
    return err(RTX_E_ARG, "bad world/rank/root%s (%lld)", "", world);
  if (width <= 0 || height <= 0 || row_block <= 0) return err(RTX_E_ARG, "bad frame/tile geometry%s", "");
  if (out_kind < 0 || out_kind > 2) return err(RTX_E_ARG, "bad out_kind%s %lld", "", out_kind);
  if (slots < 1 || slots > RTX_TILES_MAX_SLOTS) return err(RTX_E_ARG, "bad slot count%s (%lld)", "", slots);
  if (flags & ~(unsigned)(RTX_TILES_LOOPBACK | RTX_TILES_ROWS | RTX_TILES_TIMED | RTX_F_RESERVE(0xFFF)))
    return err(RTX_E_ARG, "unknown flags%s (%lld)", "", (long long)flags);
  const bool loop = world == 1 && (flags & RTX_TILES_LOOPBACK);
  const bool rows = (flags & RTX_TILES_ROWS) && (world > 1 || loop);
  if (rows && out_kind != RTX_OUT_U8_HWC)
    return err(RTX_E_ARG, "RTX_TILES_ROWS needs uint8 frames (a row block is contiguous there)%s", "");
  if ((world > 1 || loop) && (!comm || !rccl_ready()))
    return err(RTX_E_COMM, "world > 1 (or a loopback plan) needs an RCCL communicator%s", "");
  if (root_run < 1 || run < 1 || (world == 1 && (root_run != 1 || run != 1)) || (root != 0 && root_run != run))
    return err(RTX_E_ARG, "bad runs%s (root_run %lld)", "", root_run);
  if (rows && (root_run != 1 || run != 1)) return err(RTX_E_ARG, "RTX_TILES_ROWS needs runs of one part%s", "");
  const int np = root_run + (world - 1) * run;
  int rows_max = 0;  // the longest run's tile
  for (int r = 0; r < world; ++r) {
    const int n = r == 0 ? local_rows(height, row_block, np, 0, root_run)
                         : local_rows(height, row_block, np, root_run + (r - 1) * run, run);
    rows_max = n > rows_max ? n : rows_max;
  }
  if (part_bytes < rows_max * (int64_t)width * bytes_per_pixel(out_kind) || part_bytes % 16 != 0)
    return err(RTX_E_ARG, "part_bytes must hold the longest share's tile and be a multiple of 16%s (%lld)", "", part_bytes);
  for (int s = 0; s < slots; ++s) {
    if (rank == root && (world > 1 || loop) && (!recv || !recv[s]))
      return err(RTX_E_ARG, "the root needs a receive buffer per slot%s", "");
    if ((rank != root || loop) && (!send || !send[s]))
      return err(RTX_E_ARG, "a peer (or a loopback plan) needs a send buffer per slot%s", "");
  }
  Tiles* t = new Tiles{};
  t->comm = (ncclComm_t)comm;
  t->world = world;
  t->rank = rank;
  t->root = root;
  t->width = width;
  t->height = height;
  t->row_block = row_block;
  t->out_kind = out_kind;
  t->slots = slots;
  t->part_bytes = part_bytes;
  t->root_run = root_run;
  t->run = run;
  t->n_parts = np;
  // uniform runs (root_run == run) keep rank order whatever the root; otherwise the root is rank 0
  t->first = rank == 0 ? 0 : root_run + (rank - 1) * run;
  t->my_run = rank == 0 ? root_run : run;
  t->local_rows = local_rows(height, row_block, np, t->first, t->my_run);
  t->loop = loop;
  t->rows = rows;
  t->timed = (flags & RTX_TILES_TIMED) && (world > 1 || loop);
  t->reserve = (world > 1 || loop) ? (flags & RTX_F_RESERVE(0xFFF)) : 0u;
  (void)hipGetDevice(&t->device);
  hipError_t e = hipStreamCreateWithFlags(&t->cs, hipStreamNonBlocking);
  for (int s = 0; s < slots && e == hipSuccess; ++s) {
    t->send[s] = send ? send[s] : nullptr;
    t->recv[s] = recv ? recv[s] : nullptr;
    e = hipEventCreateWithFlags(&t->rendered[s], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->done[s], hipEventDisableTiming);
    if (t->timed) {
      if (e == hipSuccess) e = hipEventCreate(&t->g0[s]);
      if (e == hipSuccess) e = hipEventCreate(&t->g1[s]);
      if (e == hipSuccess) e = hipEventCreate(&t->a1[s]);
    }
  }
  if (e != hipSuccess) {
    rtx_tiles_destroy(t);
    return err(RTX_E_LAUNCH, "rtx_tiles_create: %s", hipGetErrorString(e));
  }
  *plan_out = t;
  return RTX_OK;
}

int rtx_tiles_submit(void* plan, int slot, const double* scene, int n_spheres, int max_bounces, void* workspace,
                     size_t workspace_bytes, unsigned flags, uint32_t* deferred_out, const uint32_t* tile_order,
                     uint32_t* tile_cost, void* frame, void* stream) {
  Tiles* t = (Tiles*)plan;
  if (!t) return err(RTX_E_ARG, "null plan%s", "");
  if (slot < 0 || slot >= t->slots) return err(RTX_E_ARG, "bad slot%s (%lld)", "", slot);
  hipStream_t s = (hipStream_t)stream;
  const bool root = t->rank == t->root;
  if (root && !frame) return err(RTX_E_ARG, "the root needs a frame buffer%s", "");
  // a one-rank plan without loopback renders straight into the caller's frame on the caller's
  // stream: stream order is all the ordering it needs (no event: each costs the stream a barrier)
  const bool single = t->world == 1 && !t->loop;
  // the slot's buffers are free once its previous frame's gather and assembly have run
  if (t->used[slot] && !single) {
    if (hipError_t e = hipStreamWaitEvent(s, t->done[slot], 0))
      return err(RTX_E_LAUNCH, "hipStreamWaitEvent: %s", hipGetErrorString(e));
  }
  t->used[slot] = true;
  // a single part IS the frame (local rows = global rows): render straight into it
  void* dst = t->loop        ? t->send[slot]
              : t->world == 1 ? frame
              : root          ? (uint8_t*)t->recv[slot] + (t->rows ? 0 : (int64_t)t->root * t->part_bytes)
                              : t->send[slot];
  if (int rc = rtx_render_camera_sched(scene, n_spheres, t->width, t->height, t->row_block, t->n_parts, t->first,
                                       t->my_run, t->local_rows, max_bounces, dst, t->out_kind, workspace, workspace_bytes,
                                       nullptr, stream, flags | t->reserve, deferred_out, tile_order, tile_cost))
    return rc;
  if (single) return RTX_OK;
  hipError_t e = hipEventRecord(t->rendered[slot], s);
  if (e == hipSuccess) e = hipStreamWaitEvent(t->cs, t->rendered[slot], 0);
  if (e == hipSuccess && t->timed) e = hipEventRecord(t->g0[slot], t->cs);
  if (e != hipSuccess) return err(RTX_E_LAUNCH, "event: %s", hipGetErrorString(e));
  if (t->rows) return gather_rows(t, slot, root, (uint8_t*)frame);
  if (ncclResult_t r = g_rccl.group_start()) return nccl_err("ncclGroupStart", r);
  ncclResult_t r = ncclSuccess;
  if (t->loop) {
    r = g_rccl.send(t->send[slot], (size_t)t->part_bytes, ncclUint8, 0, t->comm, t->cs);
    if (r == ncclSuccess) r = g_rccl.recv(t->recv[slot], (size_t)t->part_bytes, ncclUint8, 0, t->comm, t->cs);
  } else if (root) {
    for (int p = 0; p < t->world && r == ncclSuccess; ++p) {
      if (p == t->root) continue;
      r = g_rccl.recv((uint8_t*)t->recv[slot] + (int64_t)p * t->part_bytes, (size_t)t->part_bytes, ncclUint8, p, t->comm,
                      t->cs);
    }
  } else {
    r = g_rccl.send(t->send[slot], (size_t)t->part_bytes, ncclUint8, t->root, t->comm, t->cs);
  }
  const ncclResult_t r2 = g_rccl.group_end();
  if (r != ncclSuccess) return nccl_err(root ? "ncclRecv" : "ncclSend", r);
  if (r2 != ncclSuccess) return nccl_err("ncclGroupEnd", r2);
  if (t->timed && (e = hipEventRecord(t->g1[slot], t->cs)))
    return err(RTX_E_LAUNCH, "hipEventRecord: %s", hipGetErrorString(e));
  if (root) {
    if (int rc = rtx_assemble_runs(t->recv[slot], t->part_bytes, t->world, t->root_run, t->run, t->width, t->height,
                                   t->row_block, t->out_kind, frame, t->cs))
      return rc;
  }
  if (t->timed && (e = hipEventRecord(t->a1[slot], t->cs)))
    return err(RTX_E_LAUNCH, "hipEventRecord: %s", hipGetErrorString(e));
  if ((e = hipEventRecord(t->done[slot], t->cs))) return err(RTX_E_LAUNCH, "hipEventRecord: %s", hipGetErrorString(e));
  return RTX_OK;
}

int rtx_tiles_timing(void* plan, int slot, float* gather_ms, float* assemble_ms) {
  Tiles* t = (Tiles*)plan;
  if (!t || !gather_ms || !assemble_ms) return err(RTX_E_ARG, "null argument%s", "");
  if (slot < 0 || slot >= t->slots) return err(RTX_E_ARG, "bad slot%s (%lld)", "", slot);
  if (!t->timed) return err(RTX_E_ARG, "the plan was not created with RTX_TILES_TIMED (or does not gather)%s", "");
  if (!t->used[slot]) return err(RTX_E_ARG, "slot%s %lld has carried no frame", "", slot);
  hipError_t e = hipEventSynchronize(t->a1[slot]);
  if (e == hipSuccess) e = hipEventElapsedTime(gather_ms, t->g0[slot], t->g1[slot]);
  if (e == hipSuccess) e = hipEventElapsedTime(assemble_ms, t->g1[slot], t->a1[slot]);
  if (e != hipSuccess) return err(RTX_E_LAUNCH, "rtx_tiles_timing: %s", hipGetErrorString(e));
  return RTX_OK;
}

int rtx_tiles_finish(void* plan, int slot, void* stream) {
  Tiles* t = (Tiles*)plan;
  if (!t) return err(RTX_E_ARG, "null plan%s", "");
  if (slot < 0 || slot >= t->slots) return err(RTX_E_ARG, "bad slot%s (%lld)", "", slot);
  if (!t->used[slot] || (t->world == 1 && !t->loop)) return RTX_OK;  // direct: in stream order already
  if (hipError_t e = hipStreamWaitEvent((hipStream_t)stream, t->done[slot], 0))
    return err(RTX_E_LAUNCH, "hipStreamWaitEvent: %s", hipGetErrorString(e));
  return RTX_OK;
}

int rtx_tiles_destroy(void* plan) {
  Tiles* t = (Tiles*)plan;
  if (!t) return RTX_OK;
  // the plan's stream may still run a gather: let it finish before its events go
  if (t->cs) (void)hipStreamSynchronize(t->cs);
  for (int s = 0; s < t->slots; ++s) {
    if (t->rendered[s]) (void)hipEventDestroy(t->rendered[s]);
    if (t->done[s]) (void)hipEventDestroy(t->done[s]);
    for (hipEvent_t ev : {t->g0[s], t->g1[s], t->a1[s]})
      if (ev) (void)hipEventDestroy(ev);
  }
  if (t->cs) (void)hipStreamDestroy(t->cs);
  delete t;
  return RTX_OK;
}

}  // extern "C"
