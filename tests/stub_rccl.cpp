// stub_rccl.cpp — TEST-ONLY stand-in for librccl, so that the native row-tiled frame's world > 1
// code (csrc/rtx_tiles.hip: the root's per-peer ncclRecv into recv + p * part_bytes while it renders
// its own share, the peers' ncclSend, rtx_assemble_runs over unequal shares, gather_rows) runs on the
// one-GPU box: every rank of the frame lives in ONE process, each on its own host thread and HIP
// stream of the same device, and rtx_rccl_load(path-of-this-library) binds the render library to it.
//
// Semantics kept from RCCL point-to-point (what rtx_tiles relies on):
//  * sends and receives between a pair of ranks match in posting order (the k-th ncclSend from a to b
//    with the k-th ncclRecv at b from a), the byte counts must agree (else ncclInvalidUsage);
//  * the operations of a ncclGroupStart/End group are posted together, so a group that sends to and
//    receives from itself (the loopback plan) or a root posting one receive per peer cannot deadlock;
//  * stream order: the copy runs on the RECEIVER's stream after an event recorded on the sender's
//    stream when it posted (the sender's buffer is complete in its stream order then), and the
//    sender's stream waits for the copy before anything it enqueues later (its buffer may be reused).
// Where RCCL would rendezvous on the device, ncclGroupEnd here waits on the host until every operation
// of its group has met its partner (a condition variable, with a time limit: an unmatched operation
// returns ncclInternalError instead of hanging). Ranks therefore must run on separate host threads.
//
// Every operation is logged (comm, kind, rank, peer, bytes, buffer address, group, order) for the tests
// to check what rtx_tiles asked for (tests/test_rccl_stub.py, tests/test_gpu_tiles_stub.py). In "dry"
// mode (stub_rccl_set_dry) no HIP call is made and matched buffers are copied on the host: the CPU test
// drives the matching logic with host buffers. Never part of the product: nothing under
// python_ray_tracer_amd/ loads it (distributed.rccl_comm binds torch's librccl).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

struct ncclComm {
  int id, world, rank, device;
};

namespace {

constexpr uint32_t kMagic = 0x53545542u;  // "STUB"

struct Op {
  int comm, kind;  // kind 0: send, 1: recv
  int src, dst;    // the pair (sender, receiver)
  void* buf;
  size_t bytes;
  hipStream_t stream;
  hipEvent_t posted = nullptr;  // sends: recorded on the sender's stream when posted
  long long seq = 0;            // order of this operation among the pair's operations of its kind
  bool matched = false;
  int err = 0;
};

struct Rec {  // one logged operation
  long long comm, kind, rank, peer, bytes, ptr, group, seq;
};

std::mutex mu;
std::condition_variable cv;
std::vector<Op*> pending;  // posted, not yet matched
std::vector<Rec> log_recs;
std::map<std::tuple<int, int, int, int>, long long> seqs;  // (comm, kind, src, dst) -> next seq
std::map<std::tuple<int, int>, long long> groups;          // (comm, rank) -> groups posted
int next_id = 1;
int dry = 0;
int timeout_ms = 60000;
thread_local int depth = 0;
thread_local std::vector<Op*> group_ops;

size_t type_bytes(ncclDataType_t t) {
  switch (t) {
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    case ncclFloat16: case ncclBfloat16: return 2;
    default: return 1;
  }
}

// the partner of a send (recv) is the recv (send) of the same pair and order
Op* partner(const Op* o) {
  for (Op* q : pending)
    if (q != o && !q->matched && q->comm == o->comm && q->kind != o->kind && q->src == o->src && q->dst == o->dst &&
        q->seq == o->seq)
      return q;
  return nullptr;
}

// called with mu held: move the bytes of a matched pair, in stream order
void transfer(Op* s, Op* r) {
  s->matched = r->matched = true;
  if (s->bytes != r->bytes) {
    s->err = r->err = ncclInvalidUsage;
    return;
  }
  if (dry) {
    if (s->bytes && s->buf && r->buf) memcpy(r->buf, s->buf, s->bytes);
    return;
  }
  hipError_t e = hipStreamWaitEvent(r->stream, s->posted, 0);
  if (e == hipSuccess && s->bytes) e = hipMemcpyAsync(r->buf, s->buf, s->bytes, hipMemcpyDeviceToDevice, r->stream);
  hipEvent_t done = nullptr;
  if (e == hipSuccess) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(done, r->stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(s->stream, done, 0);
  if (done) (void)hipEventDestroy(done);  // released once it has completed
  if (e != hipSuccess) s->err = r->err = ncclUnhandledCudaError;
}

ncclResult_t post_group(std::vector<Op*>& ops) {
  std::unique_lock<std::mutex> lk(mu);
  ncclResult_t rc = ncclSuccess;
  if (ops.empty()) return rc;
  // the group's index among this rank's groups (a group holds one rank's operations)
  const long long g = groups[std::make_tuple(ops[0]->comm, ops[0]->kind == 0 ? ops[0]->src : ops[0]->dst)]++;
  for (Op* o : ops) {
    const int rank = o->kind == 0 ? o->src : o->dst, peer = o->kind == 0 ? o->dst : o->src;
    o->seq = seqs[std::make_tuple(o->comm, o->kind, o->src, o->dst)]++;
    log_recs.push_back(Rec{o->comm, o->kind, rank, peer, (long long)o->bytes, (long long)(uintptr_t)o->buf, g, o->seq});
    if (o->kind == 0 && !dry) {
      if (hipEventCreateWithFlags(&o->posted, hipEventDisableTiming) != hipSuccess ||
          hipEventRecord(o->posted, o->stream) != hipSuccess)
        rc = ncclUnhandledCudaError;
    }
    pending.push_back(o);
    if (Op* q = partner(o)) transfer(o->kind == 0 ? o : q, o->kind == 0 ? q : o);
  }
  cv.notify_all();
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  const bool all = cv.wait_until(lk, deadline, [&] {
    for (Op* o : ops)
      if (!o->matched) return false;
    return true;
  });
  // leave the table: this group's operations are done (matched) or abandoned (timed out)
  std::vector<Op*> keep;
  for (Op* q : pending) {
    bool mine = false;
    for (Op* o : ops) mine = mine || q == o;
    if (!mine) keep.push_back(q);
  }
  pending.swap(keep);
  if (!all) rc = ncclInternalError;
  for (Op* o : ops) {
    if (o->err && rc == ncclSuccess) rc = (ncclResult_t)o->err;
    // a send's posted event may still be waited on by its partner's stream: destroying a recorded
    // event is fine (HIP releases it when the work completes)
    if (o->posted) (void)hipEventDestroy(o->posted);
    delete o;
  }
  ops.clear();
  return rc;
}

ncclResult_t enqueue(int kind, void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                     hipStream_t stream) {
  if (!comm) return ncclInvalidArgument;
  if (peer < 0 || peer >= comm->world) return ncclInvalidArgument;
  Op* o = new Op{};
  o->comm = comm->id;
  o->kind = kind;
  o->src = kind == 0 ? comm->rank : peer;
  o->dst = kind == 0 ? peer : comm->rank;
  o->buf = buf;
  o->bytes = count * type_bytes(type);
  o->stream = stream;
  group_ops.push_back(o);
  if (depth == 0) return post_group(group_ops);  // outside a group: a group of one
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(mu);
  memset(id, 0, sizeof(*id));
  const uint32_t w[2] = {kMagic, (uint32_t)next_id++};
  memcpy(id->internal, w, sizeof(w));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  uint32_t w[2];
  memcpy(w, id.internal, sizeof(w));
  if (!comm || w[0] != kMagic || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  int dev = 0;
  if (!dry) (void)hipGetDevice(&dev);
  *comm = new ncclComm{(int)w[1], nranks, rank, dev};
  return ncclSuccess;
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank, ncclConfig_t*) {
  return ncclCommInitRank(comm, nranks, id, rank);
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (stub)";
    case ncclInvalidArgument: return "invalid argument (stub)";
    case ncclInvalidUsage: return "invalid usage: send and receive sizes differ (stub)";
    case ncclInternalError: return "unmatched send/recv: timed out waiting for the partner (stub)";
    default: return "error (stub)";
  }
}

ncclResult_t ncclGroupStart() {
  ++depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (depth <= 0) return ncclInvalidUsage;
  if (--depth > 0) return ncclSuccess;
  return post_group(group_ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  return enqueue(0, const_cast<void*>(buf), count, type, peer, comm, stream);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream) {
  return enqueue(1, buf, count, type, peer, comm, stream);
}

// ---- test hooks ----
void stub_rccl_set_dry(int on) { dry = on; }
void stub_rccl_set_timeout_ms(int ms) { timeout_ms = ms; }
void stub_rccl_reset() {
  std::lock_guard<std::mutex> lk(mu);
  log_recs.clear();
  seqs.clear();
  groups.clear();
}
// up to cap records of 8 int64 each (comm, kind 0 send / 1 recv, rank, peer, bytes, buffer address,
// the rank's group index, order within the pair); returns the number logged
int stub_rccl_log(long long* out, int cap) {
  std::lock_guard<std::mutex> lk(mu);
  const int n = (int)log_recs.size();
  for (int i = 0; i < n && i < cap; ++i) memcpy(out + 8 * i, &log_recs[i], sizeof(Rec));
  return n;
}
int stub_rccl_pending() {
  std::lock_guard<std::mutex> lk(mu);
  return (int)pending.size();
}

}  // extern "C"
