// TEST INFRASTRUCTURE, not product code.  A stand-in for the nine RCCL entry
// points pt_api.cpp's rccl_api() resolves (loaded through PT_RCCL_LIB), so
// pt_dist_run's N > 1 schedule -- the grouped ncclSend/ncclRecv of every
// frame, the per-rank send slots, the root's receive sets and its fused
// assembly -- runs with several processes on ONE GPU.  Real RCCL refuses two
// ranks on one device; this library moves the same bytes point to point:
//   - ncclGetUniqueId names a POSIX shared-memory rendezvous;
//   - ncclCommInitRank maps it and waits until every rank has joined;
//   - a send publishes a hipIpc handle of its buffer's allocation (plus the
//     offset and size) in the (sender, receiver) mailbox after its stream has
//     drained (the data is final), then waits for the receiver's ack -- the
//     buffer is the caller's again only once it has been read, as with RCCL;
//   - a receive waits for the matching post, copies device to device out of
//     the opened handle on its stream, drains that stream, and acks.
// Calls inside ncclGroupStart/End are queued and run at GroupEnd: every send
// is posted before any receive or ack wait, so no grouping deadlocks.
// Everything is host-synchronous: the stand-in checks the schedule's data
// path (offsets, sizes, buffer sets, assembly), not RCCL's overlap.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

constexpr int kMaxRanks = 16;
constexpr double kTimeoutS = 60.0;

struct Mailbox {
  std::atomic<uint64_t> posted;   // sends posted (sequence number of the last)
  std::atomic<uint64_t> acked;    // receives completed
  hipIpcMemHandle_t handle;
  uint64_t offset;
  uint64_t bytes;
};

struct Shared {
  std::atomic<int> joined;
  Mailbox box[kMaxRanks][kMaxRanks];   // [sender][receiver]
};

struct Op {
  bool send;
  void* buf;
  size_t bytes;
  int peer;
  hipStream_t stream;
};

thread_local int g_group = 0;
thread_local std::vector<std::pair<ncclComm_t, Op>> g_ops;

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

bool wait_until(const std::atomic<uint64_t>& a, uint64_t want) {
  const auto t0 = std::chrono::steady_clock::now();
  while (a.load(std::memory_order_acquire) < want) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kTimeoutS) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  return true;
}

}  // namespace

struct ncclComm {
  int nranks = 0, rank = 0;
  std::string name;
  Shared* sh = nullptr;
  uint64_t sent[kMaxRanks] = {};   // sequence numbers per peer
  uint64_t recvd[kMaxRanks] = {};
};

namespace {

ncclResult_t run_op(ncclComm_t c, const Op& op, bool phase_post) {
  if (op.peer < 0 || op.peer >= c->nranks || op.peer == c->rank) return ncclInvalidArgument;
  Mailbox& out = c->sh->box[c->rank][op.peer];
  Mailbox& in = c->sh->box[op.peer][c->rank];
  if (op.send && phase_post) {
    if (hipStreamSynchronize(op.stream) != hipSuccess) return ncclUnhandledCudaError;
    void* base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, op.buf) != hipSuccess) return ncclInvalidArgument;
    if (hipIpcGetMemHandle(&out.handle, base) != hipSuccess) return ncclUnhandledCudaError;
    out.offset = (uint64_t)((char*)op.buf - (char*)base);
    out.bytes = op.bytes;
    out.posted.store(++c->sent[op.peer], std::memory_order_release);
    return ncclSuccess;
  }
  if (op.send) {   // completion: the receiver has read the buffer
    return wait_until(out.acked, c->sent[op.peer]) ? ncclSuccess : ncclSystemError;
  }
  const uint64_t seq = ++c->recvd[op.peer];
  if (!wait_until(in.posted, seq)) return ncclSystemError;
  if (in.bytes != op.bytes) {
    fprintf(stderr, "dist_shim: rank %d receives %zu B from rank %d, which sent %llu B\n", c->rank, op.bytes,
            op.peer, (unsigned long long)in.bytes);
    return ncclInvalidUsage;
  }
  // opened, read and closed per receive: a sender may free and reallocate
  // its buffers between frames (pt_dist_run resizes them with the layout)
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, in.handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return ncclUnhandledCudaError;
  const bool ok = hipMemcpyAsync(op.buf, (char*)p + in.offset, op.bytes, hipMemcpyDeviceToDevice, op.stream) ==
                      hipSuccess &&
                  hipStreamSynchronize(op.stream) == hipSuccess;
  (void)hipIpcCloseMemHandle(p);
  if (!ok) return ncclUnhandledCudaError;
  in.acked.store(seq, std::memory_order_release);
  return ncclSuccess;
}

ncclResult_t run_ops(std::vector<std::pair<ncclComm_t, Op>>& ops) {
  ncclResult_t r = ncclSuccess;
  for (auto& o : ops)   // post every send first
    if (r == ncclSuccess && o.second.send) r = run_op(o.first, o.second, true);
  for (auto& o : ops)
    if (r == ncclSuccess && !o.second.send) r = run_op(o.first, o.second, false);
  for (auto& o : ops)
    if (r == ncclSuccess && o.second.send) r = run_op(o.first, o.second, false);
  ops.clear();
  return r;
}

ncclResult_t enqueue(ncclComm_t c, bool send, void* buf, size_t count, ncclDataType_t t, int peer, hipStream_t s) {
  if (!c || !buf || !type_size(t)) return ncclInvalidArgument;
  g_ops.push_back({c, Op{send, buf, count * type_size(t), peer, s}});
  return g_group ? ncclSuccess : run_ops(g_ops);
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  memset(id, 0, sizeof *id);
  const long long ns = std::chrono::steady_clock::now().time_since_epoch().count();
  snprintf((char*)id, sizeof *id, "/ptshim-%d-%lld", (int)getpid(), ns);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  ncclComm* c = new ncclComm();
  c->nranks = nranks;
  c->rank = rank;
  c->name.assign((const char*)&id, strnlen((const char*)&id, sizeof id));
  const int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, sizeof(Shared)) != 0) {
    if (fd >= 0) close(fd);
    delete c;
    return ncclSystemError;
  }
  void* p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    delete c;
    return ncclSystemError;
  }
  c->sh = (Shared*)p;   // a new file reads as zeros: every counter starts at 0
  c->sh->joined.fetch_add(1, std::memory_order_acq_rel);
  const auto t0 = std::chrono::steady_clock::now();
  while (c->sh->joined.load(std::memory_order_acquire) < nranks) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kTimeoutS) {
      munmap(p, sizeof(Shared));
      shm_unlink(c->name.c_str());
      delete c;
      return ncclSystemError;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  if (c->sh) munmap(c->sh, sizeof(Shared));
  shm_unlink(c->name.c_str());   // every rank mapped it before any returned from init
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) { return ncclCommDestroy(c); }

ncclResult_t ncclGroupStart() {
  ++g_group;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (g_group <= 0) return ncclInvalidUsage;
  return --g_group ? ncclSuccess : run_ops(g_ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  return enqueue(c, true, const_cast<void*>(buf), count, t, peer, s);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  return enqueue(c, false, buf, count, t, peer, s);
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "success (dist_shim)";
    case ncclUnhandledCudaError: return "HIP call failed (dist_shim)";
    case ncclSystemError: return "timeout or shared-memory failure (dist_shim)";
    case ncclInvalidArgument: return "invalid argument (dist_shim)";
    case ncclInvalidUsage: return "invalid usage (dist_shim)";
    default: return "error (dist_shim)";
  }
}

}  // extern "C"
