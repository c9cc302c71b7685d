// Native RCCL communicator (the C++ replacement of the reference's raw
// `ccall((:MPI_Iallreduce, MPI.libmpi), ...)` / `MPI_Ibcast` bindings,
// src/mpi_extensions.jl:26-88).
//
// One ncclComm_t per process group, bootstrapped from an ncclUniqueId that
// rank 0 creates and the Python layer distributes through the process-group
// TCP store. Every call is asynchronous with respect to the host and ordered
// on the caller-provided HIP stream (a dedicated high-priority comm stream
// in practice); completion is tracked by HIP events on the Python side.
//
// We link against the librccl.so that PyTorch already loaded (same SONAME),
// so a process never carries two RCCL runtimes, and use only the stable core
// API (init/destroy/abort/async-error, AllReduce/Broadcast/Reduce/AllGather/
// ReduceScatter/Send/Recv, group calls).
#include "rccl_comm.h"

#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

namespace fluxmpi {

#define RCCL_CHECK(expr)                                                                        \
  do {                                                                                          \
    ncclResult_t _r = (expr);                                                                   \
    if (_r != ncclSuccess && _r != ncclInProgress)                                              \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " (" #expr \
                               ")");                                                            \
  } while (0)

static inline ncclComm_t C(void* p) { return reinterpret_cast<ncclComm_t>(p); }

std::string rccl_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int rccl_version() {
  int v = 0;
  RCCL_CHECK(ncclGetVersion(&v));
  return v;
}

RcclComm::RcclComm(const std::string& uid, int rank, int size, int device)
    : rank_(rank), size_(size), device_(device) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclComm: bad unique id size");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("RcclComm: hipSetDevice failed");
  ncclComm_t comm = nullptr;
  RCCL_CHECK(ncclCommInitRank(&comm, size, id, rank));
  comm_.store(comm);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
}

RcclComm::~RcclComm() {
  void* c = comm_.exchange(nullptr);
  if (c != nullptr && !aborted_.load()) {
    // Best effort: never throw from a destructor.
    ncclCommDestroy(C(c));
  }
}

ncclComm_t RcclComm::open_comm() const {
  if (aborted_.load()) throw std::runtime_error("RcclComm: communicator aborted (watchdog or explicit abort)");
  void* c = comm_.load();
  if (c == nullptr) throw std::runtime_error("RcclComm: communicator destroyed");
  return C(c);
}

void RcclComm::check_not_aborted() const {
  // abort() may have torn the communicator down while this thread was inside the enqueue
  // (it only waits abort_wait_ms for the lock): report it instead of returning "success"
  if (aborted_.load()) throw std::runtime_error("RcclComm: communicator aborted during the call");
}

using Lock = std::lock_guard<std::timed_mutex>;

void RcclComm::allreduce(uintptr_t send, uintptr_t recv, size_t count, int dtype, int op,
                         uintptr_t stream) {
  Lock lk(mu_);
  ncclComm_t c = open_comm();
  RCCL_CHECK(ncclAllReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                           static_cast<ncclDataType_t>(dtype), static_cast<ncclRedOp_t>(op), c,
                           reinterpret_cast<hipStream_t>(stream)));
  check_not_aborted();
}

void RcclComm::allreduce_many(const std::vector<uintptr_t>& bufs, const std::vector<size_t>& counts,
                              const std::vector<int>& dtypes, int op, uintptr_t stream) {
  Lock lk(mu_);
  ncclComm_t c = open_comm();
  if (bufs.size() != counts.size() || bufs.size() != dtypes.size())
    throw std::runtime_error("allreduce_many: length mismatch");
  RCCL_CHECK(ncclGroupStart());
  for (size_t i = 0; i < bufs.size(); ++i) {
    ncclResult_t r = ncclAllReduce(reinterpret_cast<const void*>(bufs[i]), reinterpret_cast<void*>(bufs[i]),
                                   counts[i], static_cast<ncclDataType_t>(dtypes[i]),
                                   static_cast<ncclRedOp_t>(op), c, reinterpret_cast<hipStream_t>(stream));
    if (r != ncclSuccess && r != ncclInProgress) {
      ncclGroupEnd();
      throw std::runtime_error(std::string("RCCL error in allreduce_many: ") + ncclGetErrorString(r));
    }
  }
  RCCL_CHECK(ncclGroupEnd());
  check_not_aborted();
}

void RcclComm::broadcast(uintptr_t send, uintptr_t recv, size_t count, int dtype, int root,
                         uintptr_t stream) {
  Lock lk(mu_);
  ncclComm_t c = open_comm();
  RCCL_CHECK(ncclBroadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                           static_cast<ncclDataType_t>(dtype), root, c,
                           reinterpret_cast<hipStream_t>(stream)));
  check_not_aborted();
}

void RcclComm::reduce(uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, int root,
                      uintptr_t stream) {
  Lock lk(mu_);
  ncclComm_t c = open_comm();
  RCCL_CHECK(ncclReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                        static_cast<ncclDataType_t>(dtype), static_cast<ncclRedOp_t>(op), root, c,
                        reinterpret_cast<hipStream_t>(stream)));
  check_not_aborted();
}

int RcclComm::comm_count() {
  Lock lk(mu_);
  int n = -1;
  RCCL_CHECK(ncclCommCount(open_comm(), &n));
  return n;
}

int RcclComm::comm_user_rank() {
  Lock lk(mu_);
  int r = -1;
  RCCL_CHECK(ncclCommUserRank(open_comm(), &r));
  return r;
}

int RcclComm::comm_device() {
  Lock lk(mu_);
  int d = -1;
  RCCL_CHECK(ncclCommCuDevice(open_comm(), &d));
  return d;
}

void RcclComm::allgather(uintptr_t send, uintptr_t recv, size_t sendcount, int dtype, uintptr_t stream) {
  Lock lk(mu_);
  ncclComm_t c = open_comm();
  RCCL_CHECK(ncclAllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), sendcount,
                           static_cast<ncclDataType_t>(dtype), c, reinterpret_cast<hipStream_t>(stream)));
  check_not_aborted();
}

void RcclComm::reduce_scatter(uintptr_t send, uintptr_t recv, size_t recvcount, int dtype, int op,
                              uintptr_t stream) {
  Lock lk(mu_);
  ncclComm_t c = open_comm();
  RCCL_CHECK(ncclReduceScatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), recvcount,
                               static_cast<ncclDataType_t>(dtype), static_cast<ncclRedOp_t>(op), c,
                               reinterpret_cast<hipStream_t>(stream)));
  check_not_aborted();
}

void RcclComm::alltoall(uintptr_t send, uintptr_t recv, size_t count_per_peer, int dtype, uintptr_t stream) {
  Lock lk(mu_);
  ncclComm_t c = open_comm();
  // Built from grouped send/recv so it works on every RCCL build.
  const size_t esz = dtype_size(dtype);
  RCCL_CHECK(ncclGroupStart());
  for (int peer = 0; peer < size_; ++peer) {
    const char* s = reinterpret_cast<const char*>(send) + peer * count_per_peer * esz;
    char* r = reinterpret_cast<char*>(recv) + peer * count_per_peer * esz;
    ncclResult_t rs = ncclSend(s, count_per_peer, static_cast<ncclDataType_t>(dtype), peer, c,
                               reinterpret_cast<hipStream_t>(stream));
    ncclResult_t rr = (rs == ncclSuccess || rs == ncclInProgress)
                          ? ncclRecv(r, count_per_peer, static_cast<ncclDataType_t>(dtype), peer, c,
                                     reinterpret_cast<hipStream_t>(stream))
                          : rs;
    if (rr != ncclSuccess && rr != ncclInProgress) {
      ncclGroupEnd();  // close the group before reporting, so the communicator stays usable
      throw std::runtime_error(std::string("RCCL error in alltoall (peer ") + std::to_string(peer) +
                               "): " + ncclGetErrorString(rr));
    }
  }
  RCCL_CHECK(ncclGroupEnd());
  check_not_aborted();
}

int RcclComm::async_error() {
  // Polled from the watchdog thread: never wait behind an enqueue, just skip this poll.
  std::unique_lock<std::timed_mutex> lk(mu_, std::try_to_lock);
  void* c = comm_.load();
  if (!lk.owns_lock() || c == nullptr) return 0;
  ncclResult_t r = ncclSuccess;
  ncclResult_t q = ncclCommGetAsyncError(C(c), &r);
  if (q != ncclSuccess) return static_cast<int>(q);
  return static_cast<int>(r);
}

std::string RcclComm::error_string(int code) { return ncclGetErrorString(static_cast<ncclResult_t>(code)); }

void RcclComm::abort(int abort_wait_ms) {
  aborted_.store(true);  // new enqueues fail fast from here on
  std::unique_lock<std::timed_mutex> lk(mu_, std::defer_lock);
  (void)lk.try_lock_for(std::chrono::milliseconds(abort_wait_ms));
  // exchange: exactly one of abort/destroy/~RcclComm ever owns the handle. If the lock was not
  // obtained, an enqueue on this comm may still be running; ncclCommAbort is NCCL's documented
  // way to unblock exactly that from another thread, and that enqueue then reports "aborted
  // during the call" (check_not_aborted) instead of success.
  void* c = comm_.exchange(nullptr);
  if (c != nullptr) ncclCommAbort(C(c));
}

void RcclComm::destroy() {
  Lock lk(mu_);
  void* c = comm_.exchange(nullptr);
  if (c != nullptr) RCCL_CHECK(ncclCommDestroy(C(c)));
}

size_t RcclComm::dtype_size(int dtype) {
  switch (dtype) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 1;
  }
}

}  // namespace fluxmpi
