#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

struct ncclComm;  // rccl.h's opaque communicator (ncclComm_t), kept out of this header

namespace fluxmpi {

std::string rccl_unique_id();
int rccl_version();

// Thin owner of an ncclComm_t; all operations are stream-ordered and async.
//
// Thread safety: the training thread enqueues collectives while the watchdog
// thread polls async_error() and may abort(). Every use of comm_ holds mu_, so
// abort/destroy can never free the communicator under a running enqueue. An
// enqueue that does not return (a wedged launch queue) must not make the
// watchdog hang as well: abort() waits at most `abort_wait_ms` for the lock and
// then aborts regardless (ncclCommAbort is the documented way to unblock a
// communicator from another thread). Once aborted, every call throws
// "communicator aborted" instead of touching a freed handle.
class RcclComm {
 public:
  RcclComm(const std::string& uid, int rank, int size, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  void allreduce(uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, uintptr_t stream);
  void allreduce_many(const std::vector<uintptr_t>& bufs, const std::vector<size_t>& counts,
                      const std::vector<int>& dtypes, int op, uintptr_t stream);
  void broadcast(uintptr_t send, uintptr_t recv, size_t count, int dtype, int root, uintptr_t stream);
  void reduce(uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, int root, uintptr_t stream);
  void allgather(uintptr_t send, uintptr_t recv, size_t sendcount, int dtype, uintptr_t stream);
  void reduce_scatter(uintptr_t send, uintptr_t recv, size_t recvcount, int dtype, int op, uintptr_t stream);
  void alltoall(uintptr_t send, uintptr_t recv, size_t count_per_peer, int dtype, uintptr_t stream);
  // what the communicator itself reports (ncclCommCount / ncclCommUserRank / ncclCommCuDevice):
  // bench.py checks them against WORLD_SIZE / RANK / the pinned device before timing
  int comm_count();
  int comm_user_rank();
  int comm_device();
  int async_error();
  static std::string error_string(int code);
  void abort(int abort_wait_ms = 2000);
  void destroy();
  bool aborted() const { return aborted_.load(); }
  bool is_open() const { return comm_.load() != nullptr; }

  int rank() const { return rank_; }
  int size() const { return size_; }
  int device() const { return device_; }

 private:
  // the handle, read once per call under mu_ (abort() may clear it without the lock)
  ::ncclComm* open_comm() const;
  void check_not_aborted() const;
  static size_t dtype_size(int dtype);
  std::timed_mutex mu_;
  std::atomic<bool> aborted_{false};
  std::atomic<void*> comm_{nullptr};
  int rank_, size_, device_;
};

}  // namespace fluxmpi
