// Cross-stream fence for the communicator (parallel/comm.py RcclComm._enter): the comm stream
// waits for the work the caller's stream has enqueued so far. torch's Stream.wait_stream records
// an event created without hipEventDisableSystemFence, so every record on the COMPUTE stream —
// once per gradient bucket in the DDP backward — ends in a system-scope release. This fence
// records a pooled event created with hipEventDisableTiming | hipEventDisableSystemFence: only
// the comm stream on the same device consumes it (RCCL's kernels read the bucket on this
// device; their own transfers do their own fencing), so a device-scope release is enough.
// The wait is enqueued right after the record, so an event can be reused once the ring wraps.
// Opt-in (FLUXMPI_NATIVE_FENCE=1): measured no gain over wait_stream (rd3zd).
#include <hip/hip_runtime.h>

#include <array>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>

#include "../api.h"

namespace fluxmpi {
namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("stream_fence: ") + what + ": " + hipGetErrorString(e));
}

constexpr int kRing = 64;

struct Ring {
  std::array<hipEvent_t, kRing> ev{};
  int next = 0;
};

std::mutex g_mu;
std::map<int, Ring> g_rings;

}  // namespace

void stream_fence(hipStream_t src, hipStream_t dst) {
  int dev = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  hipEvent_t e;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    Ring& r = g_rings[dev];
    hipEvent_t& slot = r.ev[r.next];
    if (slot == nullptr)
      check(hipEventCreateWithFlags(&slot, hipEventDisableTiming | hipEventDisableSystemFence), "hipEventCreateWithFlags");
    e = slot;
    r.next = (r.next + 1) % kRing;
  }
  check(hipEventRecord(e, src), "hipEventRecord");
  check(hipStreamWaitEvent(dst, e, 0), "hipStreamWaitEvent");
}

}  // namespace fluxmpi
