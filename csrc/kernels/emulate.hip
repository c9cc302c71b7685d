// Communication-load emulator (a measurement tool, never on a production path) — gfx950.
//
// At world size 1 RCCL runs no kernels, so a one-GPU box cannot show how the collectives'
// workgroups interfere with the compute kernels they overlap during backward. This kernel
// stands in for them: `blocks` workgroups that hold their CU slots for a fixed wall time
// (the constant-rate wall clock, so the duration does not depend on the shader clock),
// launched on the communicator's stream where the allreduce would run. Bounded: every
// wave exits after `ticks` of the wall clock (the host caps the duration at 100 ms).
#include <stdexcept>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

__global__ __launch_bounds__(512) void spin_kernel(int64_t ticks) {
  extern __shared__ float lds_hold[];  // dynamic LDS: the footprint a collective's workgroup holds
  const int64_t t0 = static_cast<int64_t>(wall_clock64());
  while (static_cast<int64_t>(wall_clock64()) - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0 && ticks < 0) lds_hold[0] = 0.f;  // keeps the allocation live; never true
}

}  // namespace

void emulate_comm(int blocks, double microseconds, hipStream_t stream, int threads, int lds_bytes) {
  if (blocks < 1 || blocks > 4096) throw std::runtime_error("emulate_comm: 1 <= blocks <= 4096");
  if (threads < 64 || threads > 512 || threads % 64) throw std::runtime_error("emulate_comm: threads in 64..512");
  if (lds_bytes < 0 || lds_bytes > 64 * 1024) throw std::runtime_error("emulate_comm: lds_bytes <= 64 KiB");
  if (!(microseconds > 0.0) || microseconds > 100000.0) throw std::runtime_error("emulate_comm: 0 < us <= 100000");
  static int khz = 0;
  if (khz == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  }
  const int64_t ticks = static_cast<int64_t>(microseconds * khz / 1000.0);
  spin_kernel<<<blocks, threads, static_cast<size_t>(lds_bytes), stream>>>(ticks);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
