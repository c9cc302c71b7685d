// In-kernel BatchNorm finalize for the reduction kernels (batchnorm.hip; opt-in FLUXMPI_BN_FIN=1,
// measured slower than the finalize kernels — see fin_in_kernel there).
//
// A producer adds per-channel partial sums into one of kShards shards of the [kShards][2][C]
// fp32 workspace with global float atomics. The finalize — sum the shards, derive mean / invstd
// (forward) or copy the two reductions (backward), update the running statistics, re-zero the
// shards — used to be a separate ~5 us kernel on the critical path after every producer (98 per
// ResNet-50 step). Here the producer's LAST workgroup to finish does it: every workgroup waits
// for its own shard atomics to complete, then counts itself in on an arrival counter that lives
// behind the shards; the one that sees the final count (after an acquire) finalizes and resets.
// Row-reduction kernels use one counter (all their workgroups cover all channels).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fluxmpi {
namespace bnfin {

constexpr int kShards = 64;
constexpr int kMaxC = 2048;
// unsigned arrival counter behind the shards (kept zero between uses)
constexpr size_t kCntOff = static_cast<size_t>(kShards) * 2 * kMaxC;

struct Fin {
  int mode;  // 0: none (a finalize kernel follows); 1: forward statistics; 2: backward reductions
  int64_t rows;
  float momentum, eps;
  float* smean;  // mode 1 outputs
  float* sinv;
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float* dw;  // mode 2 outputs (dw = sum(dy_eff * xhat), db = sum(dy_eff)); dw2/db2: dual
  float* db;
  float* dw2;
  float* db2;
};

__device__ __forceinline__ void fwd_channel(const Fin& f, int c, float s, float q) {
  const float inv_n = 1.f / static_cast<float>(f.rows);
  const float mean = s * inv_n;
  float var = q * inv_n - mean * mean;
  var = var > 0.f ? var : 0.f;
  f.smean[c] = mean;
  f.sinv[c] = rsqrtf(var + f.eps);
  if (f.rmean != nullptr) {
    const float unbiased = f.rows > 1 ? var * static_cast<float>(f.rows) / static_cast<float>(f.rows - 1) : var;
    f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * mean;
    f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * unbiased;
  }
}

// Call from EVERY thread of the workgroup after its shard atomics; true in the last of
// `expected` arrivals. This thread's atomics are complete (acknowledged) before the workgroup
// counts itself in. NOT __threadfence() for that: on gfx950 an agent-scope release is
// buffer_wbl2 (a write-back of the XCD's L2) — executed by every workgroup it made the reduction
// kernels ~50 us slower each (rd3o: 11.0k vs 12.5k img/s). The shard updates are atomics, so only
// their completion has to be ordered before the counter's; the "memory" clobber keeps the
// compiler from moving them across. The acquire (one __threadfence in the last workgroup only)
// leaves no stale shard line in its XCD's caches.
__device__ __forceinline__ bool arrive_last(unsigned* cnt, unsigned expected) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(cnt, 1u) == expected - 1u ? 1u : 0u;
  __syncthreads();
  if (s_last == 0u) return false;
  __threadfence();
  return true;
}

}  // namespace bnfin

}  // namespace fluxmpi
