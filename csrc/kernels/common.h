// Shared helpers for the fluxmpi_amd CDNA4 (gfx950) kernels.
//
// Memory-bound multi-tensor kernels follow the MI355X playbook:
//  * 64-lane wavefronts, 256-thread workgroups (4 waves, one per SIMD),
//  * 16-byte per-lane vector accesses (global_load_dwordx4) on every dtype
//    (bf16/fp16 are never loaded as scalars: hipcc does not auto-vectorise them),
//  * one workgroup per fixed-size chunk of one tensor, the chunk->tensor map is
//    a prefix table in the kernel arguments (no device-side metadata, so a
//    launch is HIP-graph capturable and needs no H2D copy per call),
//  * grids of thousands of workgroups for the 256 CUs / 8 XCDs.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>

namespace fluxmpi {

// dtype codes == ncclDataType_t values
enum DType : int { kI8 = 0, kU8 = 1, kI32 = 2, kI64 = 4, kF16 = 6, kF32 = 7, kF64 = 8, kBF16 = 9 };

using bf16 = __bf16;
using f16 = _Float16;

template <typename T> struct Acc { using type = float; };
template <> struct Acc<double> { using type = double; };

template <typename T> __device__ __forceinline__ float to_f(T x) { return static_cast<float>(x); }
template <typename T> __device__ __forceinline__ T from_f(float x) { return static_cast<T>(x); }

// 8 elements per lane: 16 B for 2-byte types, 2 x 16 B for fp32, 4 x 16 B for fp64.
template <typename T> struct Vec8 {
  T v[8];
};

template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ p, T (&out)[8]) {
  constexpr int kBytes = 8 * sizeof(T);
  static_assert(kBytes % 16 == 0, "vector width");
  constexpr int kN = kBytes / 16;
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 tmp[kN];
#pragma unroll
  for (int i = 0; i < kN; ++i) tmp[i] = q[i];
  __builtin_memcpy(out, tmp, kBytes);
}

template <typename T>
__device__ __forceinline__ void store8(T* __restrict__ p, const T (&in)[8]) {
  constexpr int kBytes = 8 * sizeof(T);
  constexpr int kN = kBytes / 16;
  uint4 tmp[kN];
  __builtin_memcpy(tmp, in, kBytes);
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < kN; ++i) q[i] = tmp[i];
}

__device__ __forceinline__ bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// Binary search: largest t with start[t] <= b (start has n+1 entries, start[0] == 0).
template <int N>
__device__ __forceinline__ int find_tensor(const int32_t (&start)[N], int n, int b) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

}  // namespace fluxmpi

// Workgroups of `threads` lanes (with `smem` bytes of dynamic LDS) that one dispatch of
// `kernel` keeps resident on the current device: occupancy x CUs. Grid-stride kernels
// launched with exactly this many workgroups run as one full round — no partial last
// round of workgroups (a 2048-block grid on a 7-block/CU kernel is 1.14 rounds: the
// 0.14 tail costs as much as a whole round).
// Rounds of resident workgroups a "persistent" grid is sized to (FLUXMPI_GRID_ROUNDS, default 1).
// With several rounds, a kernel sharing the chip with others (RCCL's workgroups during the
// backward/allreduce overlap) ends with a partial round instead of waiting a whole extra one
// for the slots the other kernel holds.
inline int grid_rounds() {
  static int r = [] {
    const char* e = std::getenv("FLUXMPI_GRID_ROUNDS");
    const int v = e != nullptr ? std::atoi(e) : 1;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  return r;
}

inline int resident_blocks(const void* kernel, int threads, size_t smem) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, size_t, int>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const auto key = std::make_tuple(kernel, threads, smem, dev);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, smem) != hipSuccess || per_cu < 1)
    per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  const int n = per_cu * cus * grid_rounds();
  cache.emplace(key, n);
  return n;
}

#define FLUXMPI_HIP_CHECK(expr)                                                        \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") +        \
                                                   hipGetErrorString(_e) + " at " #expr); \
  } while (0)
