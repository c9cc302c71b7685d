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

// ---- cross-lane reductions without LDS -------------------------------------------------------
// __shfl_xor compiles to ds_bpermute_b32: an LDS-crossbar round trip per step, on the critical
// path of every reduction. gfx950 has VALU cross-lane moves instead: DPP within 16-lane rows
// (fused into the add as v_add_f32_dpp), v_permlane16_swap / v_permlane32_swap across rows and
// halves, v_readlane to scalars.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// v[lane ^ 32] and v[lane ^ 16] as the two halves of a permlane swap of v with itself:
// {r0, r1} hold {v, partner} in some order on every lane (measured on MI355X:
// scripts/probe_lanes.hip). The elements are copied out before the bit cast:
// __builtin_bit_cast(float, r[1]) on the returned ext-vector reads element 0 (clang codegen).
__device__ __forceinline__ void swap_halves(unsigned r0, unsigned r1, float& a, float& b) {
  a = __builtin_bit_cast(float, r0);
  b = __builtin_bit_cast(float, r1);
}
__device__ __forceinline__ void xor32_pair(float v, float& a, float& b) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const unsigned r0 = r[0], r1 = r[1];
  swap_halves(r0, r1, a, b);
}
__device__ __forceinline__ void xor16_pair(float v, float& a, float& b) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const unsigned r0 = r[0], r1 = r[1];
  swap_halves(r0, r1, a, b);
}

// v + v[lane ^ OFF] (OFF a power of two < 64); EXEC must be full
template <int OFF>
__device__ __forceinline__ float xor_sum(float v) {
  static_assert(OFF > 0 && OFF < 64 && (OFF & (OFF - 1)) == 0, "butterfly offset");
  if constexpr (OFF == 32) {
    float a, b;
    xor32_pair(v, a, b);
    return a + b;
  } else if constexpr (OFF == 16) {
    float a, b;
    xor16_pair(v, a, b);
    return a + b;
  } else if constexpr (OFF == 8) {
    return v + dpp_f<0x128>(v);  // row_ror:8 == lane ^ 8 within a 16-lane row
  } else if constexpr (OFF == 2) {
    return v + dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  } else if constexpr (OFF == 1) {
    return v + dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  } else {
    return v + __shfl_xor(v, OFF, 64);
  }
}

// butterfly over lane offsets OFF, 2*OFF, ..., 32: the sum over the lanes that agree with this
// one in the lane-index bits below log2(OFF)
template <int OFF>
__device__ __forceinline__ float butterfly_from(float v) {
  if constexpr (OFF >= 64) return v;
  else return butterfly_from<OFF * 2>(xor_sum<OFF>(v));
}

template <int OFF>
__device__ __forceinline__ float xor_max(float v) {
  static_assert(OFF == 16 || OFF == 32, "butterfly offset");
  float a, b;
  if constexpr (OFF == 32) xor32_pair(v, a, b);
  else xor16_pair(v, a, b);
  return fmaxf(a, b);
}

// sum over each 16-lane row, in every lane of the row (DPP only)
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  return v + dpp_f<0x128>(v);  // row_ror:8
}

// sum over all 64 lanes, wave-uniform result: DPP row sums (every lane of a row holds its
// row's total), then the four row totals read as scalars
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = row_sum16(v);
  const int b = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}

// Scheduling pattern for a software-pipelined MFMA block: MFMA i is followed by
// floor((i + 1) NR / NM) - floor(i NR / NM) of the next k-step's DS reads, so the reads stream in
// under the matrix work (and fewer than lgkmcnt's 16 are ever outstanding) instead of following it
// in a burst. Call right after the reads and MFMAs it orders, in the same basic block.
template <int I, int NM, int NR>
__device__ __forceinline__ void interleave_mfma_ds() {
  if constexpr (I < NM) {
    constexpr int nr = (I + 1) * NR / NM - I * NR / NM;
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if constexpr (nr > 0) __builtin_amdgcn_sched_group_barrier(0x100, nr, 0);
    interleave_mfma_ds<I + 1, NM, NR>();
  }
}

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
