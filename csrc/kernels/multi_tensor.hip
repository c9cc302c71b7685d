// Multi-tensor copy / cast / scale / fill / sum-of-squares for gfx950.
//
// K1/K2 of SURVEY §2.4: the reference moves every gradient leaf through host
// memory one at a time (src/optimizer.jl:47,62; src/mpi_extensions.jl:97-155).
// Here a single launch gathers many leaves into one contiguous, 16 B-aligned
// communication bucket (pack) or scatters the reduced bucket back (unpack),
// optionally casting (bf16 <-> fp32) and scaling (e.g. 1/world) on the fly.
//
// Work decomposition: workgroup b owns elements [c*kChunk, (c+1)*kChunk) of
// tensor t, where (t, c) comes from a prefix table carried in the kernel
// arguments. Each lane moves 8 elements per step with 16 B vector accesses;
// 4 steps are issued before any store so every lane keeps 4 loads in flight.
#include <stdexcept>
#include <string>
#include <vector>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;
constexpr int kIters = 4;
constexpr int kChunk = kThreads * kVec * kIters;  // 8192 elements per workgroup
constexpr int kMaxT = 40;

struct CopyArgs {
  uintptr_t src[kMaxT];
  uintptr_t dst[kMaxT];
  int64_t numel[kMaxT];
  int32_t start[kMaxT + 1];
  int n;
};

template <typename Tin, typename Tout>
__device__ __forceinline__ Tout cvt(Tin x, float scale) {
  using A = typename Acc<Tin>::type;
  return static_cast<Tout>(static_cast<A>(x) * static_cast<A>(scale));
}
template <>
__device__ __forceinline__ double cvt<double, double>(double x, float scale) {
  return x * static_cast<double>(scale);
}
template <>
__device__ __forceinline__ double cvt<float, double>(float x, float scale) {
  return static_cast<double>(x) * static_cast<double>(scale);
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(kThreads) void mt_copy_kernel(CopyArgs a, float scale) {
  const int b = blockIdx.x;
  const int t = find_tensor(a.start, a.n, b);
  const int64_t base = static_cast<int64_t>(b - a.start[t]) * kChunk;
  const int64_t n = a.numel[t];
  const int64_t end = base + kChunk < n ? base + kChunk : n;
  const Tin* __restrict__ src = reinterpret_cast<const Tin*>(a.src[t]);
  Tout* __restrict__ dst = reinterpret_cast<Tout*>(a.dst[t]);
  const int tid = threadIdx.x;
  const bool same_bits = sizeof(Tin) == sizeof(Tout);
  if (aligned16(src) && aligned16(dst)) {
    const int64_t nvec = (end - base) / kVec;  // full 8-element vectors in this chunk
    Tin in[kIters][kVec];
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const int64_t v = tid + k * kThreads;
      if (v < nvec) load8(src + base + v * kVec, in[k]);
    }
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const int64_t v = tid + k * kThreads;
      if (v < nvec) {
        Tout o[kVec];
#pragma unroll
        for (int j = 0; j < kVec; ++j) o[j] = cvt<Tin, Tout>(in[k][j], scale);
        store8(dst + base + v * kVec, o);
      }
    }
    for (int64_t i = base + nvec * kVec + tid; i < end; i += kThreads) dst[i] = cvt<Tin, Tout>(src[i], scale);
  } else {
    (void)same_bits;
    for (int64_t i = base + tid; i < end; i += kThreads) dst[i] = cvt<Tin, Tout>(src[i], scale);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void mt_fill_kernel(CopyArgs a, float value) {
  const int b = blockIdx.x;
  const int t = find_tensor(a.start, a.n, b);
  const int64_t base = static_cast<int64_t>(b - a.start[t]) * kChunk;
  const int64_t n = a.numel[t];
  const int64_t end = base + kChunk < n ? base + kChunk : n;
  T* __restrict__ dst = reinterpret_cast<T*>(a.dst[t]);
  const T val = static_cast<T>(value);
  const int tid = threadIdx.x;
  if (aligned16(dst)) {
    const int64_t nvec = (end - base) / kVec;
    T o[kVec];
#pragma unroll
    for (int j = 0; j < kVec; ++j) o[j] = val;
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const int64_t v = tid + k * kThreads;
      if (v < nvec) store8(dst + base + v * kVec, o);
    }
    for (int64_t i = base + nvec * kVec + tid; i < end; i += kThreads) dst[i] = val;
  } else {
    for (int64_t i = base + tid; i < end; i += kThreads) dst[i] = val;
  }
}

__device__ __forceinline__ float wave_sum(float x) { return wave_sum_dpp(x); }  // common.h

template <typename T>
__global__ __launch_bounds__(kThreads) void mt_sumsq_kernel(CopyArgs a, float* out) {
  __shared__ float partial[kThreads / 64];
  const int b = blockIdx.x;
  const int t = find_tensor(a.start, a.n, b);
  const int64_t base = static_cast<int64_t>(b - a.start[t]) * kChunk;
  const int64_t n = a.numel[t];
  const int64_t end = base + kChunk < n ? base + kChunk : n;
  const T* __restrict__ src = reinterpret_cast<const T*>(a.src[t]);
  const int tid = threadIdx.x;
  float acc = 0.f;
  if (aligned16(src)) {
    const int64_t nvec = (end - base) / kVec;
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const int64_t v = tid + k * kThreads;
      if (v < nvec) {
        T in[kVec];
        load8(src + base + v * kVec, in);
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
          const float f = static_cast<float>(in[j]);
          acc = fmaf(f, f, acc);
        }
      }
    }
    for (int64_t i = base + nvec * kVec + tid; i < end; i += kThreads) {
      const float f = static_cast<float>(src[i]);
      acc = fmaf(f, f, acc);
    }
  } else {
    for (int64_t i = base + tid; i < end; i += kThreads) {
      const float f = static_cast<float>(src[i]);
      acc = fmaf(f, f, acc);
    }
  }
  acc = wave_sum(acc);
  if ((tid & 63) == 0) partial[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += partial[w];
    atomicAdd(out, s);
  }
}

// Build launch groups of <= kMaxT non-empty tensors.
template <typename F>
void for_each_group(const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst,
                    const std::vector<int64_t>& numel, F&& launch) {
  CopyArgs a{};
  int n = 0;
  int32_t blocks = 0;
  auto flush = [&]() {
    if (n == 0) return;
    a.n = n;
    a.start[n] = blocks;
    launch(a, blocks);
    a = CopyArgs{};
    n = 0;
    blocks = 0;
  };
  for (size_t i = 0; i < numel.size(); ++i) {
    if (numel[i] <= 0) continue;
    const int64_t nb = (numel[i] + kChunk - 1) / kChunk;
    if (nb > (int64_t(1) << 30)) throw std::runtime_error("mt kernel: tensor too large");
    if (n == kMaxT || int64_t(blocks) + nb > (int64_t(1) << 30)) flush();
    a.src[n] = src.empty() ? 0 : src[i];
    a.dst[n] = dst.empty() ? 0 : dst[i];
    a.numel[n] = numel[i];
    a.start[n] = blocks;
    blocks += static_cast<int32_t>(nb);
    ++n;
  }
  flush();
}

template <typename Tin>
void copy_from(int out_dtype, const CopyArgs& a, int blocks, float scale, hipStream_t s) {
  switch (out_dtype) {
    case kF32: mt_copy_kernel<Tin, float><<<blocks, kThreads, 0, s>>>(a, scale); break;
    case kBF16: mt_copy_kernel<Tin, bf16><<<blocks, kThreads, 0, s>>>(a, scale); break;
    case kF16: mt_copy_kernel<Tin, f16><<<blocks, kThreads, 0, s>>>(a, scale); break;
    case kF64: mt_copy_kernel<Tin, double><<<blocks, kThreads, 0, s>>>(a, scale); break;
    default: throw std::runtime_error("mt_copy: unsupported output dtype " + std::to_string(out_dtype));
  }
}

}  // namespace

void mt_copy(const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst,
             const std::vector<int64_t>& numel, int in_dtype, int out_dtype, float scale,
             hipStream_t stream) {
  if (src.size() != numel.size() || dst.size() != numel.size())
    throw std::runtime_error("mt_copy: list length mismatch");
  for_each_group(src, dst, numel, [&](const CopyArgs& a, int blocks) {
    switch (in_dtype) {
      case kF32: copy_from<float>(out_dtype, a, blocks, scale, stream); break;
      case kBF16: copy_from<bf16>(out_dtype, a, blocks, scale, stream); break;
      case kF16: copy_from<f16>(out_dtype, a, blocks, scale, stream); break;
      case kF64:
        if (out_dtype == kF64) mt_copy_kernel<double, double><<<blocks, kThreads, 0, stream>>>(a, scale);
        else if (out_dtype == kF32) mt_copy_kernel<double, float><<<blocks, kThreads, 0, stream>>>(a, scale);
        else throw std::runtime_error("mt_copy: fp64 -> low precision not supported");
        break;
      default: throw std::runtime_error("mt_copy: unsupported input dtype " + std::to_string(in_dtype));
    }
    FLUXMPI_HIP_CHECK(hipGetLastError());
  });
}

void mt_fill(const std::vector<uintptr_t>& dst, const std::vector<int64_t>& numel, int dtype,
             float value, hipStream_t stream) {
  for_each_group({}, dst, numel, [&](const CopyArgs& a, int blocks) {
    switch (dtype) {
      case kF32: mt_fill_kernel<float><<<blocks, kThreads, 0, stream>>>(a, value); break;
      case kBF16: mt_fill_kernel<bf16><<<blocks, kThreads, 0, stream>>>(a, value); break;
      case kF16: mt_fill_kernel<f16><<<blocks, kThreads, 0, stream>>>(a, value); break;
      case kF64: mt_fill_kernel<double><<<blocks, kThreads, 0, stream>>>(a, value); break;
      default: throw std::runtime_error("mt_fill: unsupported dtype");
    }
    FLUXMPI_HIP_CHECK(hipGetLastError());
  });
}

void mt_sumsq(const std::vector<uintptr_t>& src, const std::vector<int64_t>& numel, int dtype,
              float* out, hipStream_t stream) {
  for_each_group(src, {}, numel, [&](const CopyArgs& a, int blocks) {
    switch (dtype) {
      case kF32: mt_sumsq_kernel<float><<<blocks, kThreads, 0, stream>>>(a, out); break;
      case kBF16: mt_sumsq_kernel<bf16><<<blocks, kThreads, 0, stream>>>(a, out); break;
      case kF16: mt_sumsq_kernel<f16><<<blocks, kThreads, 0, stream>>>(a, out); break;
      default: throw std::runtime_error("mt_sumsq: unsupported dtype");
    }
    FLUXMPI_HIP_CHECK(hipGetLastError());
  });
}

}  // namespace fluxmpi
