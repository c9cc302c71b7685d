// GELU backward fused with the bias gradient of the Linear that produced its input — gfx950.
//
// Transformer MLP: h = x W1^T + b1, y = gelu(h). Autograd runs the GELU backward as one
// elementwise pass (read dy, h; write dh) and then the bias gradient db1 = sum_rows dh as a
// separate column reduction that reads dh again (ViT-B/16: 50432 x 3072 bf16 per block).
// Here one pass writes dh and accumulates db1: every lane owns ONE fixed 8-column vector
// (blockDim = N/8 lanes, N/8 a multiple of 64), so its column sums stay in registers over
// the workgroup's row range; each workgroup stores one fp32 partial row (no atomics), summed
// by gemm_splitk_reduce. GELU derivative in fp32: tanh form (gelu_tanh.h; the default, gelu_set_form)
// or the exact erf form (polynomial erf, |error| <= 1.5e-7).
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"
#include "gelu_tanh.h"

namespace fluxmpi {
namespace {

// gelu'(x) = Phi(x) + x phi(x) with Phi from the Abramowitz-Stegun 7.1.26 erf (|error| <= 1.5e-7):
// erf(z) = 1 - t (a1 + t (a2 + ... + t a5)) exp(-z^2), t = 1 / (1 + p z), z = |x| / sqrt(2). Its
// exp(-z^2) = exp(-x^2 / 2) is the pdf's exponential, so one v_exp_f32 + one v_rcp_f32 + 5 FMAs
// replace erff (~30 VALU ops with branches): at 155 M elements per ViT-B/16 block the libm erf made
// this pass VALU-bound (222 us vs the 155 us HBM time of its 930 MB).
__device__ __forceinline__ float gelu_grad(float x) {
  constexpr float kP = 0.3275911f, kA1 = 0.254829592f, kA2 = -0.284496736f, kA3 = 1.421413741f,
                  kA4 = -1.453152027f, kA5 = 1.061405429f;
  constexpr float kInvSqrt2 = 0.70710678118654752f, kInvSqrt2Pi = 0.39894228040143268f;
  constexpr float kNegHalfLog2e = -0.72134752044448170f;  // -log2(e) / 2
  const float e = __builtin_amdgcn_exp2f(kNegHalfLog2e * x * x);  // exp(-x^2 / 2)
  const float t = __builtin_amdgcn_rcpf(fmaf(kP * kInvSqrt2, fabsf(x), 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, kA5, kA4), kA3), kA2), kA1);
  const float tail = 0.5f * poly * e;  // 0.5 * (1 - erf(|x| / sqrt2))
  const float cdf = x >= 0.f ? 1.f - tail : tail;
  return fmaf(x * kInvSqrt2Pi, e, cdf);
}

int g_gelu_tanh = 1;  // gelu_set_form

// x Phi(x), Phi from the same Abramowitz-Stegun erf as gelu_grad
__device__ __forceinline__ float gelu_erf(float x) {
  constexpr float kP = 0.3275911f, kA1 = 0.254829592f, kA2 = -0.284496736f, kA3 = 1.421413741f,
                  kA4 = -1.453152027f, kA5 = 1.061405429f;
  constexpr float kInvSqrt2 = 0.70710678118654752f, kNegHalfLog2e = -0.72134752044448170f;
  const float e = __builtin_amdgcn_exp2f(kNegHalfLog2e * x * x);
  const float t = __builtin_amdgcn_rcpf(fmaf(kP * kInvSqrt2, fabsf(x), 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, kA5, kA4), kA3), kA2), kA1);
  const float tail = 0.5f * poly * e;
  return x * (x >= 0.f ? 1.f - tail : tail);
}

// g = gelu(h) over n elements (n % 8 == 0, 16-B aligned): every lane keeps kU 16-B vectors'
// loads in flight per grid-stride iteration (the fc1 activation of ViT-B/16: 155 M elements,
// 620 MB per call — HBM-bound)
template <typename T, bool TANH>
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const T* __restrict__ h, T* __restrict__ g, int64_t nvec) {
  constexpr int kU = 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; v + (kU - 1) * stride < nvec; v += kU * stride) {
    T x[kU][8];
#pragma unroll
    for (int u = 0; u < kU; ++u) load8(h + (v + u * stride) * 8, x[u]);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      T o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = to_f(x[u][j]);
        o[j] = from_f<T>(TANH ? gelu_tanh(f) : gelu_erf(f));
      }
      store8(g + (v + u * stride) * 8, o);
    }
  }
  for (; v < nvec; v += stride) {
    T x[8], o[8];
    load8(h + v * 8, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = to_f(x[j]);
      o[j] = from_f<T>(TANH ? gelu_tanh(f) : gelu_erf(f));
    }
    store8(g + v * 8, o);
  }
}

template <bool TANH>
__device__ __forceinline__ float gelu_d(float x) {
  if constexpr (TANH) return gelu_tanh_grad(x);
  else return gelu_grad(x);
}

template <typename T, bool TANH>
__global__ __launch_bounds__(1024) void gelu_bwd_bias_kernel(const T* __restrict__ dy, const T* __restrict__ h,
                                                             T* __restrict__ dh, float* __restrict__ part,
                                                             int64_t rows, int64_t N, int64_t rows_per_wg) {
  const int64_t cv = threadIdx.x;  // column vector owned by this lane
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_wg;
  int64_t r1 = r0 + rows_per_wg;
  if (r1 > rows) r1 = rows;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  // kU rows per iteration with all their loads issued before any math (one row at a time
  // left the loop latency-bound at ~2.5 TB/s)
  constexpr int kU = 4;
  int64_t r = r0;
  for (; r + kU <= r1; r += kU) {
    T dv[kU][8], hv[kU][8];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      load8(dy + (r + u) * N + cv * 8, dv[u]);
      load8(h + (r + u) * N + cv * 8, hv[u]);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      T ov[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ov[j] = from_f<T>(to_f(dv[u][j]) * gelu_d<TANH>(to_f(hv[u][j])));
        acc[j] += to_f(ov[j]);  // db of the rounded dh the weight / input gradients use
      }
      store8(dh + (r + u) * N + cv * 8, ov);
    }
  }
  for (; r < r1; ++r) {
    const int64_t off = r * N + cv * 8;
    T dv[8], hv[8], ov[8];
    load8(dy + off, dv);
    load8(h + off, hv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ov[j] = from_f<T>(to_f(dv[j]) * gelu_d<TANH>(to_f(hv[j])));
      acc[j] += to_f(ov[j]);
    }
    store8(dh + off, ov);
  }
  float* out = part + static_cast<int64_t>(blockIdx.x) * N + cv * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = acc[j];
}

// Column sums of a row-major [rows][N] matrix (the bias gradient of a Linear: db = sum_rows dy),
// any N % 8 == 0: a workgroup is R row-phases x V = N/8 column vectors (V*R <= 1024); each lane
// keeps the fp32 sums of its 8 columns over the rows of its phase (kU rows' loads in flight per
// iteration), the R phases are combined through LDS and each workgroup stores one fp32 partial
// row (summed by gemm_splitk_reduce, which also casts).
template <typename T>
__global__ __launch_bounds__(1024) void colsum_kernel(const T* __restrict__ x, float* __restrict__ part, int64_t rows,
                                                      int64_t N, int64_t rows_per_wg, int R) {
  extern __shared__ float red[];  // [R][N]
  const int V = static_cast<int>(N / 8);
  const int cv = threadIdx.x % V, ph = threadIdx.x / V;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_wg;
  int64_t r1 = r0 + rows_per_wg;
  if (r1 > rows) r1 = rows;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  constexpr int kU = 4;
  int64_t r = r0 + ph;
  for (; r + (kU - 1) * R < r1; r += kU * R) {
    T v[kU][8];
#pragma unroll
    for (int u = 0; u < kU; ++u) load8(x + (r + u * R) * N + cv * 8, v[u]);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += to_f(v[u][j]);
  }
  for (; r < r1; r += R) {
    T v[8];
    load8(x + r * N + cv * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += to_f(v[j]);
  }
  if (ph < R) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[ph * N + cv * 8 + j] = acc[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < R; ++q) s += red[q * N + c];
    part[static_cast<int64_t>(blockIdx.x) * N + c] = s;
  }
}

}  // namespace

int colsum_blocks(int64_t rows) {
  int64_t b = rows / 64;  // >= 64 rows per workgroup, at most 1024 workgroups
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

void colsum(const void* x, float* partials, int blocks, int64_t rows, int64_t N, int dtype, hipStream_t stream) {
  if (N % 8 != 0 || N / 8 > 1024 || N > 8192)
    throw std::runtime_error("colsum: need N % 8 == 0 and N <= 8192 (got N=" + std::to_string(N) + ")");
  if (blocks < 1 || rows < 1) throw std::runtime_error("colsum: bad grid");
  if ((reinterpret_cast<uintptr_t>(x) & 15u) != 0) throw std::runtime_error("colsum: input must be 16-byte aligned");
  const int V = static_cast<int>(N / 8);
  int R = 256 / V;
  if (R < 1) R = 1;
  const int64_t rpw = (rows + blocks - 1) / blocks;
  const unsigned threads = static_cast<unsigned>(V * R);
  const size_t smem = static_cast<size_t>(R) * N * sizeof(float);
  switch (dtype) {
    case kBF16:
      colsum_kernel<bf16><<<blocks, threads, smem, stream>>>(static_cast<const bf16*>(x), partials, rows, N, rpw, R);
      break;
    case kF16:
      colsum_kernel<f16><<<blocks, threads, smem, stream>>>(static_cast<const f16*>(x), partials, rows, N, rpw, R);
      break;
    case kF32:
      colsum_kernel<float><<<blocks, threads, smem, stream>>>(static_cast<const float*>(x), partials, rows, N, rpw, R);
      break;
    default:
      throw std::runtime_error("colsum: bf16 / fp16 / fp32 only");
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

int gelu_bwd_bias_blocks(int64_t rows) {
  int64_t b = rows / 32;  // >= 32 rows per workgroup, at most 1024 workgroups
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

void gelu_fwd(const void* h, void* g, int64_t n, int dtype, hipStream_t stream) {
  if (n <= 0) return;
  if (n % 8 != 0) throw std::runtime_error("gelu_fwd: need n % 8 == 0 (got " + std::to_string(n) + ")");
  if (((reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(g)) & 15u) != 0)
    throw std::runtime_error("gelu_fwd: tensors must be 16-byte aligned");
  const int64_t nvec = n / 8;
  int64_t blocks = (nvec + 256 * 4 - 1) / (256 * 4);
  if (blocks > 4096) blocks = 4096;
  const bool t = g_gelu_tanh != 0;
  switch (dtype) {
    case kBF16: {
      auto k = t ? gelu_fwd_kernel<bf16, true> : gelu_fwd_kernel<bf16, false>;
      k<<<static_cast<unsigned>(blocks), 256, 0, stream>>>(static_cast<const bf16*>(h), static_cast<bf16*>(g), nvec);
      break;
    }
    case kF16: {
      auto k = t ? gelu_fwd_kernel<f16, true> : gelu_fwd_kernel<f16, false>;
      k<<<static_cast<unsigned>(blocks), 256, 0, stream>>>(static_cast<const f16*>(h), static_cast<f16*>(g), nvec);
      break;
    }
    default:
      throw std::runtime_error("gelu_fwd: bf16 / fp16 only");
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void gelu_set_form(int tanh_form) { g_gelu_tanh = tanh_form != 0 ? 1 : 0; }
int gelu_form() { return g_gelu_tanh; }

void gelu_bwd_bias(const void* dy, const void* h, void* dh, float* partials, int blocks, int64_t rows, int64_t N,
                   int dtype, hipStream_t stream) {
  if (N % 8 != 0 || (N / 8) % 64 != 0 || N / 8 > 1024)
    throw std::runtime_error("gelu_bwd_bias: need N/8 a multiple of 64 and <= 1024 (got N=" + std::to_string(N) + ")");
  if (blocks < 1 || rows < 1) throw std::runtime_error("gelu_bwd_bias: bad grid");
  if (((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(dh)) & 15u) != 0)
    throw std::runtime_error("gelu_bwd_bias: tensors must be 16-byte aligned");
  const int64_t rpw = (rows + blocks - 1) / blocks;
  const unsigned threads = static_cast<unsigned>(N / 8);
  const bool tanh_form = g_gelu_tanh != 0;
  switch (dtype) {
    case kBF16: {
      auto k = tanh_form ? gelu_bwd_bias_kernel<bf16, true> : gelu_bwd_bias_kernel<bf16, false>;
      k<<<blocks, threads, 0, stream>>>(static_cast<const bf16*>(dy), static_cast<const bf16*>(h), static_cast<bf16*>(dh),
                                        partials, rows, N, rpw);
      break;
    }
    case kF16: {
      auto k = tanh_form ? gelu_bwd_bias_kernel<f16, true> : gelu_bwd_bias_kernel<f16, false>;
      k<<<blocks, threads, 0, stream>>>(static_cast<const f16*>(dy), static_cast<const f16*>(h), static_cast<f16*>(dh),
                                        partials, rows, N, rpw);
      break;
    }
    default:
      throw std::runtime_error("gelu_bwd_bias: bf16 / fp16 only");
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
