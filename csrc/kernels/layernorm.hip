// Fused LayerNorm (+ residual add) forward / backward for transformer rows — gfx950.
//
// One 64-lane wavefront per row (ViT-B: D = 768 -> 96 16-byte vectors, 2 per lane), the
// row held in registers between the statistics and the normalisation (one read of x,
// exact two-pass variance), 4 rows per 256-thread workgroup.
//
//   forward   [h = x + r]  y = (h - mean) * rstd * w + b;  mean, rstd saved (fp32 / row)
//   backward  dh = rstd * (g - mean(g) - xhat * mean(g * xhat)) [+ dh_ext],  g = dy * w
//             dw = sum_rows dy * xhat, db = sum_rows dy
//
// The residual add of a pre-LN transformer block ("x = x + sublayer(..); ln(x)") is fused:
// the forward writes h and y in one pass, the backward adds the gradient h receives from
// the rest of the residual stream (dh_ext) in the same pass — no separate add kernels.
// dw/db: the backward grid is one full round of resident workgroups; each wave keeps its
// columns' partial sums in registers across the rows it visits, the block reduces them
// through LDS and stores one [2][D] fp32 partial (no atomics); the partials are summed by
// the split-K tree reduction (gemm_splitk_reduce).
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Forward: a persistent grid (one full round of resident workgroups); each wave walks rows
// row, row + step, ... with the NEXT row's x (and residual) loads issued before the current
// row's reductions, and the affine w/b held in registers for the whole kernel (16-byte
// loads, once). The one-row-per-wave version issued 16 scalar w/b loads per vector after
// the reductions and had only one row's loads in flight: 141-155 us per ViT-B LayerNorm
// (50432 x 768 bf16) on MI355X, ~2-3x its HBM time (s48 trace).
template <typename T, int VPL, bool ADD>
__device__ __forceinline__ void ln_fwd_load(const T* __restrict__ x, const T* __restrict__ r, int64_t row, int D,
                                            int lane, int nv, T (&rx)[VPL][8], T (&rr)[VPL][8]) {
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int v = lane + i * 64;
    if (v < nv) {
      load8(x + row * D + v * 8, rx[i]);
      if (ADD) load8(r + row * D + v * 8, rr[i]);
    }
  }
}

template <typename T, bool ADD, int VPL>
__global__ __launch_bounds__(kThreads) void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                          T* __restrict__ h, T* __restrict__ y,
                                                          const float* __restrict__ w, const float* __restrict__ b,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int64_t rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int nv = D / 8;
  const float inv_d = 1.f / static_cast<float>(D);
  float wv[VPL][8], bv[VPL][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int v = lane + i * 64;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wv[i][j] = 1.f;
      bv[i][j] = 0.f;
    }
    if (v < nv) {
      if (w) {
        const float4 a0 = *reinterpret_cast<const float4*>(w + v * 8);
        const float4 a1 = *reinterpret_cast<const float4*>(w + v * 8 + 4);
        wv[i][0] = a0.x; wv[i][1] = a0.y; wv[i][2] = a0.z; wv[i][3] = a0.w;
        wv[i][4] = a1.x; wv[i][5] = a1.y; wv[i][6] = a1.z; wv[i][7] = a1.w;
      }
      if (b) {
        const float4 a0 = *reinterpret_cast<const float4*>(b + v * 8);
        const float4 a1 = *reinterpret_cast<const float4*>(b + v * 8 + 4);
        bv[i][0] = a0.x; bv[i][1] = a0.y; bv[i][2] = a0.z; bv[i][3] = a0.w;
        bv[i][4] = a1.x; bv[i][5] = a1.y; bv[i][6] = a1.z; bv[i][7] = a1.w;
      }
    }
  }
  const int64_t step = static_cast<int64_t>(gridDim.x) * kWaves;
  int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  T rx[VPL][8], rr[VPL][8];
  if (row < rows) ln_fwd_load<T, VPL, ADD>(x, r, row, D, lane, nv, rx, rr);
  for (; row < rows; row += step) {
    float f[VPL][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int v = lane + i * 64;
      if (v < nv) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[i][j] = static_cast<float>(rx[i][j]);
        if (ADD) {
          T o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            o[j] = static_cast<T>(f[i][j] + static_cast<float>(rr[i][j]));
            f[i][j] = static_cast<float>(o[j]);  // normalise exactly the stored (rounded) h
          }
          store8(h + row * D + v * 8, o);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += f[i][j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[i][j] = 0.f;
      }
    }
    // next row's loads in flight during this row's reductions and stores
    if (row + step < rows) ln_fwd_load<T, VPL, ADD>(x, r, row + step, D, lane, nv, rx, rr);
    const float mean = wave_sum(s) * inv_d;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i)
      if (lane + i * 64 < nv)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = f[i][j] - mean;
          q = fmaf(d, d, q);
        }
    const float rstd = rsqrtf(wave_sum(q) * inv_d + eps);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int v = lane + i * 64;
      if (v < nv) {
        T o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = static_cast<T>(fmaf((f[i][j] - mean) * rstd, wv[i][j], bv[i][j]));
        store8(y + row * D + v * 8, o);
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename T, bool DH, int VPL>
__global__ __launch_bounds__(kThreads) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ dh_ext,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in,
                                                          const float* __restrict__ w, T* __restrict__ dx,
                                                          float* __restrict__ part, int64_t rows, int D) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][D]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = D / 8;
  const float inv_d = 1.f / static_cast<float>(D);
  float wv[VPL][8], dwp[VPL][8], dbp[VPL][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = (lane + i * 64) * 8 + j;
      wv[i][j] = (lane + i * 64 < nv && w) ? w[c] : 1.f;
      dwp[i][j] = dbp[i][j] = 0.f;
    }
  const int64_t step = static_cast<int64_t>(gridDim.x) * kWaves;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wave; row < rows; row += step) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float d[VPL][8], xh[VPL][8], e[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int v = lane + i * 64;
      if (v < nv) {
        T td[8], tx[8];
        load8(dy + row * D + v * 8, td);
        load8(x + row * D + v * 8, tx);
        if (DH) {
          T te[8];
          load8(dh_ext + row * D + v * 8, te);
#pragma unroll
          for (int j = 0; j < 8; ++j) e[i][j] = static_cast<float>(te[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          d[i][j] = static_cast<float>(td[j]);
          xh[i][j] = (static_cast<float>(tx[j]) - mean) * rstd;
          const float g = d[i][j] * wv[i][j];
          s1 += g;
          s2 = fmaf(g, xh[i][j], s2);
          dwp[i][j] = fmaf(d[i][j], xh[i][j], dwp[i][j]);
          dbp[i][j] += d[i][j];
        }
      }
    }
    const float m1 = wave_sum(s1) * inv_d, m2 = wave_sum(s2) * inv_d;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int v = lane + i * 64;
      if (v < nv) {
        T o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float g = rstd * (d[i][j] * wv[i][j] - m1 - xh[i][j] * m2);
          if (DH) g += e[i][j];
          o[j] = static_cast<T>(g);
        }
        store8(dx + row * D + v * 8, o);
      }
    }
  }
  // block partial of dw / db: the waves add their register partials into one [2][D] LDS
  // row in turn (8*D bytes of LDS whatever the wave count)
  for (int k = 0; k < kWaves; ++k) {
    if (wave == k) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int v = lane + i * 64;
        if (v < nv)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int c = v * 8 + j;
            red[c] = k == 0 ? dwp[i][j] : red[c] + dwp[i][j];
            red[D + c] = k == 0 ? dbp[i][j] : red[D + c] + dbp[i][j];
          }
      }
    }
    __syncthreads();
  }
  float* out = part + static_cast<int64_t>(blockIdx.x) * 2 * D;
  for (int c = threadIdx.x; c < 2 * D; c += kThreads) out[c] = red[c];
}

int vpl_for(int64_t D) {
  if (D % 8 != 0 || D < 8 || D > 8192)
    throw std::runtime_error("fused layernorm: need D % 8 == 0 and 8 <= D <= 8192 (got " + std::to_string(D) + ")");
  const int v = static_cast<int>((D / 8 + 63) / 64);  // vectors per lane actually needed
  for (int c : {1, 2, 3, 4, 6, 8, 12, 16})
    if (c >= v) return c;
  return 16;
}

template <typename T, bool ADD, int VPL>
void fwd_launch(const void* x, const void* r, void* h, void* y, const float* w, const float* b, float* mean,
                float* rstd, int64_t rows, int64_t D, float eps, hipStream_t s) {
  auto k = ln_fwd_kernel<T, ADD, VPL>;
  int64_t blocks = resident_blocks(reinterpret_cast<const void*>(k), kThreads, 0);
  const int64_t need = (rows + kWaves - 1) / kWaves;
  if (blocks > need) blocks = need;
  if (blocks < 1) blocks = 1;
  k<<<(unsigned)blocks, kThreads, 0, s>>>(
      static_cast<const T*>(x), static_cast<const T*>(r), static_cast<T*>(h), static_cast<T*>(y), w, b, mean, rstd,
      rows, static_cast<int>(D), eps);
}

template <typename T, bool DH, int VPL>
int bwd_launch(const void* dy, const void* x, const void* dh, const float* mean, const float* rstd, const float* w,
               void* dx, float* part, int max_blocks, int64_t rows, int64_t D, hipStream_t s) {
  auto k = ln_bwd_kernel<T, DH, VPL>;
  const size_t lds = static_cast<size_t>(2) * D * sizeof(float);
  int64_t blocks = resident_blocks(reinterpret_cast<const void*>(k), kThreads, lds);
  const int64_t need = (rows + kWaves - 1) / kWaves;
  if (blocks > need) blocks = need;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  k<<<(unsigned)blocks, kThreads, lds, s>>>(static_cast<const T*>(dy), static_cast<const T*>(x),
                                            static_cast<const T*>(dh), mean, rstd, w, static_cast<T*>(dx), part, rows,
                                            static_cast<int>(D));
  return static_cast<int>(blocks);
}

// compiled vectors-per-lane variants (D up to 8192)
#define LN_VPL_SWITCH(VPL_VAR, CALL) \
  switch (VPL_VAR) {                 \
    case 1: CALL(1); break;          \
    case 2: CALL(2); break;          \
    case 3: CALL(3); break;          \
    case 4: CALL(4); break;          \
    case 6: CALL(6); break;          \
    case 8: CALL(8); break;          \
    case 12: CALL(12); break;        \
    default: CALL(16); break;        \
  }

}  // namespace

void layernorm_fwd(const void* x, const void* residual, void* h, void* y, const float* w, const float* b, float* mean,
                   float* rstd, int64_t rows, int64_t D, float eps, int dtype, hipStream_t stream) {
  const int vpl = vpl_for(D);
  const bool add = residual != nullptr;
  if ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(b)) % 16 != 0)
    throw std::runtime_error("fused layernorm: w and b must be 16-byte aligned fp32");
#define CALL_ADD(V) fwd_launch<TT, true, V>(x, residual, h, y, w, b, mean, rstd, rows, D, eps, stream)
#define CALL_NOADD(V) fwd_launch<TT, false, V>(x, residual, h, y, w, b, mean, rstd, rows, D, eps, stream)
  switch (dtype) {
    case kBF16: {
      using TT = bf16;
      if (add) { LN_VPL_SWITCH(vpl, CALL_ADD) } else { LN_VPL_SWITCH(vpl, CALL_NOADD) }
      break;
    }
    case kF16: {
      using TT = f16;
      if (add) { LN_VPL_SWITCH(vpl, CALL_ADD) } else { LN_VPL_SWITCH(vpl, CALL_NOADD) }
      break;
    }
    case kF32: {
      using TT = float;
      if (add) { LN_VPL_SWITCH(vpl, CALL_ADD) } else { LN_VPL_SWITCH(vpl, CALL_NOADD) }
      break;
    }
    default:
      throw std::runtime_error("fused layernorm: unsupported dtype");
  }
#undef CALL_ADD
#undef CALL_NOADD
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

int layernorm_bwd(const void* dy, const void* x, const void* dh_ext, const float* mean, const float* rstd,
                  const float* w, void* dx, float* partials, int max_blocks, int64_t rows, int64_t D, int dtype,
                  hipStream_t stream) {
  const int vpl = vpl_for(D);
  const bool dh = dh_ext != nullptr;
  int blocks = 0;
#define CALL_DH(V) blocks = bwd_launch<TT, true, V>(dy, x, dh_ext, mean, rstd, w, dx, partials, max_blocks, rows, D, stream)
#define CALL_NODH(V) blocks = bwd_launch<TT, false, V>(dy, x, dh_ext, mean, rstd, w, dx, partials, max_blocks, rows, D, stream)
  switch (dtype) {
    case kBF16: {
      using TT = bf16;
      if (dh) { LN_VPL_SWITCH(vpl, CALL_DH) } else { LN_VPL_SWITCH(vpl, CALL_NODH) }
      break;
    }
    case kF16: {
      using TT = f16;
      if (dh) { LN_VPL_SWITCH(vpl, CALL_DH) } else { LN_VPL_SWITCH(vpl, CALL_NODH) }
      break;
    }
    case kF32: {
      using TT = float;
      if (dh) { LN_VPL_SWITCH(vpl, CALL_DH) } else { LN_VPL_SWITCH(vpl, CALL_NODH) }
      break;
    }
    default:
      throw std::runtime_error("fused layernorm: unsupported dtype");
  }
#undef CALL_DH
#undef CALL_NODH
  FLUXMPI_HIP_CHECK(hipGetLastError());
  return blocks;
}

}  // namespace fluxmpi
