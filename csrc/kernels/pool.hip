// Fused BatchNorm-affine + ReLU + max-pool (the ResNet stem) and its backward — gfx950.
//
// Unfused, the stem writes the normalised 112x112x64 activation, re-reads it in
// the max-pool, and the pool stores int64 argmax indices (8 B per pooled
// element); its backward zero-fills and scatters into a full-resolution tensor.
// Here:
//   forward   p = relu(max_{window} (x*scale + shift)) read straight from the conv
//             output x (the per-channel scale/shift come from the BN statistics
//             pass), plus a 1-byte window index per pooled element (0xFF when the
//             max is <= 0: the ReLU blocks the gradient);
//   backward  dz[h,w] = sum of dp over the (at most ceil(K/S)^2) windows whose
//             recorded argmax is (h,w) — a gather, every dz element written once,
//             no zero fill, no atomics. dz is the gradient of the pre-ReLU BN output
//             and feeds the plain BatchNorm backward.
// Layout NHWC, 8 channels (16 B) per lane; consecutive lanes walk channels, then
// output columns, so a wave reads whole contiguous pixel rows.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

constexpr int kThreads = 256;

struct PoolGeo {
  int64_t N, H, W, C, OH, OW;
  int K, S, P;
};

// One workgroup per output row (n, oh); lanes walk (ow, channel vector) of the row with
// 32-bit index math (64-bit division per element made the first version ALU-bound).
// KK > 0: the window size at compile time; every in-image tap's load is issued before the first
// compare (the generic loop's branches kept one 16-B load in flight per lane at a time).
template <typename T, int KK = 0>
__global__ __launch_bounds__(1024) void bn_relu_maxpool_fwd_kernel(const T* __restrict__ x,
                                                                       const float* __restrict__ scale,
                                                                       const float* __restrict__ shift,
                                                                       T* __restrict__ y, uint8_t* __restrict__ idx,
                                                                       PoolGeo g) {
  const int cv = static_cast<int>(g.C / 8);
  const int row = blockIdx.x;  // n * OH + oh
  const int oh = row % static_cast<int>(g.OH);
  const int64_t n = row / static_cast<int>(g.OH);
  const int h0 = oh * g.S - g.P;
  const int per_row = static_cast<int>(g.OW) * cv;
  const T* xn = x + n * g.H * g.W * g.C;
  for (int t = threadIdx.x; t < per_row; t += blockDim.x) {
    const int ow = t / cv, c8 = t - ow * cv;
    const int c0 = c8 * 8;
    const int w0 = ow * g.S - g.P;
    float sc[8], sh[8], best[8];
    int arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = scale[c0 + j];
      sh[j] = shift[c0 + j];
      best[j] = -INFINITY;
      arg[j] = 0;
    }
    if constexpr (KK > 0) {
      T raw[KK * KK][8];
      bool ok[KK * KK];
#pragma unroll
      for (int k = 0; k < KK * KK; ++k) {
        const int h = h0 + k / KK, w = w0 + k % KK;
        ok[k] = h >= 0 && h < g.H && w >= 0 && w < g.W;
        load8(xn + (static_cast<int64_t>(ok[k] ? h : 0) * g.W + (ok[k] ? w : 0)) * g.C + c0, raw[k]);
      }
#pragma unroll
      for (int k = 0; k < KK * KK; ++k) {
        if (!ok[k]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float z = fmaf(static_cast<float>(raw[k][j]), sc[j], sh[j]);  // as below
          if (z > best[j]) {
            best[j] = z;
            arg[j] = k;
          }
        }
      }
    }
    for (int kh = 0; KK == 0 && kh < g.K; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= g.H) continue;
      for (int kw = 0; kw < g.K; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= g.W) continue;
        T raw[8];
        load8(xn + (static_cast<int64_t>(h) * g.W + w) * g.C + c0, raw);
        const int k = kh * g.K + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // bit-identical to bn_norm_kernel's fmaf(x, scale, shift); first max wins on ties
          const float z = fmaf(static_cast<float>(raw[j]), sc[j], sh[j]);
          if (z > best[j]) {
            best[j] = z;
            arg[j] = k;
          }
        }
      }
    }
    T out[8];
    uint8_t a8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool pos = best[j] > 0.f;
      out[j] = static_cast<T>(pos ? best[j] : 0.f);
      a8[j] = pos ? static_cast<uint8_t>(arg[j]) : static_cast<uint8_t>(0xFF);
    }
    const int64_t o = static_cast<int64_t>(row) * per_row * 8 + static_cast<int64_t>(t) * 8;
    store8(y + o, out);
    uint2 packed;
    __builtin_memcpy(&packed, a8, 8);
    *reinterpret_cast<uint2*>(idx + o) = packed;
  }
}

// NW = max windows covering one input position per dimension (ceil(K/S)): the candidate
// windows are visited in a fixed, fully unrolled NW x NW pattern and all of their index
// and gradient loads are issued before any is consumed (no load -> compare -> load chains).
template <typename T, int NW>
__global__ __launch_bounds__(kThreads) void maxpool_bwd_gather_kernel(const T* __restrict__ dy,
                                                                      const uint8_t* __restrict__ idx,
                                                                      T* __restrict__ dx, PoolGeo g) {
  const int cv = static_cast<int>(g.C / 8);
  const int row = blockIdx.x;  // n * H + h of the input
  const int h = row % static_cast<int>(g.H);
  const int64_t n = row / static_cast<int>(g.H);
  // windows oh with oh*S - P <= h <= oh*S - P + K - 1
  int oh_lo = h + g.P - g.K + 1;
  oh_lo = oh_lo <= 0 ? 0 : (oh_lo + g.S - 1) / g.S;
  int oh_hi = (h + g.P) / g.S;
  if (oh_hi > g.OH - 1) oh_hi = static_cast<int>(g.OH) - 1;
  const int per_row = static_cast<int>(g.W) * cv;
  const int64_t obase = n * g.OH * g.OW * g.C;
  for (int t = threadIdx.x; t < per_row; t += kThreads) {
    const int w = t / cv, c8 = t - w * cv;
    int ow_lo = w + g.P - g.K + 1;
    ow_lo = ow_lo <= 0 ? 0 : (ow_lo + g.S - 1) / g.S;
    int ow_hi = (w + g.P) / g.S;
    if (ow_hi > g.OW - 1) ow_hi = static_cast<int>(g.OW) - 1;
    uint2 ix[NW][NW];
    T d[NW][NW][8];
    int kk[NW][NW];
#pragma unroll
    for (int i = 0; i < NW; ++i)
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const int oh = oh_lo + i, ow = ow_lo + j;
        const bool ok = oh <= oh_hi && ow <= ow_hi;
        kk[i][j] = ok ? (h - (oh * g.S - g.P)) * g.K + (w - (ow * g.S - g.P)) : -1;
        if (ok) {
          const int64_t o = obase + (static_cast<int64_t>(oh) * g.OW + ow) * g.C + c8 * 8;
          ix[i][j] = *reinterpret_cast<const uint2*>(idx + o);
          load8(dy + o, d[i][j]);
        } else {
          ix[i][j] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        }
      }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NW; ++i)
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        uint8_t a8[8];
        __builtin_memcpy(a8, &ix[i][j], 8);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (static_cast<int>(a8[e]) == kk[i][j]) acc[e] += static_cast<float>(d[i][j][e]);
      }
    T out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] = static_cast<T>(acc[e]);
    store8(dx + static_cast<int64_t>(row) * per_row * 8 + static_cast<int64_t>(t) * 8, out);
  }
}

PoolGeo make_geo(int64_t N, int64_t H, int64_t W, int64_t C, int K, int S, int P) {
  if (C % 8 != 0) throw std::runtime_error("maxpool: C % 8 == 0 required (got " + std::to_string(C) + ")");
  if (K < 1 || K * K > 255 || S < 1 || P < 0 || P >= K)
    throw std::runtime_error("maxpool: need 1 <= K, K*K <= 255, S >= 1, 0 <= P < K");
  PoolGeo g{N, H, W, C, (H + 2 * P - K) / S + 1, (W + 2 * P - K) / S + 1, K, S, P};
  if (g.OH < 1 || g.OW < 1) throw std::runtime_error("maxpool: empty output");
  if (N * H >= (int64_t(1) << 31) || W * (C / 8) >= (int64_t(1) << 31))
    throw std::runtime_error("maxpool: tensor too large for the row-per-workgroup grid");
  return g;
}

// Stem input channel pad: NHWC [P][3] 16-bit pixels -> [P][4] with a zero 4th channel, in one
// pass (read 6 B, write 8 B per pixel). A lane moves 8 pixels: three 16-byte loads, four
// 16-byte stores. (PyTorch's version is a strided fill plus a strided copy: ~80 us for a
// 256x224x224 batch on MI355X, s47 trace.)
union Vec48 {
  uint4 v[3];
  uint16_t h[24];
};
union Vec64 {
  uint4 v[4];
  uint16_t h[32];
};

__global__ __launch_bounds__(kThreads) void pad_c3_to_c4_kernel(const uint16_t* __restrict__ x,
                                                                uint16_t* __restrict__ y, int64_t npix) {
  const int64_t groups = npix / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; g < groups; g += stride) {
    Vec48 in;
    const uint4* src = reinterpret_cast<const uint4*>(x + g * 24);
#pragma unroll
    for (int i = 0; i < 3; ++i) in.v[i] = src[i];
    Vec64 out;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      out.h[4 * p] = in.h[3 * p];
      out.h[4 * p + 1] = in.h[3 * p + 1];
      out.h[4 * p + 2] = in.h[3 * p + 2];
      out.h[4 * p + 3] = 0;
    }
    uint4* dst = reinterpret_cast<uint4*>(y + g * 32);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = out.v[i];
  }
  // tail pixels (npix % 8), one per lane of the first workgroup
  if (blockIdx.x == 0 && threadIdx.x < (npix & 7)) {
    const int64_t p = groups * 8 + threadIdx.x;
#pragma unroll
    for (int c = 0; c < 3; ++c) y[p * 4 + c] = x[p * 3 + c];
    y[p * 4 + 3] = 0;
  }
}

}  // namespace

void pad_c3_to_c4(const void* x, void* y, int64_t npix, int dtype, hipStream_t s) {
  if (dtype != kBF16 && dtype != kF16) throw std::runtime_error("pad_c3_to_c4: bf16/fp16 only");
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) % 16 != 0)
    throw std::runtime_error("pad_c3_to_c4: x and y must be 16-byte aligned");
  if (npix <= 0) return;
  int64_t nb = (npix / 8 + kThreads - 1) / kThreads;
  if (nb < 1) nb = 1;
  if (nb > 65536) nb = 65536;
  pad_c3_to_c4_kernel<<<static_cast<unsigned>(nb), kThreads, 0, s>>>(static_cast<const uint16_t*>(x),
                                                                      static_cast<uint16_t*>(y), npix);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void bn_relu_maxpool_fwd(const void* x, const float* scale, const float* shift, void* y, uint8_t* idx, int64_t N,
                         int64_t H, int64_t W, int64_t C, int K, int S, int P, int dtype, hipStream_t s) {
  const PoolGeo g = make_geo(N, H, W, C, K, S, P);
  const int nb = static_cast<int>(N * g.OH);  // one workgroup per output row
  // one lane per (output column, 8 channels) of the row when it fits a workgroup (ResNet stem:
  // 56 x 8 = 448 lanes; a 256-lane workgroup looping over it left a quarter of its lanes idle)
  const int64_t per_row = g.OW * (C / 8);
  const int thr = per_row <= 1024 ? static_cast<int>((per_row + 63) / 64 * 64) : kThreads;
  switch (dtype) {
    case kBF16:
      if (g.K == 3 && !std::getenv("FLUXMPI_POOL_GENERIC"))
        bn_relu_maxpool_fwd_kernel<bf16, 3><<<nb, thr, 0, s>>>(static_cast<const bf16*>(x), scale, shift,
                                                                  static_cast<bf16*>(y), idx, g);
      else
        bn_relu_maxpool_fwd_kernel<bf16><<<nb, thr, 0, s>>>(static_cast<const bf16*>(x), scale, shift,
                                                                 static_cast<bf16*>(y), idx, g);
      break;
    case kF16:
      bn_relu_maxpool_fwd_kernel<f16><<<nb, thr, 0, s>>>(static_cast<const f16*>(x), scale, shift,
                                                              static_cast<f16*>(y), idx, g);
      break;
    case kF32:
      bn_relu_maxpool_fwd_kernel<float><<<nb, thr, 0, s>>>(static_cast<const float*>(x), scale, shift,
                                                                static_cast<float*>(y), idx, g);
      break;
    default:
      throw std::runtime_error("bn_relu_maxpool_fwd: unsupported dtype");
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int64_t N, int64_t H, int64_t W, int64_t C, int K,
                 int S, int P, int dtype, hipStream_t s) {
  const PoolGeo g = make_geo(N, H, W, C, K, S, P);
  const int nb = static_cast<int>(N * H);  // one workgroup per input row
  const int nw = (K + S - 1) / S;
#define POOL_BWD(T, NW)                                                                                         \
  maxpool_bwd_gather_kernel<T, NW><<<nb, kThreads, 0, s>>>(static_cast<const T*>(dy), idx, static_cast<T*>(dx), g)
#define POOL_BWD_NW(T)                              \
  {                                                 \
    if (nw == 1) POOL_BWD(T, 1);                    \
    else if (nw == 2) POOL_BWD(T, 2);               \
    else if (nw == 3) POOL_BWD(T, 3);               \
    else throw std::runtime_error("maxpool_bwd: ceil(K/S) > 3 unsupported"); \
  }
  switch (dtype) {
    case kBF16: POOL_BWD_NW(bf16) break;
    case kF16: POOL_BWD_NW(f16) break;
    case kF32: POOL_BWD_NW(float) break;
    default: throw std::runtime_error("maxpool_bwd: unsupported dtype");
  }
#undef POOL_BWD_NW
#undef POOL_BWD
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
