// 3x3 convolutions over a 3-channel image (an RGB stem: the CIFAR DEQ's stem1, models/deq.py) —
// forward and filter gradient, NHWC bf16, pad 1, stride 1 or 2, Cout a multiple of 128.
//
// Three input channels are below every implicit-GEMM kernel's channel granularity (an MFMA
// k-step is 16-32 deep; the whole reduction here is 27), so round 5 ran the forward on a CK
// grouped convolution (91 us) and the filter gradient dW[co][27] = dY^T im2col(X) as one
// hipBLASLt GEMM with K = 262,144 pixels and a 128 x 27 output: 2 output tiles on 256 CUs,
// 753 us. Both are bandwidth problems: the forward writes Y (67 MB at
// batch 256, 32 x 32, Cout 128), the filter gradient reads dY (the same 67 MB) — ~13 us each at
// HBM rate — and carry 0.9 GMAC each, ~7 us of packed-bf16 dot products (v_dot2_f32_bf16, two
// MACs per lane per instruction) spread over the chip.
//
// Layout of the work: a lane owns TWO output channels (64 lanes x 2 = 128 channels per
// workgroup column), so every global access of Y / dY is one dword per lane, 256 contiguous
// bytes per wave. The 27 taps x channels of a pixel's window are wave-uniform: they are staged
// once per workgroup in LDS and read back as broadcast ds_read_b128 (all lanes, one address).
//  * forward: LDS holds each pixel's window as 14 packed k-pairs (x[2j], x[2j+1]); a lane keeps
//    its two channels' filter as the matching 2 x 14 k-pairs in registers; one output = 14 dot2;
//  * filter gradient: LDS holds each PIXEL PAIR's window as 27 packed (x_p0[k], x_p1[k]); a
//    lane packs (dY_p0[co], dY_p1[co]) from two dword loads, so one dot2 accumulates two pixels
//    of one (co, k) product; 2 x 27 fp32 accumulators per lane; eight waves per workgroup, each
//    over 32 consecutive pixel pairs with the next 4 pairs' dY loads in flight while 4 compute
//    (measured 74 us without that pipeline: latency-bound at 2 waves per SIMD); the waves sum in
//    LDS and write one fp32 partial [Cout][27] per workgroup (reduced by gemm_splitk_reduce into
//    the filter's bucket slice).
// Window values outside the image (padding) are zeros written by the staging loop, so the inner
// loops carry no bounds logic.
#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

constexpr int kCin = 3;
constexpr int kTaps = 9 * kCin;       // 27
constexpr int kPairsK = (kTaps + 1) / 2;  // 14 k-pairs (the 28th k is a zero)
constexpr int kFwdPx = 256;           // pixels per forward workgroup
constexpr int kFwdRow = 16;           // LDS dwords per pixel window (14 used; 64-B rows for b128 reads)
constexpr int kWgPx = 512;            // pixels per filter-gradient workgroup (256 pixel pairs)
constexpr int kWgRow = 28;            // LDS dwords per pixel-pair window (27 used; 112-B rows)

struct C3Geo {
  int H, W, Ho, Wo, stride;
  int64_t pixels;  // N * Ho * Wo
};

__device__ __forceinline__ uint32_t as_u32(bf16x2_t v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ bf16x2_t as_b2(uint32_t v) { return __builtin_bit_cast(bf16x2_t, v); }

// Row-major window of output pixel ``px``: ``base`` = the element (kh = kw = ci = 0) offset,
// ``rok`` / ``cok`` = bit masks of the 3 rows / 3 columns inside the image.
struct Win {
  int64_t base;
  int rok, cok;
};

__device__ __forceinline__ Win window_of(int64_t px, const C3Geo& g) {
  Win w{0, 0, 0};
  if (px >= g.pixels) return w;  // a padding pixel: all zeros
  const int64_t hw = static_cast<int64_t>(g.Ho) * g.Wo;
  const int64_t n = px / hw;
  const int r = static_cast<int>(px - n * hw);
  const int oh = r / g.Wo, ow = r - oh * g.Wo;
  const int ih0 = oh * g.stride - 1, iw0 = ow * g.stride - 1;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    w.rok |= (ih0 + t >= 0 && ih0 + t < g.H) << t;
    w.cok |= (iw0 + t >= 0 && iw0 + t < g.W) << t;
  }
  w.base = ((n * g.H + ih0) * g.W + iw0) * kCin;
  return w;
}

// element k (= (kh * 3 + kw) * 3 + ci) of the window, as raw bf16 bits (0 outside the image)
__device__ __forceinline__ uint32_t wval(const uint16_t* __restrict__ x, const Win& w, int k, int W) {
  const int kh = k / 9, kw = (k / 3) % 3, ci = k % 3;
  if (!((w.rok >> kh) & 1) || !((w.cok >> kw) & 1)) return 0u;
  return x[w.base + (static_cast<int64_t>(kh) * W + kw) * kCin + ci];
}

__global__ __launch_bounds__(256) void c3_fwd_kernel(const uint16_t* __restrict__ x, const uint32_t* __restrict__ wt,
                                                      uint32_t* __restrict__ y, C3Geo g, int co_total) {
  __shared__ __attribute__((aligned(16))) uint32_t win[kFwdPx * kFwdRow];
  const int64_t p0 = static_cast<int64_t>(blockIdx.x) * kFwdPx;
  {
    // one pixel per thread: its 14 k-pairs (k = 27 is the zero pad)
    const Win w = window_of(p0 + threadIdx.x, g);
    uint32_t v[kFwdRow];
#pragma unroll
    for (int j = 0; j < kPairsK; ++j) {
      const uint32_t lo = wval(x, w, 2 * j, g.W);
      const uint32_t hi = 2 * j + 1 < kTaps ? wval(x, w, 2 * j + 1, g.W) : 0u;
      v[j] = lo | (hi << 16);
    }
    v[14] = v[15] = 0u;
    uint4* dst = reinterpret_cast<uint4*>(win + threadIdx.x * kFwdRow);
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int co = blockIdx.y * 128 + 2 * lane;
  // the lane's two filters as k-pairs: wt is [Cout][14] packed pairs (k 27 = 0), prepared on the host
  bf16x2_t f0[kPairsK], f1[kPairsK];
#pragma unroll
  for (int j = 0; j < kPairsK; ++j) {
    f0[j] = as_b2(wt[static_cast<int64_t>(co) * kPairsK + j]);
    f1[j] = as_b2(wt[static_cast<int64_t>(co + 1) * kPairsK + j]);
  }
  __syncthreads();
  const int np = static_cast<int>(min<int64_t>(kFwdPx, g.pixels - p0));
  for (int p = wave; p < np; p += 4) {
    const uint4* src = reinterpret_cast<const uint4*>(win + p * kFwdRow);
    uint32_t v[kFwdRow];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 t = src[q];
      v[4 * q] = t.x, v[4 * q + 1] = t.y, v[4 * q + 2] = t.z, v[4 * q + 3] = t.w;
    }
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int j = 0; j < kPairsK; ++j) {
      a0 = __builtin_amdgcn_fdot2_f32_bf16(f0[j], as_b2(v[j]), a0, false);
      a1 = __builtin_amdgcn_fdot2_f32_bf16(f1[j], as_b2(v[j]), a1, false);
    }
    const bf16x2_t o = {static_cast<bf16>(a0), static_cast<bf16>(a1)};
    y[((p0 + p) * co_total + co) >> 1] = as_u32(o);
  }
}

constexpr int kWgThreads = 512;  // 8 waves: each owns 32 consecutive pixel pairs of the chunk
constexpr int kWgU = 4;          // pixel pairs per load group (8 dword loads in flight per lane)

__device__ __forceinline__ void load_dy(const uint32_t* __restrict__ dy, int64_t px, int64_t pixels, int64_t row,
                                        int cd, uint32_t& d0, uint32_t& d1) {
  // clamped addresses + value selects, no branch around a load (a branch per element makes hipcc
  // wait vmcnt(0) at each one: cdna_hip_programming.md, projection GEMM trap (c))
  const int64_t a = px < pixels ? px : pixels - 1, b = px + 1 < pixels ? px + 1 : pixels - 1;
  d0 = dy[a * row + cd];
  d1 = dy[b * row + cd];
  d0 = px < pixels ? d0 : 0u;
  d1 = px + 1 < pixels ? d1 : 0u;
}

__global__ __launch_bounds__(kWgThreads) void c3_wgrad_kernel(const uint16_t* __restrict__ x, const uint32_t* __restrict__ dy,
                                                               float* __restrict__ part, C3Geo g, int co_total) {
  __shared__ __attribute__((aligned(16))) uint32_t win[(kWgPx / 2) * kWgRow];
  const int64_t p0 = static_cast<int64_t>(blockIdx.x) * kWgPx;
  if (threadIdx.x < kWgPx / 2) {
    // one pixel pair per thread: 27 packed (x_p0[k], x_p1[k])
    const Win w0 = window_of(p0 + 2 * threadIdx.x, g), w1 = window_of(p0 + 2 * threadIdx.x + 1, g);
    uint32_t v[kWgRow];
#pragma unroll
    for (int k = 0; k < kTaps; ++k) v[k] = wval(x, w0, k, g.W) | (wval(x, w1, k, g.W) << 16);
    v[27] = 0u;
    uint4* dst = reinterpret_cast<uint4*>(win + threadIdx.x * kWgRow);
#pragma unroll
    for (int q = 0; q < kWgRow / 4; ++q) dst[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int co = blockIdx.y * 128 + 2 * lane;
  const int64_t row = co_total >> 1;  // dwords per dY row
  constexpr int kPerWave = kWgPx / 2 / (kWgThreads / 64);  // 32 pairs
  const int pp0 = wave * kPerWave;
  float acc0[kTaps], acc1[kTaps];
#pragma unroll
  for (int k = 0; k < kTaps; ++k) acc0[k] = acc1[k] = 0.f;
  // software pipeline: the next group's dY loads are in flight while this group computes
  uint32_t cur[kWgU][2], nxt[kWgU][2];
#pragma unroll
  for (int u = 0; u < kWgU; ++u) load_dy(dy, p0 + 2 * (pp0 + u), g.pixels, row, co >> 1, cur[u][0], cur[u][1]);
  __syncthreads();
  for (int i = 0; i < kPerWave; i += kWgU) {
    if (i + kWgU < kPerWave) {
#pragma unroll
      for (int u = 0; u < kWgU; ++u)
        load_dy(dy, p0 + 2 * (pp0 + i + kWgU + u), g.pixels, row, co >> 1, nxt[u][0], nxt[u][1]);
    }
#pragma unroll
    for (int u = 0; u < kWgU; ++u) {
      const uint32_t d0 = cur[u][0], d1 = cur[u][1];
      // (dY_p0[co], dY_p1[co]) and (dY_p0[co + 1], dY_p1[co + 1])
      const bf16x2_t a0 = as_b2((d0 & 0xffffu) | (d1 << 16));
      const bf16x2_t a1 = as_b2((d0 >> 16) | (d1 & 0xffff0000u));
      const uint4* src = reinterpret_cast<const uint4*>(win + (pp0 + i + u) * kWgRow);
      uint32_t v[kWgRow];
#pragma unroll
      for (int q = 0; q < kWgRow / 4; ++q) {
        const uint4 t = src[q];
        v[4 * q] = t.x, v[4 * q + 1] = t.y, v[4 * q + 2] = t.z, v[4 * q + 3] = t.w;
      }
#pragma unroll
      for (int k = 0; k < kTaps; ++k) {
        acc0[k] = __builtin_amdgcn_fdot2_f32_bf16(a0, as_b2(v[k]), acc0[k], false);
        acc1[k] = __builtin_amdgcn_fdot2_f32_bf16(a1, as_b2(v[k]), acc1[k], false);
      }
    }
#pragma unroll
    for (int u = 0; u < kWgU; ++u) cur[u][0] = nxt[u][0], cur[u][1] = nxt[u][1];
  }
  // the eight waves' sums: LDS float adds over the (now free) window buffer [128][27]
  __syncthreads();
  float* red = reinterpret_cast<float*>(win);
  for (int i = threadIdx.x; i < 128 * kTaps; i += kWgThreads) red[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kTaps; ++k) {
    atomicAdd(red + (2 * lane) * kTaps + k, acc0[k]);
    atomicAdd(red + (2 * lane + 1) * kTaps + k, acc1[k]);
  }
  __syncthreads();
  float* out = part + (static_cast<int64_t>(blockIdx.x) * co_total + blockIdx.y * 128) * kTaps;
  for (int i = threadIdx.x; i < 128 * kTaps; i += kWgThreads) out[i] = red[i];
}

C3Geo geo(int H, int W, int stride, int64_t N) {
  C3Geo g{};
  g.H = H, g.W = W, g.stride = stride;
  g.Ho = (H + 2 - 3) / stride + 1, g.Wo = (W + 2 - 3) / stride + 1;
  g.pixels = N * g.Ho * g.Wo;
  return g;
}

void check(const void* a, const void* b, const void* c, int64_t N, int H, int W, int stride, int Cout) {
  if (!conv_c3_supported(N, H, W, stride, Cout))
    throw std::runtime_error("conv_c3: unsupported shape (3 input channels, 3x3, pad 1, stride 1/2, Cout % 128 == 0)");
  if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 3u) != 0)
    throw std::runtime_error("conv_c3: operands must be 4-byte aligned");
}

}  // namespace

bool conv_c3_supported(int64_t N, int H, int W, int stride, int Cout) {
  if (N < 1 || H < 1 || W < 1 || (stride != 1 && stride != 2) || Cout < 128 || Cout % 128 != 0 || Cout > 8192)
    return false;
  const C3Geo g = geo(H, W, stride, N);
  return g.pixels > 0 && g.pixels * Cout < (int64_t(1) << 40) && N * H * W * kCin < (int64_t(1) << 40);
}

int64_t conv_c3_wgrad_blocks(int64_t N, int H, int W, int stride) {
  const C3Geo g = geo(H, W, stride, N);
  return (g.pixels + kWgPx - 1) / kWgPx;
}

void conv_c3_fwd(const void* x, const void* w_pairs, void* y, int64_t N, int H, int W, int stride, int Cout,
                 hipStream_t stream) {
  check(x, w_pairs, y, N, H, W, stride, Cout);
  const C3Geo g = geo(H, W, stride, N);
  const dim3 grid(static_cast<unsigned>((g.pixels + kFwdPx - 1) / kFwdPx), static_cast<unsigned>(Cout / 128));
  c3_fwd_kernel<<<grid, 256, 0, stream>>>(static_cast<const uint16_t*>(x), static_cast<const uint32_t*>(w_pairs),
                                          static_cast<uint32_t*>(y), g, Cout);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void conv_c3_wgrad(const void* x, const void* dy, float* part, int64_t N, int H, int W, int stride, int Cout,
                   hipStream_t stream) {
  check(x, dy, part, N, H, W, stride, Cout);
  const C3Geo g = geo(H, W, stride, N);
  const dim3 grid(static_cast<unsigned>((g.pixels + kWgPx - 1) / kWgPx), static_cast<unsigned>(Cout / 128));
  c3_wgrad_kernel<<<grid, kWgThreads, 0, stream>>>(static_cast<const uint16_t*>(x), static_cast<const uint32_t*>(dy), part,
                                            g, Cout);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
