// Fused NHWC BatchNorm (+ReLU, +residual add) for gfx950.
//
// ResNet-50's non-GEMM time is dominated by memory passes over activations:
// eager BatchNorm + ReLU + residual add + ReLU costs ~7 passes forward and
// ~10 backward. These kernels cut that to 2 forward (stats read; normalise
// read + write) and 2 backward (reduce read; dx read + write) passes.
//
// Layout: x is [R, C] row-major (R = N*H*W, channels innermost = NHWC /
// channels_last), C % 8 == 0. Each lane owns 8 consecutive channels of one
// row (one 16 B vector for bf16/fp16), so every access is a full-width
// coalesced global_load_dwordx4.
//
// Reductions: a workgroup accumulates fp32 per-channel partials over its rows
// in registers, reduces the lanes that share a channel vector through LDS and
// adds its partial to one of 64 shards of a [64][2][C] fp32 accumulator with
// global float atomics. A tiny finalize kernel sums the shards into the
// per-channel statistics (and re-zeroes them, so the persistent workspace
// needs no memset per call); the consumer kernels derive their per-channel
// coefficients from those statistics (registers, or LDS when C/8 does not divide
// the workgroup). Grids are one full round of resident workgroups (occupancy x CUs).
#include <cstdlib>
#include <initializer_list>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxC = 2048;

template <typename T>
struct V8 {
  T v[8];
};

template <typename T>
__device__ __forceinline__ void ld8f(const T* __restrict__ p, float (&f)[8]) {
  T t[8];
  load8(p, t);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = static_cast<float>(t[j]);
}

template <typename T>
__device__ __forceinline__ void st8f(T* __restrict__ p, const float (&f)[8]) {
  T t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = static_cast<T>(f[j]);
  store8(p, t);
}

// 8 consecutive per-channel floats (c0 % 8 == 0, 16-B aligned array) with two 16-B loads:
// the lanes of a wave read consecutive 32-B pieces, where 8 scalar loads per lane would each
// touch a different cache line (a kernel-wide prologue that alone cost ~25 us per launch)
__device__ __forceinline__ void ld8ch(const float* __restrict__ p, int c0, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p + c0);
  const float4 b = *reinterpret_cast<const float4*>(p + c0 + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

struct Geo {
  int cv;    // channel vectors per row (C / 8)
  int rpi;   // rows handled concurrently by a workgroup (kThreads / cv)
  int64_t rows_per_block;
  int blocks;
};

Geo geometry(int64_t rows, int64_t C, int64_t max_blocks = 2048) {
  Geo g;
  g.cv = static_cast<int>(C / 8);
  g.rpi = kThreads / g.cv;
  if (g.rpi < 1) g.rpi = 1;
  // >= 32K elements per workgroup, at most one full round of resident workgroups
  int64_t min_rows = (32768 + C - 1) / C;
  int64_t blocks = (rows + min_rows - 1) / min_rows;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  int64_t rpb = (rows + blocks - 1) / blocks;
  rpb = (rpb + g.rpi - 1) / g.rpi * g.rpi;
  g.rows_per_block = rpb;
  g.blocks = static_cast<int>((rows + rpb - 1) / rpb);
  return g;
}

// Block-level reduction of two 8-float accumulators over lanes sharing a
// channel vector, then one atomic per channel per workgroup into shard
// (blockIdx % kShards) of acc[kShards][2][C]. Sharding keeps the number of
// same-address atomics per line ~blocks/kShards: float atomics execute at the
// memory side, and thousands of workgroups adding into ONE line serialise.
constexpr int kShards = 64;  // <= ~200 same-address atomics even for 12k-block GEMM grids
// The row-reduction kernels here run at most one round of resident workgroups (<= 2048): 16
// shards keep <= 128 same-address atomics and make the finalize kernel's read 4x smaller.
constexpr int kRedShards = 16;

__device__ __forceinline__ void block_reduce_atomic(float (&a)[8], float (&b)[8], int cv, int rpi, int C,
                                                    float* __restrict__ acc, float* smem) {
  const int t = threadIdx.x;
  const int r0 = t / cv, c8 = t % cv;
  const bool active = r0 < rpi;
  float* sa = smem;
  float* sb = smem + rpi * C;
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa[r0 * C + c8 * 8 + j] = a[j];
      sb[r0 * C + c8 * 8 + j] = b[j];
    }
  }
  __syncthreads();
  float* shard = acc + static_cast<size_t>(blockIdx.x % kRedShards) * 2 * C;
  for (int c = t; c < C; c += kThreads) {
    float x = 0.f, y = 0.f;
    for (int r = 0; r < rpi; ++r) {
      x += sa[r * C + c];
      y += sb[r * C + c];
    }
    atomicAdd(shard + c, x);
    atomicAdd(shard + C + c, y);
  }
}

// Sum the shards of a channel and re-zero them (the workspace is left zeroed for the next call,
// so no memset is needed per launch). A finalize workgroup is 64 channels x 4 shard groups:
// each lane sums 16 shards of one channel (independent loads, all issued before the zeroing
// stores), the 4 partial sums meet in LDS. (One lane per channel walking all 64 shards was a
// chain of dependent L2 round trips: ~5 us per launch, 106 launches per ResNet-50 step.)
constexpr int kFinCh = 64, kFinGroups = 4, kFinPer = kShards / kFinGroups;

__device__ __forceinline__ bool take_shards(float* __restrict__ acc, int C, float& a, float& b, int& c_out) {
  __shared__ float red[2][kFinGroups][kFinCh];
  const int cl = threadIdx.x % kFinCh, g = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    float va[kFinPer], vb[kFinPer];
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
      const float* sh = acc + static_cast<size_t>(g * kFinPer + k) * 2 * C;
      va[k] = sh[c];
      vb[k] = sh[C + c];
    }
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
      sa += va[k];
      sb += vb[k];
    }
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
      float* sh = acc + static_cast<size_t>(g * kFinPer + k) * 2 * C;
      sh[c] = 0.f;
      sh[C + c] = 0.f;
    }
  }
  red[0][g][cl] = sa;
  red[1][g][cl] = sb;
  __syncthreads();
  c_out = c;
  if (g != 0 || c >= C) return false;
  a = (red[0][0][cl] + red[0][1][cl]) + (red[0][2][cl] + red[0][3][cl]);
  b = (red[1][0][cl] + red[1][1][cl]) + (red[1][2][cl] + red[1][3][cl]);
  return true;
}

int finalize_blocks(int64_t C) { return static_cast<int>((C + kFinCh - 1) / kFinCh); }

__global__ __launch_bounds__(kFinCh * kFinGroups) void bn_finalize_fwd_kernel(
    float* __restrict__ acc, int C, int64_t rows, float momentum, float eps, float* __restrict__ smean,
    float* __restrict__ sinv, float* __restrict__ rmean, float* __restrict__ rvar, const float* __restrict__ w,
    const float* __restrict__ b, float* __restrict__ scale, float* __restrict__ shift, int64_t* __restrict__ nbt) {
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;  // num_batches_tracked, no launch of its own
  float s, q;
  int c;
  if (!take_shards(acc, C, s, q, c)) return;
  const float inv_n = 1.f / static_cast<float>(rows);
  const float mean = s * inv_n;
  float var = q * inv_n - mean * mean;
  var = var > 0.f ? var : 0.f;
  const float invstd = rsqrtf(var + eps);
  smean[c] = mean;
  sinv[c] = invstd;
  if (scale != nullptr) {  // the affine a consumer GEMM applies on load (bit-identical to bn_norm_kernel)
    const float sc = (w ? w[c] : 1.f) * invstd;
    scale[c] = sc;
    shift[c] = fmaf(-mean, sc, b ? b[c] : 0.f);
  }
  if (rmean != nullptr) {
    const float unbiased = rows > 1 ? var * static_cast<float>(rows) / static_cast<float>(rows - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unbiased;
  }
}

__global__ __launch_bounds__(kFinCh * kFinGroups) void bn_finalize_bwd_kernel(float* __restrict__ acc, int C,
                                                                              float* __restrict__ dw,
                                                                              float* __restrict__ db) {
  float s, q;
  int c;
  if (!take_shards(acc, C, s, q, c)) return;
  db[c] = s;  // sum(dy_eff)
  dw[c] = q;  // sum(dy_eff * xhat)
}

// the dual (bn3 + downsample) backward's two finalizes in one launch: blockIdx.y picks the workspace
__global__ __launch_bounds__(kFinCh * kFinGroups) void bn_finalize_bwd2_kernel(float* __restrict__ acc, float* __restrict__ acc2,
                                                                               int C, float* __restrict__ dw,
                                                                               float* __restrict__ db, float* __restrict__ dw2,
                                                                               float* __restrict__ db2) {
  float s, q;
  int c;
  const bool second = blockIdx.y != 0;
  if (!take_shards(second ? acc2 : acc, C, s, q, c)) return;
  (second ? db2 : db)[c] = s;
  (second ? dw2 : dw)[c] = q;
}

// ---------------------------------------------------------------- forward
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const T* __restrict__ x, int64_t rows, int C, Geo g,
                                                            float* __restrict__ acc) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = threadIdx.x;
  const int r0 = t / g.cv, c8 = t % g.cv;
  float s[8] = {0}, q[8] = {0};
  if (r0 < g.rpi) {
    const int64_t start = static_cast<int64_t>(blockIdx.x) * g.rows_per_block;
    int64_t end = start + g.rows_per_block;
    if (end > rows) end = rows;
    int64_t r = start + r0;
    // 8 rows (8 x 16 B) in flight per lane: the reduction is latency bound otherwise
    constexpr int U = 8;
    for (; r + (U - 1) * g.rpi < end; r += U * g.rpi) {
      T raw[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) load8(x + (r + u * g.rpi) * C + c8 * 8, raw[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = static_cast<float>(raw[u][j]);
          s[j] += f;
          q[j] = fmaf(f, f, q[j]);
        }
    }
    for (; r < end; r += g.rpi) {
      float f[8];
      ld8f(x + r * C + c8 * 8, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += f[j];
        q[j] = fmaf(f[j], f[j], q[j]);
      }
    }
  }
  block_reduce_atomic(s, q, g.cv, g.rpi, C, acc, smem);
}

// y = act(x*scale + shift [+ res]); scale/shift derived from (mean, invstd) = batch
// statistics (training) or running statistics (eval).
// FIXED (C/8 divides the 256-lane workgroup): the grid stride is a multiple of C/8, so
// every lane keeps the same 8 channels for the whole kernel and holds its coefficients
// in registers; otherwise they are staged in LDS and indexed per vector.
// Two vectors per lane per iteration (loads of both issued before any math).
template <typename T, bool RELU, bool RES>
__device__ __forceinline__ void norm_vec(float (&f)[8], const float (&rr)[8], const float* sc, const float* sh,
                                         unsigned& bits) {
  bits = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float o = fmaf(f[j], sc[j], sh[j]);  // explicit fma: backward recomputes it bit-identically
    if (RES) o += rr[j];
    if (RELU) {
      bits |= (o > 0.f ? 1u : 0u) << j;
      o = o > 0.f ? o : 0.f;
    }
    f[j] = o;
  }
}

template <typename T, bool RELU, bool RES, bool FIXED, int U = 2>
__global__ __launch_bounds__(kThreads) void bn_norm_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                           const T* __restrict__ res, const float* __restrict__ w,
                                                           const float* __restrict__ b,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ stat2, int C, float eps,
                                                           int train, int64_t nvec, uint8_t* __restrict__ mask) {
  // mask (optional, RELU only): bit j of byte v = (element 8v+j > 0). One byte per
  // 8 elements lets the backward apply the ReLU of a residual block without
  // re-reading y (2 B/element -> 1/8 B/element).
  extern __shared__ __attribute__((aligned(16))) float smem[];
  auto coef = [&](int c, float& sc, float& sh) {
    const float mean = mean_in[c];
    const float invstd = train ? stat2[c] : rsqrtf(stat2[c] + eps);  // save_invstd | running_var
    sc = (w ? w[c] : 1.f) * invstd;
    sh = fmaf(-mean, sc, b ? b[c] : 0.f);
  };
  float rsc[8], rsh[8];
  if (FIXED) {
    const int c0 = (threadIdx.x % (C / 8)) * 8;
    float mu[8], s2[8], ww[8], bb[8];
    ld8ch(mean_in, c0, mu);
    ld8ch(stat2, c0, s2);
    // unconditional (a stand-in source when absent): a load under `if (w)` is waited for at the
    // join, one exposed latency each before the streaming starts
    ld8ch(w ? w : mean_in, c0, ww);
    ld8ch(b ? b : mean_in, c0, bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float invstd = train ? s2[j] : rsqrtf(s2[j] + eps);  // save_invstd | running_var
      rsc[j] = (w ? ww[j] : 1.f) * invstd;
      rsh[j] = fmaf(-mu[j], rsc[j], b ? bb[j] : 0.f);
    }
  } else {
    for (int c = threadIdx.x; c < C; c += kThreads) coef(c, smem[c], smem[C + c]);
    __syncthreads();
  }
  // U vectors per lane per iteration, every load issued before any math
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (; v + (U - 1) * stride < nvec; v += U * stride) {
    float f[U][8], r[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ld8f(x + (v + u * stride) * 8, f[u]);
      if (RES) ld8f(res + (v + u * stride) * 8, r[u]);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every load ahead of the first store
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t vu = v + u * stride;
      unsigned bits;
      norm_vec<T, RELU, RES>(f[u], r[u], FIXED ? rsc : smem + (vu * 8) % C, FIXED ? rsh : smem + C + (vu * 8) % C,
                             bits);
      st8f(y + vu * 8, f[u]);
      if (RELU && mask != nullptr) mask[vu] = static_cast<uint8_t>(bits);
    }
  }
  for (; v < nvec; v += stride) {
    float f0[8], r0[8];
    ld8f(x + v * 8, f0);
    if (RES) ld8f(res + v * 8, r0);
    unsigned b0;
    norm_vec<T, RELU, RES>(f0, r0, FIXED ? rsc : smem + (v * 8) % C, FIXED ? rsh : smem + C + (v * 8) % C, b0);
    st8f(y + v * 8, f0);
    if (RELU && mask != nullptr) mask[v] = static_cast<uint8_t>(b0);
  }
}

// ---------------------------------------------------------------- backward
// acc[0:C] += sum(dy_eff), acc[C:2C] += sum(dy_eff * xhat)
// RM (ReLU mode): 0 none; 1 mask from the saved output y (needed when a residual
// was added before the ReLU); 2 mask recomputed from x as fmaf(x, scale, shift) > 0
// with scale/shift computed bit-identically to the forward prologue, so y is
// neither saved nor re-read (one fewer activation read per element, both passes).
template <typename T, int RM>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                 const T* __restrict__ y,
                                                                 const uint8_t* __restrict__ mask,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ b,
                                                                 const float* __restrict__ smean,
                                                                 const float* __restrict__ sinv, int64_t rows, int C,
                                                                 Geo g, float* __restrict__ acc) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = threadIdx.x;
  const int r0 = t / g.cv, c8 = t % g.cv;
  float s[8] = {0}, q[8] = {0};
  if (r0 < g.rpi) {
    float mu[8], is[8], sc[8], sh[8], ww[8], bb[8];
    ld8ch(smean, c8 * 8, mu);
    ld8ch(sinv, c8 * 8, is);
    ld8ch(w ? w : smean, c8 * 8, ww);  // unconditional: see bn_norm_kernel
    ld8ch(b ? b : smean, c8 * 8, bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = (w ? ww[j] : 1.f) * is[j];
      sh[j] = fmaf(-mu[j], sc[j], b ? bb[j] : 0.f);
    }
    const int64_t start = static_cast<int64_t>(blockIdx.x) * g.rows_per_block;
    int64_t end = start + g.rows_per_block;
    if (end > rows) end = rows;
    int64_t r = start + r0;
    constexpr int U = 4;  // 4 rows x (2|3) tensors of 16 B loads in flight per lane
    for (; r + (U - 1) * g.rpi < end; r += U * g.rpi) {
      T d[U][8], xv[U][8], yv[U][8];
      unsigned mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t off = (r + u * g.rpi) * C + c8 * 8;
        load8(dy + off, d[u]);
        load8(x + off, xv[u]);
        if (RM == 1) load8(y + off, yv[u]);
        if (RM == 3) mb[u] = mask[off >> 3];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float dd = static_cast<float>(d[u][j]);
          const float xf = static_cast<float>(xv[u][j]);
          if (RM == 1) dd = static_cast<float>(yv[u][j]) > 0.f ? dd : 0.f;
          if (RM == 2) dd = fmaf(xf, sc[j], sh[j]) > 0.f ? dd : 0.f;
          if (RM == 3) dd = (mb[u] >> j) & 1u ? dd : 0.f;
          s[j] += dd;
          q[j] = fmaf(dd, (xf - mu[j]) * is[j], q[j]);
        }
    }
    for (; r < end; r += g.rpi) {
      const int64_t off = r * C + c8 * 8;
      float d[8], xv[8], yv[8];
      ld8f(dy + off, d);
      ld8f(x + off, xv);
      if (RM == 1) ld8f(y + off, yv);
      const unsigned mbs = RM == 3 ? mask[off >> 3] : 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float dd = d[j];
        if (RM == 1) dd = yv[j] > 0.f ? dd : 0.f;
        if (RM == 2) dd = fmaf(xv[j], sc[j], sh[j]) > 0.f ? dd : 0.f;
        if (RM == 3) dd = (mbs >> j) & 1u ? dd : 0.f;
        s[j] += dd;
        q[j] = fmaf(dd, (xv[j] - mu[j]) * is[j], q[j]);
      }
    }
  }
  block_reduce_atomic(s, q, g.cv, g.rpi, C, acc, smem);
}

// dx = w*invstd * (dy_eff - sum_dy/R - xhat * sum_dy_xhat/R); dres = dy_eff
// (sum_dy = db, sum_dy_xhat = dw, produced by bn_finalize_bwd_kernel), evaluated as
// dx = A*dy_eff + B*x + D with per-channel A = w*invstd, B = -A*invstd*mean(dy_eff*xhat),
// D = A*(mean*invstd*mean(dy_eff*xhat) - mean(dy_eff)). Coefficients in registers
// (FIXED) or LDS as in bn_norm_kernel; two vectors per lane per iteration.
struct DxCoef {
  float a, b, d, sh;  // sh: forward shift (RM == 2 mask recompute, with a == forward scale)
};

__device__ __forceinline__ DxCoef dx_coef(int c, const float* __restrict__ w, const float* __restrict__ bias,
                                          const float* __restrict__ smean, const float* __restrict__ sinv,
                                          const float* __restrict__ dw, const float* __restrict__ db, float inv_n) {
  const float iv = sinv[c], m = smean[c];
  const float sc = (w ? w[c] : 1.f) * iv;
  const float k2 = db[c] * inv_n, k3 = dw[c] * inv_n;
  DxCoef k;
  k.a = sc;
  k.b = -sc * iv * k3;
  k.d = sc * (m * iv * k3 - k2);
  k.sh = fmaf(-m, sc, bias ? bias[c] : 0.f);
  return k;
}

template <typename T, int RM, bool DRES>
__device__ __forceinline__ void dx_vec(float (&d)[8], float (&xv)[8], const float (&yv)[8], unsigned mbs,
                                       const DxCoef* k) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float dd = d[j];
    if (RM == 1) dd = yv[j] > 0.f ? dd : 0.f;
    if (RM == 3) dd = (mbs >> j) & 1u ? dd : 0.f;
    if (RM == 2) dd = fmaf(xv[j], k[j].a, k[j].sh) > 0.f ? dd : 0.f;
    d[j] = dd;
    xv[j] = fmaf(k[j].a, dd, fmaf(k[j].b, xv[j], k[j].d));
  }
}

template <typename T, int RM, bool DRES, bool FIXED, int U = 2>
__global__ __launch_bounds__(kThreads) void bn_bwd_dx_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                             const T* __restrict__ y,
                                                             const uint8_t* __restrict__ mask,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ smean,
                                                             const float* __restrict__ sinv,
                                                             const float* __restrict__ dw,
                                                             const float* __restrict__ db, T* __restrict__ dx,
                                                             T* __restrict__ dres, int64_t rows, int C,
                                                             int64_t nvec) {
  extern __shared__ __attribute__((aligned(16))) DxCoef ksm[];
  const float inv_n = 1.f / static_cast<float>(rows);
  DxCoef rk[8];
  if (FIXED) {
    const int c0 = (threadIdx.x % (C / 8)) * 8;
    float iv[8], m[8], ww[8], bb[8], kdb[8], kdw[8];
    ld8ch(sinv, c0, iv);
    ld8ch(smean, c0, m);
    ld8ch(db, c0, kdb);
    ld8ch(dw, c0, kdw);
    ld8ch(w ? w : smean, c0, ww);  // unconditional: see bn_norm_kernel
    ld8ch(bias ? bias : smean, c0, bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // == dx_coef, from vector loads
      const float sc = (w ? ww[j] : 1.f) * iv[j];
      const float k2 = kdb[j] * inv_n, k3 = kdw[j] * inv_n;
      rk[j].a = sc;
      rk[j].b = -sc * iv[j] * k3;
      rk[j].d = sc * (m[j] * iv[j] * k3 - k2);
      rk[j].sh = fmaf(-m[j], sc, bias ? bb[j] : 0.f);
    }
  } else {
    for (int c = threadIdx.x; c < C; c += kThreads) ksm[c] = dx_coef(c, w, bias, smean, sinv, dw, db, inv_n);
    __syncthreads();
  }
  // U vectors per lane per iteration, every load issued before any math
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (; v + (U - 1) * stride < nvec; v += U * stride) {
    float d[U][8], xv[U][8], yv[U][8];
    unsigned mb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t vu = v + u * stride;
      ld8f(dy + vu * 8, d[u]);
      ld8f(x + vu * 8, xv[u]);
      if (RM == 1) ld8f(y + vu * 8, yv[u]);
      mb[u] = RM == 3 ? mask[vu] : 0u;
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every load ahead of the first store
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t vu = v + u * stride;
      dx_vec<T, RM, DRES>(d[u], xv[u], yv[u], mb[u], FIXED ? rk : ksm + (vu * 8) % C);
      st8f(dx + vu * 8, xv[u]);
      if (DRES) st8f(dres + vu * 8, d[u]);
    }
  }
  for (; v < nvec; v += stride) {
    float d0[8], x0[8], y0[8];
    ld8f(dy + v * 8, d0);
    ld8f(x + v * 8, x0);
    if (RM == 1) ld8f(y + v * 8, y0);
    const unsigned m0 = RM == 3 ? mask[v] : 0u;
    dx_vec<T, RM, DRES>(d0, x0, y0, m0, FIXED ? rk : ksm + (v * 8) % C);
    st8f(dx + v * 8, x0);
    if (DRES) st8f(dres + v * 8, d0);
  }
}

// ---------------------------------------------------------------- dual (downsample block)
// y = relu(BN_a(x) + BN_b(x2)): a ResNet downsample block's bn3 with the downsample branch's
// BatchNorm folded into the residual read. The branch output BN_b(x2) is never materialised:
// forward saves one write + one read per element, backward computes both input gradients in
// one pass from (dy, relu mask, x, x2) (dy_eff is the same for both BatchNorms) instead of
// bn3 writing dres and the branch BN reading it twice. FIXED channel mapping only
// (C/8 divides the workgroup), per-lane coefficients of both BatchNorms in registers.
__device__ __forceinline__ void coef8(const float* __restrict__ w, const float* __restrict__ b,
                                      const float* __restrict__ mean, const float* __restrict__ inv, int c0,
                                      float (&sc)[8], float (&sh)[8]) {
  float mu[8], iv[8], ww[8], bb[8];
  ld8ch(mean, c0, mu);
  ld8ch(inv, c0, iv);
  ld8ch(w ? w : mean, c0, ww);  // unconditional: see bn_norm_kernel
  ld8ch(b ? b : mean, c0, bb);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = (w ? ww[j] : 1.f) * iv[j];
    sh[j] = fmaf(-mu[j], sc[j], b ? bb[j] : 0.f);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void bn_norm_dual_kernel(
    const T* __restrict__ x, const T* __restrict__ x2, T* __restrict__ y, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ mean, const float* __restrict__ inv,
    const float* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ mean2,
    const float* __restrict__ inv2, int C, int64_t nvec, uint8_t* __restrict__ mask) {
  const int c0 = (threadIdx.x % (C / 8)) * 8;
  float sc[8], sh[8], sc2[8], sh2[8];
  coef8(w, b, mean, inv, c0, sc, sh);
  coef8(w2, b2, mean2, inv2, c0, sc2, sh2);
  auto vec = [&](float (&f)[8], const float (&g)[8]) {
    unsigned bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float o = fmaf(f[j], sc[j], sh[j]) + fmaf(g[j], sc2[j], sh2[j]);
      bits |= (o > 0.f ? 1u : 0u) << j;
      f[j] = o > 0.f ? o : 0.f;
    }
    return bits;
  };
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (; v + stride < nvec; v += 2 * stride) {
    float f0[8], f1[8], g0[8], g1[8];
    ld8f(x + v * 8, f0);
    ld8f(x + (v + stride) * 8, f1);
    ld8f(x2 + v * 8, g0);
    ld8f(x2 + (v + stride) * 8, g1);
    const unsigned b0 = vec(f0, g0), b1 = vec(f1, g1);
    st8f(y + v * 8, f0);
    st8f(y + (v + stride) * 8, f1);
    mask[v] = static_cast<uint8_t>(b0);
    mask[v + stride] = static_cast<uint8_t>(b1);
  }
  if (v < nvec) {
    float f0[8], g0[8];
    ld8f(x + v * 8, f0);
    ld8f(x2 + v * 8, g0);
    const unsigned b0 = vec(f0, g0);
    st8f(y + v * 8, f0);
    mask[v] = static_cast<uint8_t>(b0);
  }
}

// acc[0:C] += sum(dy_eff), acc[C:2C] += sum(dy_eff * xhat) and acc2 likewise with xhat2
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce_dual_kernel(
    const T* __restrict__ dy, const uint8_t* __restrict__ mask, const T* __restrict__ x, const T* __restrict__ x2,
    const float* __restrict__ mean, const float* __restrict__ inv, const float* __restrict__ mean2,
    const float* __restrict__ inv2, int64_t rows, int C, Geo g, float* __restrict__ acc, float* __restrict__ acc2) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = threadIdx.x;
  const int r0 = t / g.cv, c8 = t % g.cv;
  float s[8] = {0}, q[8] = {0}, q2[8] = {0};
  if (r0 < g.rpi) {
    float mu[8], is[8], mu2[8], is2[8];
    ld8ch(mean, c8 * 8, mu);
    ld8ch(inv, c8 * 8, is);
    ld8ch(mean2, c8 * 8, mu2);
    ld8ch(inv2, c8 * 8, is2);
    const int64_t start = static_cast<int64_t>(blockIdx.x) * g.rows_per_block;
    int64_t end = start + g.rows_per_block;
    if (end > rows) end = rows;
    int64_t r = start + r0;
    constexpr int U = 4;  // 4 rows x 3 tensors of 16 B loads in flight per lane
    for (; r + (U - 1) * g.rpi < end; r += U * g.rpi) {
      T d[U][8], xv[U][8], x2v[U][8];
      unsigned mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t off = (r + u * g.rpi) * C + c8 * 8;
        load8(dy + off, d[u]);
        load8(x + off, xv[u]);
        load8(x2 + off, x2v[u]);
        mb[u] = mask[off >> 3];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dd = (mb[u] >> j) & 1u ? static_cast<float>(d[u][j]) : 0.f;
          s[j] += dd;
          q[j] = fmaf(dd, (static_cast<float>(xv[u][j]) - mu[j]) * is[j], q[j]);
          q2[j] = fmaf(dd, (static_cast<float>(x2v[u][j]) - mu2[j]) * is2[j], q2[j]);
        }
    }
    for (; r < end; r += g.rpi) {
      const int64_t off = r * C + c8 * 8;
      float d[8], xv[8], x2v[8];
      ld8f(dy + off, d);
      ld8f(x + off, xv);
      ld8f(x2 + off, x2v);
      const unsigned mbs = mask[off >> 3];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dd = (mbs >> j) & 1u ? d[j] : 0.f;
        s[j] += dd;
        q[j] = fmaf(dd, (xv[j] - mu[j]) * is[j], q[j]);
        q2[j] = fmaf(dd, (x2v[j] - mu2[j]) * is2[j], q2[j]);
      }
    }
  }
  block_reduce_atomic(s, q, g.cv, g.rpi, C, acc, smem);
  __syncthreads();  // the LDS staging is reused
  block_reduce_atomic(s, q2, g.cv, g.rpi, C, acc2, smem);
}

// dx = A*dy_eff + B*x + D, dx2 = A2*dy_eff + B2*x2 + D2 (coefficients as in bn_bwd_dx_kernel)
__device__ __forceinline__ void dx_coef8(const float* __restrict__ w, const float* __restrict__ mean,
                                         const float* __restrict__ inv, const float* __restrict__ dw,
                                         const float* __restrict__ db, float inv_n, int c0, float (&a)[8],
                                         float (&bb)[8], float (&d)[8]) {
  float iv[8], m[8], ww[8], kdb[8], kdw[8];
  ld8ch(inv, c0, iv);
  ld8ch(mean, c0, m);
  ld8ch(db, c0, kdb);
  ld8ch(dw, c0, kdw);
  ld8ch(w ? w : mean, c0, ww);  // unconditional: see bn_norm_kernel
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float sc = (w ? ww[j] : 1.f) * iv[j];
    const float k2 = kdb[j] * inv_n, k3 = kdw[j] * inv_n;
    a[j] = sc;
    bb[j] = -sc * iv[j] * k3;
    d[j] = sc * (m[j] * iv[j] * k3 - k2);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void bn_bwd_dx_dual_kernel(
    const T* __restrict__ dy, const uint8_t* __restrict__ mask, const T* __restrict__ x, const T* __restrict__ x2,
    const float* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ inv,
    const float* __restrict__ dw, const float* __restrict__ db, const float* __restrict__ w2,
    const float* __restrict__ mean2, const float* __restrict__ inv2, const float* __restrict__ dw2,
    const float* __restrict__ db2, T* __restrict__ dx, T* __restrict__ dx2, int64_t rows, int C, int64_t nvec) {
  const float inv_n = 1.f / static_cast<float>(rows);
  const int c0 = (threadIdx.x % (C / 8)) * 8;
  float a[8], bq[8], dq[8], a2[8], bq2[8], dq2[8];
  dx_coef8(w, mean, inv, dw, db, inv_n, c0, a, bq, dq);
  dx_coef8(w2, mean2, inv2, dw2, db2, inv_n, c0, a2, bq2, dq2);
  auto vec = [&](float (&d)[8], float (&xv)[8], float (&x2v)[8], unsigned mbs) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dd = (mbs >> j) & 1u ? d[j] : 0.f;
      xv[j] = fmaf(a[j], dd, fmaf(bq[j], xv[j], dq[j]));
      x2v[j] = fmaf(a2[j], dd, fmaf(bq2[j], x2v[j], dq2[j]));
    }
  };
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (; v + stride < nvec; v += 2 * stride) {
    const int64_t v1 = v + stride;
    float d0[8], x0[8], z0[8], d1[8], x1[8], z1[8];
    ld8f(dy + v * 8, d0);
    ld8f(x + v * 8, x0);
    ld8f(x2 + v * 8, z0);
    ld8f(dy + v1 * 8, d1);
    ld8f(x + v1 * 8, x1);
    ld8f(x2 + v1 * 8, z1);
    const unsigned m0 = mask[v], m1 = mask[v1];
    vec(d0, x0, z0, m0);
    vec(d1, x1, z1, m1);
    st8f(dx + v * 8, x0);
    st8f(dx2 + v * 8, z0);
    st8f(dx + v1 * 8, x1);
    st8f(dx2 + v1 * 8, z1);
  }
  if (v < nvec) {
    float d0[8], x0[8], z0[8];
    ld8f(dy + v * 8, d0);
    ld8f(x + v * 8, x0);
    ld8f(x2 + v * 8, z0);
    vec(d0, x0, z0, mask[v]);
    st8f(dx + v * 8, x0);
    st8f(dx2 + v * 8, z0);
  }
}

// vectors per lane per iteration of the elementwise BN kernels: 2 (4 measured equal, round 4:
// profiles/rd4ak_bench_bn_unroll_ab.jsonl — the passes run at 4.4-5.8 TB/s either way)

// one full round of resident workgroups (or fewer if the tensor is small)
int elementwise_grid(const void* kernel, size_t smem, int64_t nvec) {
  // >= 4 vectors per lane: every workgroup pays its coefficient prologue once
  int64_t b = (nvec + 4 * kThreads - 1) / (4 * kThreads);
  const int64_t cap = resident_blocks(kernel, kThreads, smem);
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

bool fixed_channels(int64_t C) { return kThreads % (C / 8) == 0; }

void check(int64_t C) {
  if (C % 8 != 0 || C > kMaxC || C < 8)
    throw std::runtime_error("fused batchnorm: need C % 8 == 0 and 8 <= C <= 2048 (got " + std::to_string(C) + ")");
}

// the per-channel arrays are read 8 channels at a time with 16-B loads
void check_aligned(std::initializer_list<const void*> ptrs) {
  for (const void* p : ptrs)
    if (p != nullptr && (reinterpret_cast<uintptr_t>(p) & 15u) != 0)
      throw std::runtime_error("fused batchnorm: per-channel parameter / statistics arrays must be 16-B aligned");
}

size_t reduce_smem(const Geo& g, int64_t C) { return static_cast<size_t>(2 * g.rpi * C) * sizeof(float); }

// Geometry of a row-reduction kernel capped at one full round of its resident workgroups.
Geo reduce_geometry(const void* kernel, int64_t rows, int64_t C) {
  const Geo g0 = geometry(rows, C);
  return geometry(rows, C, resident_blocks(kernel, kThreads, reduce_smem(g0, C)));
}


template <typename T>
void norm_t(const void* x, void* y, const void* res, const float* w, const float* b, const float* mean,
            const float* stat2, int64_t rows, int64_t C, float eps, int train, int relu, uint8_t* mask,
            hipStream_t s) {
  const int64_t nvec = rows * C / 8;
  const T* xr = static_cast<const T*>(x);
  T* yr = static_cast<T*>(y);
  const T* rr = static_cast<const T*>(res);
  const bool fixed = fixed_channels(C);
#define LAUNCH(RELU, RES, FX)                                                                                   \
  {                                                                                                            \
    const size_t sm = FX ? 0 : 2 * C * sizeof(float);                                                          \
    auto k = bn_norm_kernel<T, RELU, RES, FX, 2>;   \
    k<<<elementwise_grid(reinterpret_cast<const void*>(k), sm, nvec), kThreads, sm, s>>>(                      \
        xr, yr, rr, w, b, mean, stat2, (int)C, eps, train, nvec, mask);                                        \
  }
#define LAUNCH_F(RELU, RES)                \
  {                                        \
    if (fixed) LAUNCH(RELU, RES, true)     \
    else LAUNCH(RELU, RES, false)          \
  }
  const bool has_res = res != nullptr;
  if (relu && has_res) LAUNCH_F(true, true)
  else if (relu) LAUNCH_F(true, false)
  else if (has_res) LAUNCH_F(false, true)
  else LAUNCH_F(false, false)
#undef LAUNCH_F
#undef LAUNCH
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

template <typename T>
void fwd_train_t(const void* x, void* y, const void* res, const float* w, const float* b, float* rm, float* rv,
                 float* sm, float* si, float* ws, int64_t rows, int64_t C, float momentum, float eps, int relu,
                 uint8_t* mask, int64_t* nbt, hipStream_t s) {
  const Geo g = reduce_geometry(reinterpret_cast<const void*>(bn_stats_kernel<T>), rows, C);
  bn_stats_kernel<T><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(static_cast<const T*>(x), rows, (int)C, g, ws);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  bn_finalize_fwd_kernel<<<finalize_blocks(C), kFinCh * kFinGroups, 0, s>>>(ws, (int)C, rows, momentum, eps, sm, si, rm,
                                                                            rv, nullptr, nullptr, nullptr, nullptr, nbt);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  norm_t<T>(x, y, res, w, b, sm, si, rows, C, eps, 1, relu, mask, s);
}

template <typename T>
void bwd_t(const void* dy, const void* x, const void* y, const uint8_t* mask, const float* w, const float* b,
           const float* sm, const float* si, void* dx, void* dres, float* dw, float* db, float* ws, int64_t rows,
           int64_t C, int relu, int stats_ready, hipStream_t s) {
  const T* dyr = static_cast<const T*>(dy);
  const T* xr = static_cast<const T*>(x);
  const T* yr = static_cast<const T*>(y);
  // relu: 0 none; 1 mask from y; 2 mask recomputed from x (no residual); 3 mask from saved bits
  const int rm = relu == 0 ? 0 : (mask != nullptr ? 3 : (y != nullptr ? 1 : 2));
#define RED(RM)                                                                                                  \
  {                                                                                                             \
    const Geo g = reduce_geometry(reinterpret_cast<const void*>(bn_bwd_reduce_kernel<T, RM>), rows, C);          \
    bn_bwd_reduce_kernel<T, RM><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(dyr, xr, yr, mask, w, b, sm, si,   \
                                                                              rows, (int)C, g, ws);             \
  }
  // stats_ready: the reductions were accumulated into ws by the producer of dy (the GEMM's
  // BN-backward epilogue), so the reduce pass over (dy, x) is skipped
  if (stats_ready) {}
  else if (rm == 0) RED(0)
  else if (rm == 1) RED(1)
  else if (rm == 2) RED(2)
  else RED(3)
#undef RED
  FLUXMPI_HIP_CHECK(hipGetLastError());
  bn_finalize_bwd_kernel<<<finalize_blocks(C), kFinCh * kFinGroups, 0, s>>>(ws, (int)C, dw, db);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  const int64_t nvec = rows * C / 8;
  T* dxr = static_cast<T*>(dx);
  T* drr = static_cast<T*>(dres);
  const bool fixed = fixed_channels(C);
#define LAUNCH(RM, DRES, FX)                                                                                    \
  {                                                                                                            \
    const size_t lds = FX ? 0 : C * sizeof(DxCoef);                                                            \
    auto k = bn_bwd_dx_kernel<T, RM, DRES, FX, 2>;   \
    k<<<elementwise_grid(reinterpret_cast<const void*>(k), lds, nvec), kThreads, lds, s>>>(                    \
        dyr, xr, yr, mask, w, b, sm, si, dw, db, dxr, drr, rows, (int)C, nvec);                                \
  }
#define LAUNCH_F(RM, DRES)             \
  {                                    \
    if (fixed) LAUNCH(RM, DRES, true)  \
    else LAUNCH(RM, DRES, false)       \
  }
  const bool has_dres = dres != nullptr;
  if (rm == 0) { if (has_dres) LAUNCH_F(0, true) else LAUNCH_F(0, false) }
  else if (rm == 1) { if (has_dres) LAUNCH_F(1, true) else LAUNCH_F(1, false) }
  else if (rm == 2) { if (has_dres) LAUNCH_F(2, true) else LAUNCH_F(2, false) }
  else { if (has_dres) LAUNCH_F(3, true) else LAUNCH_F(3, false) }
#undef LAUNCH_F
#undef LAUNCH
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

template <typename T>
void apply_dual_t(const void* x, const void* x2, void* y, const float* w, const float* b, const float* sm,
                  const float* si, const float* w2, const float* b2, const float* sm2, const float* si2, int64_t rows,
                  int64_t C, uint8_t* mask, hipStream_t s) {
  const int64_t nvec = rows * C / 8;
  auto k = bn_norm_dual_kernel<T>;
  k<<<elementwise_grid(reinterpret_cast<const void*>(k), 0, nvec), kThreads, 0, s>>>(
      static_cast<const T*>(x), static_cast<const T*>(x2), static_cast<T*>(y), w, b, sm, si, w2, b2, sm2, si2,
      (int)C, nvec, mask);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

template <typename T>
void bwd_dual_t(const void* dy, const uint8_t* mask, const void* x, const void* x2, const float* w, const float* sm,
                const float* si, const float* w2, const float* sm2, const float* si2, void* dx, void* dx2, float* dw,
                float* db, float* dw2, float* db2, float* ws, float* ws2, int64_t rows, int64_t C, hipStream_t s) {
  const T* dyr = static_cast<const T*>(dy);
  const T* xr = static_cast<const T*>(x);
  const T* x2r = static_cast<const T*>(x2);
  const Geo g = reduce_geometry(reinterpret_cast<const void*>(bn_bwd_reduce_dual_kernel<T>), rows, C);
  bn_bwd_reduce_dual_kernel<T><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(dyr, mask, xr, x2r, sm, si, sm2, si2,
                                                                             rows, (int)C, g, ws, ws2);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  bn_finalize_bwd2_kernel<<<dim3(finalize_blocks(C), 2), kFinCh * kFinGroups, 0, s>>>(ws, ws2, (int)C, dw, db, dw2,
                                                                                      db2);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  const int64_t nvec = rows * C / 8;
  auto k = bn_bwd_dx_dual_kernel<T>;
  k<<<elementwise_grid(reinterpret_cast<const void*>(k), 0, nvec), kThreads, 0, s>>>(
      dyr, mask, xr, x2r, w, sm, si, dw, db, w2, sm2, si2, dw2, db2, static_cast<T*>(dx), static_cast<T*>(dx2), rows,
      (int)C, nvec);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void check_dual(int64_t C, const uint8_t* mask) {
  check(C);
  if (!fixed_channels(C))
    throw std::runtime_error("dual batchnorm: C/8 must divide 256 (got C=" + std::to_string(C) + ")");
  if (mask == nullptr) throw std::runtime_error("dual batchnorm: the ReLU mask is required");
}

}  // namespace

void bn_apply_dual(const void* x, const void* x2, void* y, const float* w, const float* b, const float* sm,
                   const float* si, const float* w2, const float* b2, const float* sm2, const float* si2,
                   int64_t rows, int64_t C, uint8_t* mask, int dtype, hipStream_t s) {
  check_dual(C, mask);
  check_aligned({w, b, sm, si, w2, b2, sm2, si2});
  switch (dtype) {
    case kBF16: apply_dual_t<bf16>(x, x2, y, w, b, sm, si, w2, b2, sm2, si2, rows, C, mask, s); break;
    case kF16: apply_dual_t<f16>(x, x2, y, w, b, sm, si, w2, b2, sm2, si2, rows, C, mask, s); break;
    case kF32: apply_dual_t<float>(x, x2, y, w, b, sm, si, w2, b2, sm2, si2, rows, C, mask, s); break;
    default: throw std::runtime_error("dual batchnorm: unsupported dtype");
  }
}

void bn_bwd_dual(const void* dy, const uint8_t* mask, const void* x, const void* x2, const float* w, const float* sm,
                 const float* si, const float* w2, const float* sm2, const float* si2, void* dx, void* dx2, float* dw,
                 float* db, float* dw2, float* db2, float* ws, float* ws2, int64_t rows, int64_t C, int dtype,
                 hipStream_t s) {
  check_dual(C, mask);
  check_aligned({w, sm, si, w2, sm2, si2, dw, db, dw2, db2});
  switch (dtype) {
    case kBF16: bwd_dual_t<bf16>(dy, mask, x, x2, w, sm, si, w2, sm2, si2, dx, dx2, dw, db, dw2, db2, ws, ws2, rows, C, s); break;
    case kF16: bwd_dual_t<f16>(dy, mask, x, x2, w, sm, si, w2, sm2, si2, dx, dx2, dw, db, dw2, db2, ws, ws2, rows, C, s); break;
    case kF32: bwd_dual_t<float>(dy, mask, x, x2, w, sm, si, w2, sm2, si2, dx, dx2, dw, db, dw2, db2, ws, ws2, rows, C, s); break;
    default: throw std::runtime_error("dual batchnorm: unsupported dtype");
  }
}

size_t bn_workspace_floats(int64_t rows, int64_t C) {
  (void)rows;
  return static_cast<size_t>(kShards) * 2 * static_cast<size_t>(C);
}

void bn_fwd_train(const void* x, void* y, const void* residual, const float* weight, const float* bias,
                  float* running_mean, float* running_var, float* save_mean, float* save_invstd, float* workspace,
                  int64_t rows, int64_t C, float momentum, float eps, int relu, uint8_t* relu_mask, int dtype,
                  hipStream_t stream, int64_t* nbt) {
  check(C);
  check_aligned({weight, bias, save_mean, save_invstd});
  switch (dtype) {
    case kBF16: fwd_train_t<bf16>(x, y, residual, weight, bias, running_mean, running_var, save_mean, save_invstd,
                                  workspace, rows, C, momentum, eps, relu, relu_mask, nbt, stream); break;
    case kF16: fwd_train_t<f16>(x, y, residual, weight, bias, running_mean, running_var, save_mean, save_invstd,
                                workspace, rows, C, momentum, eps, relu, relu_mask, nbt, stream); break;
    case kF32: fwd_train_t<float>(x, y, residual, weight, bias, running_mean, running_var, save_mean, save_invstd,
                                  workspace, rows, C, momentum, eps, relu, relu_mask, nbt, stream); break;
    default: throw std::runtime_error("fused batchnorm: unsupported dtype");
  }
}

void bn_finalize_bwd(float* ws, int64_t C, float* dw, float* db, hipStream_t s) {
  check(C);
  bn_finalize_bwd_kernel<<<finalize_blocks(C), kFinCh * kFinGroups, 0, s>>>(ws, (int)C, dw, db);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void bn_stats_finalize(const void* x, const float* w, const float* b, float* rm, float* rv, float* sm, float* si,
                       float* scale, float* shift, float* ws, int64_t rows, int64_t C, float momentum, float eps,
                       int stats_ready, int dtype, hipStream_t s, int64_t* nbt) {
  check(C);
  if (!stats_ready) {
#define STATS(T)                                                                                              \
  {                                                                                                          \
    const Geo g = reduce_geometry(reinterpret_cast<const void*>(bn_stats_kernel<T>), rows, C);               \
    bn_stats_kernel<T><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(static_cast<const T*>(x), rows, (int)C, g, \
                                                                     ws);                                      \
  }
    switch (dtype) {
      case kBF16: STATS(bf16) break;
      case kF16: STATS(f16) break;
      case kF32: STATS(float) break;
      default: throw std::runtime_error("fused batchnorm: unsupported dtype");
    }
#undef STATS
    FLUXMPI_HIP_CHECK(hipGetLastError());
  }
  bn_finalize_fwd_kernel<<<finalize_blocks(C), kFinCh * kFinGroups, 0, s>>>(ws, (int)C, rows, momentum, eps, sm, si, rm,
                                                                            rv, w, b, scale, shift, nbt);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void bn_apply(const void* x, void* y, const void* res, const float* w, const float* b, const float* sm,
              const float* si, int64_t rows, int64_t C, int relu, uint8_t* mask, int dtype, hipStream_t s) {
  check(C);
  check_aligned({w, b, sm, si});
  switch (dtype) {
    case kBF16: norm_t<bf16>(x, y, res, w, b, sm, si, rows, C, 0.f, 1, relu, mask, s); break;
    case kF16: norm_t<f16>(x, y, res, w, b, sm, si, rows, C, 0.f, 1, relu, mask, s); break;
    case kF32: norm_t<float>(x, y, res, w, b, sm, si, rows, C, 0.f, 1, relu, mask, s); break;
    default: throw std::runtime_error("fused batchnorm: unsupported dtype");
  }
}

void bn_fwd_infer(const void* x, void* y, const void* residual, const float* weight, const float* bias,
                  const float* running_mean, const float* running_var, int64_t rows, int64_t C, float eps, int relu,
                  int dtype, hipStream_t stream) {
  check(C);
  check_aligned({weight, bias, running_mean, running_var});
  switch (dtype) {
    case kBF16: norm_t<bf16>(x, y, residual, weight, bias, running_mean, running_var, rows, C, eps, 0, relu, nullptr, stream); break;
    case kF16: norm_t<f16>(x, y, residual, weight, bias, running_mean, running_var, rows, C, eps, 0, relu, nullptr, stream); break;
    case kF32: norm_t<float>(x, y, residual, weight, bias, running_mean, running_var, rows, C, eps, 0, relu, nullptr, stream); break;
    default: throw std::runtime_error("fused batchnorm: unsupported dtype");
  }
}

void bn_bwd(const void* dy, const void* x, const void* y, const uint8_t* relu_mask, const float* weight,
            const float* bias, const float* save_mean,
            const float* save_invstd, void* dx, void* dres, float* dweight, float* dbias, float* workspace,
            int64_t rows, int64_t C, int relu, int dtype, hipStream_t stream, int stats_ready) {
  check(C);
  check_aligned({weight, bias, save_mean, save_invstd, dweight, dbias});
  switch (dtype) {
    case kBF16: bwd_t<bf16>(dy, x, y, relu_mask, weight, bias, save_mean, save_invstd, dx, dres, dweight, dbias, workspace, rows, C,
                            relu, stats_ready, stream); break;
    case kF16: bwd_t<f16>(dy, x, y, relu_mask, weight, bias, save_mean, save_invstd, dx, dres, dweight, dbias, workspace, rows, C,
                          relu, stats_ready, stream); break;
    case kF32: bwd_t<float>(dy, x, y, relu_mask, weight, bias, save_mean, save_invstd, dx, dres, dweight, dbias, workspace, rows, C,
                            relu, stats_ready, stream); break;
    default: throw std::runtime_error("fused batchnorm: unsupported dtype");
  }
}

}  // namespace fluxmpi
