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
// adds its partial to one of 16 shards of a [16][2][C] fp32 accumulator with
// global float atomics. A tiny finalize kernel sums the shards into the
// per-channel statistics (and re-zeroes them, so the persistent workspace
// needs no memset per call); the consumer kernels derive their per-channel
// coefficients from those statistics in an LDS prologue.
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

struct Geo {
  int cv;    // channel vectors per row (C / 8)
  int rpi;   // rows handled concurrently by a workgroup (kThreads / cv)
  int64_t rows_per_block;
  int blocks;
};

Geo geometry(int64_t rows, int64_t C) {
  Geo g;
  g.cv = static_cast<int>(C / 8);
  g.rpi = kThreads / g.cv;
  if (g.rpi < 1) g.rpi = 1;
  // >= 64K elements per workgroup, at most 2048 workgroups
  int64_t min_rows = (32768 + C - 1) / C;
  int64_t blocks = (rows + min_rows - 1) / min_rows;
  if (blocks > 2048) blocks = 2048;
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
  float* shard = acc + static_cast<size_t>(blockIdx.x % kShards) * 2 * C;
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

// Sum the shards of channel c and re-zero them (the workspace is left zeroed
// for the next call, so no memset is needed per launch).
__device__ __forceinline__ void take_shards(float* __restrict__ acc, int C, int c, float& a, float& b) {
  a = 0.f;
  b = 0.f;
#pragma unroll
  for (int k = 0; k < kShards; ++k) {
    float* sh = acc + static_cast<size_t>(k) * 2 * C;
    a += sh[c];
    b += sh[C + c];
    sh[c] = 0.f;
    sh[C + c] = 0.f;
  }
}

__global__ void bn_finalize_fwd_kernel(float* __restrict__ acc, int C, int64_t rows, float momentum, float eps,
                                       float* __restrict__ smean, float* __restrict__ sinv,
                                       float* __restrict__ rmean, float* __restrict__ rvar,
                                       const float* __restrict__ w, const float* __restrict__ b,
                                       float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s, q;
  take_shards(acc, C, c, s, q);
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

__global__ void bn_finalize_bwd_kernel(float* __restrict__ acc, int C, float* __restrict__ dw,
                                       float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s, q;
  take_shards(acc, C, c, s, q);
  db[c] = s;  // sum(dy_eff)
  dw[c] = q;  // sum(dy_eff * xhat)
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

// y = act(x*scale + shift [+ res]); scale/shift derived in the LDS prologue from
// (mean, invstd) = batch statistics (training) or running statistics (eval).
template <typename T, bool RELU, bool RES>
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
  float* scale = smem;
  float* shift = smem + C;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float mean = mean_in[c];
    const float invstd = train ? stat2[c] : rsqrtf(stat2[c] + eps);  // save_invstd | running_var
    const float sc = (w ? w[c] : 1.f) * invstd;
    scale[c] = sc;
    shift[c] = fmaf(-mean, sc, b ? b[c] : 0.f);  // explicit fma: backward recomputes it bit-identically
  }
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; v < nvec; v += stride) {
    const int64_t e = v * 8;
    const int c0 = static_cast<int>(e % C);
    float f[8];
    ld8f(x + e, f);
    float rr[8];
    if (RES) ld8f(res + e, rr);
    unsigned bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = fmaf(f[j], scale[c0 + j], shift[c0 + j]);
      if (RES) o += rr[j];
      if (RELU) {
        bits |= (o > 0.f ? 1u : 0u) << j;
        o = o > 0.f ? o : 0.f;
      }
      f[j] = o;
    }
    st8f(y + e, f);
    if (RELU && mask != nullptr) mask[v] = static_cast<uint8_t>(bits);
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
    float mu[8], is[8], sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c8 * 8 + j;
      mu[j] = smean[c];
      is[j] = sinv[c];
      sc[j] = (w ? w[c] : 1.f) * is[j];
      sh[j] = fmaf(-mu[j], sc[j], b ? b[c] : 0.f);
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
// (sum_dy = db, sum_dy_xhat = dw, produced by bn_finalize_bwd_kernel)
template <typename T, int RM, bool DRES>
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
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* k1 = smem;          // w*invstd (== forward scale)
  float* k2 = smem + C;      // mean(dy_eff)
  float* k3 = smem + 2 * C;  // mean(dy_eff*xhat)
  float* mu = smem + 3 * C;
  float* is = smem + 4 * C;
  float* sh = smem + 5 * C;  // forward shift (RM == 2)
  const float inv_n = 1.f / static_cast<float>(rows);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float iv = sinv[c];
    const float m = smean[c];
    const float sc = (w ? w[c] : 1.f) * iv;
    k1[c] = sc;
    k2[c] = db[c] * inv_n;
    k3[c] = dw[c] * inv_n;
    mu[c] = m;
    is[c] = iv;
    sh[c] = fmaf(-m, sc, bias ? bias[c] : 0.f);
  }
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; v < nvec; v += stride) {
    const int64_t e = v * 8;
    const int c0 = static_cast<int>(e % C);
    float d[8], xv[8], yv[8];
    ld8f(dy + e, d);
    ld8f(x + e, xv);
    if (RM == 1) ld8f(y + e, yv);
    const unsigned mbs = RM == 3 ? mask[v] : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float dd = d[j];
      if (RM == 1) dd = yv[j] > 0.f ? dd : 0.f;
      if (RM == 3) dd = (mbs >> j) & 1u ? dd : 0.f;
      if (RM == 2) dd = fmaf(xv[j], k1[c], sh[c]) > 0.f ? dd : 0.f;
      d[j] = dd;
      const float xh = (xv[j] - mu[c]) * is[c];
      xv[j] = k1[c] * (dd - k2[c] - xh * k3[c]);
    }
    st8f(dx + e, xv);
    if (DRES) st8f(dres + e, d);
  }
}

int elementwise_blocks(int64_t nvec) {
  int64_t b = (nvec + kThreads - 1) / kThreads;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

void check(int64_t C) {
  if (C % 8 != 0 || C > kMaxC || C < 8)
    throw std::runtime_error("fused batchnorm: need C % 8 == 0 and 8 <= C <= 2048 (got " + std::to_string(C) + ")");
}

size_t reduce_smem(const Geo& g, int64_t C) { return static_cast<size_t>(2 * g.rpi * C) * sizeof(float); }

#define FLUXMPI_BN_DISPATCH2(F, A, B, ...) \
  if ((A) && (B)) F(true, true, __VA_ARGS__);  \
  else if (A) F(true, false, __VA_ARGS__);    \
  else if (B) F(false, true, __VA_ARGS__);    \
  else F(false, false, __VA_ARGS__);

template <typename T>
void norm_t(const void* x, void* y, const void* res, const float* w, const float* b, const float* mean,
            const float* stat2, int64_t rows, int64_t C, float eps, int train, int relu, uint8_t* mask,
            hipStream_t s) {
  const int64_t nvec = rows * C / 8;
  const int nb = elementwise_blocks(nvec);
  const size_t sm2 = 2 * C * sizeof(float);
  const T* xr = static_cast<const T*>(x);
  T* yr = static_cast<T*>(y);
  const T* rr = static_cast<const T*>(res);
#define LAUNCH(RELU, RES, _)                                                                                     \
  bn_norm_kernel<T, RELU, RES><<<nb, kThreads, sm2, s>>>(xr, yr, rr, w, b, mean, stat2, (int)C, eps, train, nvec, \
                                                         mask)
  FLUXMPI_BN_DISPATCH2(LAUNCH, relu, res != nullptr, 0)
#undef LAUNCH
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

template <typename T>
void fwd_train_t(const void* x, void* y, const void* res, const float* w, const float* b, float* rm, float* rv,
                 float* sm, float* si, float* ws, int64_t rows, int64_t C, float momentum, float eps, int relu,
                 uint8_t* mask, hipStream_t s) {
  Geo g = geometry(rows, C);
  bn_stats_kernel<T><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(static_cast<const T*>(x), rows, (int)C, g, ws);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  bn_finalize_fwd_kernel<<<(int)((C + 255) / 256), 256, 0, s>>>(ws, (int)C, rows, momentum, eps, sm, si, rm, rv,
                                                                 nullptr, nullptr, nullptr, nullptr);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  norm_t<T>(x, y, res, w, b, sm, si, rows, C, eps, 1, relu, mask, s);
}

template <typename T>
void bwd_t(const void* dy, const void* x, const void* y, const uint8_t* mask, const float* w, const float* b,
           const float* sm, const float* si, void* dx, void* dres, float* dw, float* db, float* ws, int64_t rows,
           int64_t C, int relu, hipStream_t s) {
  Geo g = geometry(rows, C);
  const T* dyr = static_cast<const T*>(dy);
  const T* xr = static_cast<const T*>(x);
  const T* yr = static_cast<const T*>(y);
  // relu: 0 none; 1 mask from y; 2 mask recomputed from x (no residual); 3 mask from saved bits
  const int rm = relu == 0 ? 0 : (mask != nullptr ? 3 : (y != nullptr ? 1 : 2));
  const size_t rsm = reduce_smem(g, C);
#define RED(RM) \
  bn_bwd_reduce_kernel<T, RM><<<g.blocks, kThreads, rsm, s>>>(dyr, xr, yr, mask, w, b, sm, si, rows, (int)C, g, ws)
  if (rm == 0) RED(0);
  else if (rm == 1) RED(1);
  else if (rm == 2) RED(2);
  else RED(3);
#undef RED
  FLUXMPI_HIP_CHECK(hipGetLastError());
  bn_finalize_bwd_kernel<<<(int)((C + 255) / 256), 256, 0, s>>>(ws, (int)C, dw, db);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  const int64_t nvec = rows * C / 8;
  const int nb = elementwise_blocks(nvec);
  const size_t sm6 = 6 * C * sizeof(float);
  T* dxr = static_cast<T*>(dx);
  T* drr = static_cast<T*>(dres);
#define LAUNCH(RM, DRES)                                                                                          \
  bn_bwd_dx_kernel<T, RM, DRES><<<nb, kThreads, sm6, s>>>(dyr, xr, yr, mask, w, b, sm, si, dw, db, dxr, drr, rows, \
                                                          (int)C, nvec)
  const bool has_dres = dres != nullptr;
  if (rm == 0) { if (has_dres) LAUNCH(0, true); else LAUNCH(0, false); }
  else if (rm == 1) { if (has_dres) LAUNCH(1, true); else LAUNCH(1, false); }
  else if (rm == 2) { if (has_dres) LAUNCH(2, true); else LAUNCH(2, false); }
  else { if (has_dres) LAUNCH(3, true); else LAUNCH(3, false); }
#undef LAUNCH
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

size_t bn_workspace_floats(int64_t rows, int64_t C) {
  (void)rows;
  return static_cast<size_t>(kShards) * 2 * static_cast<size_t>(C);
}

void bn_fwd_train(const void* x, void* y, const void* residual, const float* weight, const float* bias,
                  float* running_mean, float* running_var, float* save_mean, float* save_invstd, float* workspace,
                  int64_t rows, int64_t C, float momentum, float eps, int relu, uint8_t* relu_mask, int dtype,
                  hipStream_t stream) {
  check(C);
  switch (dtype) {
    case kBF16: fwd_train_t<bf16>(x, y, residual, weight, bias, running_mean, running_var, save_mean, save_invstd,
                                  workspace, rows, C, momentum, eps, relu, relu_mask, stream); break;
    case kF16: fwd_train_t<f16>(x, y, residual, weight, bias, running_mean, running_var, save_mean, save_invstd,
                                workspace, rows, C, momentum, eps, relu, relu_mask, stream); break;
    case kF32: fwd_train_t<float>(x, y, residual, weight, bias, running_mean, running_var, save_mean, save_invstd,
                                  workspace, rows, C, momentum, eps, relu, relu_mask, stream); break;
    default: throw std::runtime_error("fused batchnorm: unsupported dtype");
  }
}

void bn_stats_finalize(const void* x, const float* w, const float* b, float* rm, float* rv, float* sm, float* si,
                       float* scale, float* shift, float* ws, int64_t rows, int64_t C, float momentum, float eps,
                       int stats_ready, int dtype, hipStream_t s) {
  check(C);
  if (!stats_ready) {
    Geo g = geometry(rows, C);
    switch (dtype) {
      case kBF16: bn_stats_kernel<bf16><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(static_cast<const bf16*>(x), rows, (int)C, g, ws); break;
      case kF16: bn_stats_kernel<f16><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(static_cast<const f16*>(x), rows, (int)C, g, ws); break;
      case kF32: bn_stats_kernel<float><<<g.blocks, kThreads, reduce_smem(g, C), s>>>(static_cast<const float*>(x), rows, (int)C, g, ws); break;
      default: throw std::runtime_error("fused batchnorm: unsupported dtype");
    }
    FLUXMPI_HIP_CHECK(hipGetLastError());
  }
  bn_finalize_fwd_kernel<<<(int)((C + 255) / 256), 256, 0, s>>>(ws, (int)C, rows, momentum, eps, sm, si, rm, rv, w, b,
                                                                 scale, shift);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void bn_apply(const void* x, void* y, const void* res, const float* w, const float* b, const float* sm,
              const float* si, int64_t rows, int64_t C, int relu, uint8_t* mask, int dtype, hipStream_t s) {
  check(C);
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
            int64_t rows, int64_t C, int relu, int dtype, hipStream_t stream) {
  check(C);
  switch (dtype) {
    case kBF16: bwd_t<bf16>(dy, x, y, relu_mask, weight, bias, save_mean, save_invstd, dx, dres, dweight, dbias, workspace, rows, C,
                            relu, stream); break;
    case kF16: bwd_t<f16>(dy, x, y, relu_mask, weight, bias, save_mean, save_invstd, dx, dres, dweight, dbias, workspace, rows, C,
                          relu, stream); break;
    case kF32: bwd_t<float>(dy, x, y, relu_mask, weight, bias, save_mean, save_invstd, dx, dres, dweight, dbias, workspace, rows, C,
                            relu, stream); break;
    default: throw std::runtime_error("fused batchnorm: unsupported dtype");
  }
}

}  // namespace fluxmpi
