// Fused NHWC GroupNorm (+ residual add, + ReLU on its input) forward / backward — gfx950.
//
// For the DEQ cell  f(z, x) = GN3(relu(z + GN2(x + conv2(GN1(relu(conv1 z))))))  on
// channels_last activations. PyTorch's GroupNorm wants NCHW, so on NHWC tensors every call
// pays two layout copies plus separate moment / apply / add / relu kernels; here one
// workgroup owns one sample (HW x C contiguous in NHWC):
//   forward   h = [relu](x [+ a]);  y = (h - mean_g) * rstd_g * w_c + b_c
//             pass 1 per-channel sum / sumsq in registers (each lane keeps ONE fixed 8-channel
//             vector: blockDim = PL * (C/8) lanes, PL pixel lanes (up to 256 lanes, the reduction
//             scratch within 64 KB of LDS), so a lane's channels never change),
//             LDS reduce -> group stats; pass 2 (L2-hot re-read) applies and writes y [and h].
//   backward  per-channel sums of dy and dy*h in one pass give db_c, dw_c and the two group
//             terms; pass 2 writes dh = rstd (dy w - s1/M - xhat s2/M) [* (h > 0)], which is the
//             gradient of both x and a. dw/db: one [2][C] fp32 partial per sample (no atomics).
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

// lanes per workgroup, one workgroup per sample. 1024 lanes (GN_THREADS=1024, A/B builds only)
// measured 4-8 % slower than 256 at the DEQ shapes (profiles/rd5l_bench_gn.jsonl)
#ifndef GN_THREADS
#define GN_THREADS 256
#endif
constexpr int kMaxThreads = GN_THREADS;
constexpr int kLdsBudget = 64 * 1024;  // dynamic LDS without a per-kernel attribute
constexpr int kMaxG = 64;
// pixels per lane whose loads are issued together (one workgroup per sample: at one pixel per
// iteration every pass was a chain of dependent memory round trips, ~2.6 TB/s on the DEQ cell)
// (GN_KU = 8 / 16, A/B builds only: equal or slower at the DEQ shapes, profiles/rd5y_bench_gn_ku.jsonl —
// the forward is at ~4.4 TB/s of algorithmic traffic already)
#ifndef GN_KU
#define GN_KU 4
#endif
constexpr int kU = GN_KU;

struct GnShape {
  int HW, C, G, CV, PL, T;  // CV = C/8 channel vectors per pixel, PL pixel lanes, T = PL*CV lanes
};

GnShape gn_shape(int64_t HW, int64_t C, int64_t G) {
  if (C % 8 != 0 || C / 8 > kMaxThreads || G < 1 || G > kMaxG || C % G != 0)
    throw std::runtime_error("fused groupnorm: need C % 8 == 0, C <= 2048, G <= 64, C % G == 0");
  GnShape s;
  s.HW = static_cast<int>(HW);
  s.C = static_cast<int>(C);
  s.G = static_cast<int>(G);
  s.CV = s.C / 8;
  // pixel lanes: as many as fit the workgroup and the reduction's LDS (red[2][PL][C] floats plus
  // chan[2][C] and grp[2][G])
  const int by_lds = (kLdsBudget / 4 - 2 * s.C - 2 * s.G) / (2 * s.C);
  s.PL = kMaxThreads / s.CV < by_lds ? kMaxThreads / s.CV : by_lds;
  if (s.PL < 1) s.PL = 1;
  s.T = s.PL * s.CV;
  return s;
}

// LDS: red[2][PL][C] floats, then chan[2][C] + grp[2][G]
// (every (pixel lane, channel vector) slot is written by exactly one active lane)
__device__ __forceinline__ void reduce_channels(float* red, const float (&a)[8], const float (&q)[8], int pl, int cv,
                                                int PL, int C, float* chan, bool active) {
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[pl * C + cv * 8 + j] = a[j];
      red[PL * C + pl * C + cv * 8 + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) {
    const int which = c / C, ch = c % C;
    const float* r = red + which * PL * C + ch;
    float s = 0.f;
    for (int p = 0; p < PL; ++p) s += r[p * C];
    chan[c] = s;
  }
  __syncthreads();
}

template <typename T, bool ADD, bool RELU, bool SAVEH>
__global__ __launch_bounds__(kMaxThreads) void gn_fwd_kernel(const T* __restrict__ x, const T* __restrict__ a,
                                                             T* __restrict__ h, T* __restrict__ y,
                                                             const float* __restrict__ w, const float* __restrict__ b,
                                                             float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                             GnShape s, float eps, int64_t y_stride) {
  extern __shared__ float lds[];
  float* red = lds;
  float* chan = red + 2 * s.PL * s.C;
  float* grp = chan + 2 * s.C;
  const int n = blockIdx.x;
  const int cv = threadIdx.x % s.CV, pl = threadIdx.x / s.CV;
  const int64_t base = static_cast<int64_t>(n) * s.HW * s.C + cv * 8;
  y += static_cast<int64_t>(n) * (y_stride - static_cast<int64_t>(s.HW) * s.C);  // y's sample n at n * y_stride
  const bool active = threadIdx.x < s.T;
  float sum[8], sq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sum[j] = sq[j] = 0.f;
  if (active) {
    auto acc = [&](const T (&xv)[8], const T (&av)[8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = to_f(xv[j]);
        if (ADD) v += to_f(av[j]);
        if (RELU) v = fmaxf(v, 0.f);
        v = to_f(from_f<T>(v));  // statistics of the rounded h the backward will see
        sum[j] += v;
        sq[j] += v * v;
      }
    };
    int p = pl;
    for (; p + (kU - 1) * s.PL < s.HW; p += kU * s.PL) {  // kU pixels' loads in flight
      T xv[kU][8], av[kU][8];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        load8(x + base + static_cast<int64_t>(p + u * s.PL) * s.C, xv[u]);
        if (ADD) load8(a + base + static_cast<int64_t>(p + u * s.PL) * s.C, av[u]);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) acc(xv[u], av[u]);
    }
    for (; p < s.HW; p += s.PL) {
      T xv[8], av[8];
      load8(x + base + static_cast<int64_t>(p) * s.C, xv);
      if (ADD) load8(a + base + static_cast<int64_t>(p) * s.C, av);
      acc(xv, av);
    }
  }
  reduce_channels(red, sum, sq, pl, cv, s.PL, s.C, chan, active);
  const int cpg = s.C / s.G;
  const float inv_m = 1.f / (static_cast<float>(s.HW) * cpg);
  if (threadIdx.x < s.G) {
    float gs = 0.f, gq = 0.f;
    for (int c = threadIdx.x * cpg; c < (threadIdx.x + 1) * cpg; ++c) {
      gs += chan[c];
      gq += chan[s.C + c];
    }
    const float mu = gs * inv_m;
    const float var = fmaxf(gq * inv_m - mu * mu, 0.f);
    const float r = rsqrtf(var + eps);
    grp[threadIdx.x] = mu;
    grp[s.G + threadIdx.x] = r;
    mean_out[static_cast<int64_t>(n) * s.G + threadIdx.x] = mu;
    rstd_out[static_cast<int64_t>(n) * s.G + threadIdx.x] = r;
  }
  __syncthreads();
  if (!active) return;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cv * 8 + j, g = c / cpg;
    const float wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
    sc[j] = grp[s.G + g] * wc;
    sh[j] = bc - grp[g] * sc[j];
  }
  auto apply = [&](int64_t off, const T (&xv)[8], const T (&av)[8]) {
    T hv[8], yv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = to_f(xv[j]);
      if (ADD) v += to_f(av[j]);
      if (RELU) v = fmaxf(v, 0.f);
      hv[j] = from_f<T>(v);
      yv[j] = from_f<T>(to_f(hv[j]) * sc[j] + sh[j]);
    }
    if (SAVEH) store8(h + off, hv);
    store8(y + off, yv);
  };
  int p = pl;
  for (; p + (kU - 1) * s.PL < s.HW; p += kU * s.PL) {
    T xv[kU][8], av[kU][8];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t off = base + static_cast<int64_t>(p + u * s.PL) * s.C;
      load8(x + off, xv[u]);
      if (ADD) load8(a + off, av[u]);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) apply(base + static_cast<int64_t>(p + u * s.PL) * s.C, xv[u], av[u]);
  }
  for (; p < s.HW; p += s.PL) {
    const int64_t off = base + static_cast<int64_t>(p) * s.C;
    T xv[8], av[8];
    load8(x + off, xv);
    if (ADD) load8(a + off, av);
    apply(off, xv, av);
  }
}

template <typename T, bool RELU>
__global__ __launch_bounds__(kMaxThreads) void gn_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ h,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ w, T* __restrict__ dh,
                                                             float* __restrict__ part, GnShape s) {
  extern __shared__ float lds[];
  float* red = lds;
  float* chan = red + 2 * s.PL * s.C;
  float* grp = chan + 2 * s.C;
  const int n = blockIdx.x;
  const int cv = threadIdx.x % s.CV, pl = threadIdx.x / s.CV;
  const int64_t base = static_cast<int64_t>(n) * s.HW * s.C + cv * 8;
  const bool active = threadIdx.x < s.T;
  float sdy[8], sdyh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sdy[j] = sdyh[j] = 0.f;
  if (active) {
    auto acc = [&](const T (&dv)[8], const T (&hv)[8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = to_f(dv[j]);
        sdy[j] += d;
        sdyh[j] += d * to_f(hv[j]);
      }
    };
    int p = pl;
    for (; p + (kU - 1) * s.PL < s.HW; p += kU * s.PL) {  // kU pixels' loads in flight
      T dv[kU][8], hv[kU][8];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        load8(dy + base + static_cast<int64_t>(p + u * s.PL) * s.C, dv[u]);
        load8(h + base + static_cast<int64_t>(p + u * s.PL) * s.C, hv[u]);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) acc(dv[u], hv[u]);
    }
    for (; p < s.HW; p += s.PL) {
      T dv[8], hv[8];
      load8(dy + base + static_cast<int64_t>(p) * s.C, dv);
      load8(h + base + static_cast<int64_t>(p) * s.C, hv);
      acc(dv, hv);
    }
  }
  reduce_channels(red, sdy, sdyh, pl, cv, s.PL, s.C, chan, active);
  const int cpg = s.C / s.G;
  const float inv_m = 1.f / (static_cast<float>(s.HW) * cpg);
  // per channel: db = sum dy, dw = sum dy * xhat = rstd (sum dy h - mean sum dy)
  for (int c = threadIdx.x; c < s.C; c += blockDim.x) {
    const int g = c / cpg;
    const float mu = mean[static_cast<int64_t>(n) * s.G + g], r = rstd[static_cast<int64_t>(n) * s.G + g];
    const float db = chan[c], dw = r * (chan[s.C + c] - mu * db);
    part[static_cast<int64_t>(n) * 2 * s.C + c] = dw;
    part[static_cast<int64_t>(n) * 2 * s.C + s.C + c] = db;
  }
  if (threadIdx.x < s.G) {  // s1 = sum dy w, s2 = sum dy w xhat over the group
    const int g = threadIdx.x;
    const float mu = mean[static_cast<int64_t>(n) * s.G + g], r = rstd[static_cast<int64_t>(n) * s.G + g];
    float s1 = 0.f, s2 = 0.f;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      const float wc = w ? w[c] : 1.f;
      s1 += wc * chan[c];
      s2 += wc * r * (chan[s.C + c] - mu * chan[c]);
    }
    grp[g] = s1 * inv_m;
    grp[s.G + g] = s2 * inv_m;
  }
  __syncthreads();
  if (!active) return;
  float wv[8], mu[8], rs[8], m1[8], m2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cv * 8 + j, g = c / cpg;
    wv[j] = w ? w[c] : 1.f;
    mu[j] = mean[static_cast<int64_t>(n) * s.G + g];
    rs[j] = rstd[static_cast<int64_t>(n) * s.G + g];
    m1[j] = grp[g];
    m2[j] = grp[s.G + g];
  }
  auto apply = [&](int64_t off, const T (&dv)[8], const T (&hv)[8]) {
    T ov[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float hf = to_f(hv[j]);
      const float xhat = (hf - mu[j]) * rs[j];
      float g = rs[j] * (to_f(dv[j]) * wv[j] - m1[j] - xhat * m2[j]);
      if (RELU && !(hf > 0.f)) g = 0.f;
      ov[j] = from_f<T>(g);
    }
    store8(dh + off, ov);
  };
  int p = pl;
  for (; p + (kU - 1) * s.PL < s.HW; p += kU * s.PL) {
    T dv[kU][8], hv[kU][8];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t off = base + static_cast<int64_t>(p + u * s.PL) * s.C;
      load8(dy + off, dv[u]);
      load8(h + off, hv[u]);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) apply(base + static_cast<int64_t>(p + u * s.PL) * s.C, dv[u], hv[u]);
  }
  for (; p < s.HW; p += s.PL) {
    const int64_t off = base + static_cast<int64_t>(p) * s.C;
    T dv[8], hv[8];
    load8(dy + off, dv);
    load8(h + off, hv);
    apply(off, dv, hv);
  }
}

unsigned block_of(const GnShape& s) { return static_cast<unsigned>((s.T + 63) / 64 * 64); }

size_t gn_lds(const GnShape& s) { return sizeof(float) * (2 * s.PL * s.C + 2 * s.C + 2 * s.G); }

template <typename T>
void fwd_dispatch(const void* x, const void* a, void* h, void* y, const float* w, const float* b, float* mean,
                  float* rstd, int64_t N, const GnShape& s, bool relu, float eps, hipStream_t st, int64_t ys) {
  const T* xp = static_cast<const T*>(x);
  const T* ap = static_cast<const T*>(a);
  T* hp = static_cast<T*>(h);
  T* yp = static_cast<T*>(y);
  const size_t lds = gn_lds(s);
  const dim3 grid(static_cast<unsigned>(N));
  const bool add = a != nullptr, saveh = h != nullptr;
#define GN_FWD(A, R, H) \
  gn_fwd_kernel<T, A, R, H><<<grid, block_of(s), lds, st>>>(xp, ap, hp, yp, w, b, mean, rstd, s, eps, ys)
  if (add && relu) { if (saveh) GN_FWD(true, true, true); else GN_FWD(true, true, false); }
  else if (add) { if (saveh) GN_FWD(true, false, true); else GN_FWD(true, false, false); }
  else if (relu) { if (saveh) GN_FWD(false, true, true); else GN_FWD(false, true, false); }
  else GN_FWD(false, false, false);
#undef GN_FWD
}

template <typename T>
void bwd_dispatch(const void* dy, const void* h, const float* mean, const float* rstd, const float* w, void* dh,
                  float* part, int64_t N, const GnShape& s, bool relu, hipStream_t st) {
  const size_t lds = gn_lds(s);
  const dim3 grid(static_cast<unsigned>(N));
  if (relu)
    gn_bwd_kernel<T, true><<<grid, block_of(s), lds, st>>>(static_cast<const T*>(dy), static_cast<const T*>(h), mean,
                                                          rstd, w, static_cast<T*>(dh), part, s);
  else
    gn_bwd_kernel<T, false><<<grid, block_of(s), lds, st>>>(static_cast<const T*>(dy), static_cast<const T*>(h), mean,
                                                           rstd, w, static_cast<T*>(dh), part, s);
}

void check_ptrs(std::initializer_list<const void*> ps) {
  for (const void* p : ps)
    if (p != nullptr && (reinterpret_cast<uintptr_t>(p) & 15u) != 0)
      throw std::runtime_error("fused groupnorm: tensors must be 16-byte aligned");
}

}  // namespace

void groupnorm_nhwc_fwd(const void* x, const void* add, void* h, void* y, const float* w, const float* b, float* mean,
                        float* rstd, int64_t N, int64_t HW, int64_t C, int64_t G, bool relu, float eps, int dtype,
                        hipStream_t stream, int64_t y_stride) {
  const GnShape s = gn_shape(HW, C, G);
  check_ptrs({x, add, h, y});
  if (N < 1 || N > 2147483647LL) throw std::runtime_error("fused groupnorm: bad N");
  if (y_stride == 0) y_stride = HW * C;
  if (y_stride < HW * C || y_stride % 8 != 0) throw std::runtime_error("fused groupnorm: bad output sample stride");
  switch (dtype) {
    case kBF16: fwd_dispatch<bf16>(x, add, h, y, w, b, mean, rstd, N, s, relu, eps, stream, y_stride); break;
    case kF16: fwd_dispatch<f16>(x, add, h, y, w, b, mean, rstd, N, s, relu, eps, stream, y_stride); break;
    case kF32: fwd_dispatch<float>(x, add, h, y, w, b, mean, rstd, N, s, relu, eps, stream, y_stride); break;
    default: throw std::runtime_error("fused groupnorm: unsupported dtype");
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void groupnorm_nhwc_bwd(const void* dy, const void* h, const float* mean, const float* rstd, const float* w, void* dh,
                        float* partials, int64_t N, int64_t HW, int64_t C, int64_t G, bool relu, int dtype,
                        hipStream_t stream) {
  const GnShape s = gn_shape(HW, C, G);
  check_ptrs({dy, h, dh});
  if (N < 1 || N > 2147483647LL) throw std::runtime_error("fused groupnorm: bad N");
  switch (dtype) {
    case kBF16: bwd_dispatch<bf16>(dy, h, mean, rstd, w, dh, partials, N, s, relu, stream); break;
    case kF16: bwd_dispatch<f16>(dy, h, mean, rstd, w, dh, partials, N, s, relu, stream); break;
    case kF32: bwd_dispatch<float>(dy, h, mean, rstd, w, dh, partials, N, s, relu, stream); break;
    default: throw std::runtime_error("fused groupnorm: unsupported dtype");
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
