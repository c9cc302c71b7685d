// Anderson-acceleration solver kernels for the Deep Equilibrium Model — gfx950.
//
// The solver keeps a history of m iterates X[b, i, :] (fp32) and their images F[b, i, :] (fp32,
// or bf16 when the model computes in bf16 — the cell's outputs are bf16 values either way),
// row length d = C*H*W, e.g. 48*28*28 = 37632) and, every iteration, needs
//   gram[b]  = G G^T  with G = F[b, :n] - X[b, :n]         (n <= m <= 8 rows)
//   X[b, s]  = beta * alpha[b] F[b, :n] + (1 - beta) * alpha[b] X[b, :n]
// PyTorch composes these as a strided subtract (materialising G), a batched fp32 GEMM whose
// output is n x n (hipBLASLt picks a 256x16 macro tile: ~570 us per call on MI355X for
// bsz 256, ~0.34 TB/s) and two more batched GEMMs for the mix. Both are HBM-bound
// streaming reductions, so here:
//   anderson_gram: one pass over F and X rows (G formed in registers, never stored); each
//       workgroup owns one (batch, d-chunk), keeps the n(n+1)/2 pair sums plus |F[s]|^2 of
//       the newest row in registers, reduces them across its 4 waves through LDS and stores
//       one partial row (no atomics; the host sums the chunk partials).
//   anderson_mix:  one pass that writes the new iterate and, optionally, its cast copy in
//       the model dtype (the next f(z) input) — no separate cast kernel.
// 16-byte (float4) accesses throughout; grids are bsz x chunks >= 2048 workgroups.
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxRows = 8;
constexpr int kPairs = kMaxRows * (kMaxRows + 1) / 2;  // 36 upper-triangle pairs
constexpr int kOut = kPairs + 1;                        // + |F[last]|^2

__device__ __forceinline__ float wave_sum(float v) { return wave_sum_dpp(v); }  // common.h

__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

// 4 consecutive elements of an F history row at element offset e, widened to fp32. F is bf16 when
// the model computes in bf16: its values are the cell's bf16 outputs either way, so the narrower
// history is exact and halves the bytes of the mix's N-row read.
template <typename FT>
__device__ __forceinline__ float4 ldf4(const FT* __restrict__ p, int64_t e) {
  if constexpr (sizeof(FT) == 4) {
    return *reinterpret_cast<const float4*>(p + e);
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p + e);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
  }
}

// 4 elements to a history row (fp32, or bf16 rounded to nearest even)
template <typename HT>
__device__ __forceinline__ void st4(HT* __restrict__ p, int64_t e, const float4& v) {
  if constexpr (sizeof(HT) == 4) {
    *reinterpret_cast<float4*>(p + e) = v;
  } else {
    const bf16 h[4] = {static_cast<bf16>(v.x), static_cast<bf16>(v.y), static_cast<bf16>(v.z), static_cast<bf16>(v.w)};
    uint2 u;
    __builtin_memcpy(&u, h, 8);
    *reinterpret_cast<uint2*>(p + e) = u;
  }
}

// grid (chunks, bsz). part[b][chunk][kOut]
// ONE = false: every row's G = F - X is formed from the history (and written to G when G is
// given). ONE = true (the steady state): only row `fr` is new; it is formed from F - X and
// written to G, the other rows are read from G. Every load is unconditional from a
// wave-uniformly chosen address (a load under a branch is waited for at the join: N serial
// memory latencies per iteration otherwise): with ONE, row fr's G load re-reads its X line (a
// cache hit) instead of a stale G line. |F[last]|^2 needs last == fr with ONE (host-checked).
template <int N, bool ONE, typename FT, typename HT>
__global__ __launch_bounds__(kThreads) void gram_kernel(const HT* __restrict__ X, const FT* __restrict__ F,
                                                        HT* __restrict__ G, float* __restrict__ part, int64_t d4,
                                                        int64_t row_stride, int64_t batch_stride, int64_t chunk4,
                                                        int last, int fr) {
  const int b = blockIdx.y;
  const int c = blockIdx.x;
  const HT* xb = X + b * batch_stride;
  const FT* fb = F + b * batch_stride;
  HT* gb = G != nullptr ? G + b * batch_stride : nullptr;
  float acc[kPairs];
  float fn = 0.f;
#pragma unroll
  for (int p = 0; p < kPairs; ++p) acc[p] = 0.f;
  const int64_t v0 = static_cast<int64_t>(c) * chunk4;
  int64_t v1 = v0 + chunk4;
  if (v1 > d4) v1 = d4;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads) {
    const int64_t e = 4 * v;
    float4 g[N];
    if constexpr (ONE) {
      const float4 f = ldf4(fb, fr * row_stride + e);
      const float4 x = ldf4(xb, fr * row_stride + e);
#pragma unroll
      for (int i = 0; i < N; ++i) g[i] = ldf4((i == fr ? xb : static_cast<const HT*>(gb)), i * row_stride + e);
      const float4 gn = make_float4(f.x - x.x, f.y - x.y, f.z - x.z, f.w - x.w);
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (i == fr) g[i] = gn;
      st4(gb, fr * row_stride + e, gn);
      fn += dot4(f, f);
    } else {
      float4 f[N], x[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        f[i] = ldf4(fb, i * row_stride + e);
        x[i] = ldf4(xb, i * row_stride + e);
      }
#pragma unroll
      for (int i = 0; i < N; ++i) {
        g[i] = make_float4(f[i].x - x[i].x, f[i].y - x[i].y, f[i].z - x[i].z, f[i].w - x[i].w);
        if (gb != nullptr) st4(gb, i * row_stride + e, g[i]);
        if (i == last) fn += dot4(f[i], f[i]);
      }
    }
    int p = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = i; j < N; ++j) acc[p++] += dot4(g[i], g[j]);
  }
  __shared__ float red[kThreads / 64][kOut];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int kUsed = N * (N + 1) / 2;
#pragma unroll
  for (int p = 0; p < kUsed; ++p) {
    const float s = wave_sum(acc[p]);
    if (lane == 0) red[wave][p] = s;
  }
  {
    const float s = wave_sum(fn);
    if (lane == 0) red[wave][kPairs] = s;
  }
  __syncthreads();
  float* out = part + (static_cast<int64_t>(b) * gridDim.x + c) * kOut;
  for (int p = threadIdx.x; p < kOut; p += kThreads) {
    if (p < kUsed || p == kPairs) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kThreads / 64; ++w) s += red[w][p];
      out[p] = s;
    } else {
      out[p] = 0.f;
    }
  }
}

// grid (ceil(d4 / kThreads), bsz): X[b, slot] = beta * sum_i a_i F[b,i] + (1-beta) * sum_i a_i X[b,i]
template <int N, bool MIXX, typename Z, typename FT, typename HT>
__global__ __launch_bounds__(kThreads) void mix_kernel(HT* __restrict__ X, const FT* __restrict__ F,
                                                       const float* __restrict__ alpha, Z* __restrict__ z, int64_t d4,
                                                       int64_t row_stride, int64_t batch_stride, int slot, float beta) {
  const int b = blockIdx.y;
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (v >= d4) return;
  const int64_t e = 4 * v;
  HT* xb = X + b * batch_stride;
  const FT* fb = F + b * batch_stride;
  float a[N];
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = alpha[b * N + i];
  float4 sf = make_float4(0.f, 0.f, 0.f, 0.f), sx = sf;
  float4 fv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) fv[i] = ldf4(fb, i * row_stride + e);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    sf.x += a[i] * fv[i].x; sf.y += a[i] * fv[i].y; sf.z += a[i] * fv[i].z; sf.w += a[i] * fv[i].w;
    if (MIXX) {
      const float4 x = ldf4(static_cast<const HT*>(xb), i * row_stride + e);
      sx.x += a[i] * x.x; sx.y += a[i] * x.y; sx.z += a[i] * x.z; sx.w += a[i] * x.w;
    }
  }
  float4 o = sf;
  if (MIXX) {
    const float c = 1.f - beta;
    o = make_float4(beta * sf.x + c * sx.x, beta * sf.y + c * sx.y, beta * sf.z + c * sx.z, beta * sf.w + c * sx.w);
  }
  st4(xb, slot * row_stride + e, o);
  if (z != nullptr) {
    Z* zp = z + static_cast<int64_t>(b) * d4 * 4 + e;
    zp[0] = static_cast<Z>(o.x);
    zp[1] = static_cast<Z>(o.y);
    zp[2] = static_cast<Z>(o.z);
    zp[3] = static_cast<Z>(o.w);
  }
}

// One launch for everything between the Gram pass and the mix (was ~15 tiny PyTorch / rocSOLVER
// launches per solver iteration: chunk sum, symmetric gather, residual sums / sqrt / divide, H
// assembly, getrf + two triangular solves, the alpha slice copy). One workgroup, thread b owns
// batch element b: it sums its Gram chunk partials, builds
//     H = [[0, 1^T], [1, G G^T + lam I]]   ((n+1) x (n+1)),  y = e_0
// in registers and solves H a = y by Gaussian elimination with partial pivoting (LAPACK getrf's
// pivot choice: the first largest |H[r][k]|; row swaps as compile-time-indexed selects, so
// nothing is dynamically indexed / spilled); alpha[b] = a[1..n]. `res` (nullable): the relative
// residual of the previous iterate, sqrt(sum_b G G^T[last][last]) / (1e-5 + sqrt(sum_b |F_last|^2)),
// reduced over the workgroup.
template <int N>
__global__ __launch_bounds__(1024) void solve_kernel(const float* __restrict__ part, int chunks, int bsz, int last,
                                                     float lam, float* __restrict__ alpha, float* __restrict__ res) {
  constexpr int P = N * (N + 1) / 2, M = N + 1;
  const int b = threadIdx.x;
  float g[P];
  float fn = 0.f;
#pragma unroll
  for (int p = 0; p < P; ++p) g[p] = 0.f;
  if (b < bsz) {
    const float* pp = part + static_cast<int64_t>(b) * chunks * kOut;
    for (int c = 0; c < chunks; ++c) {
#pragma unroll
      for (int p = 0; p < P; ++p) g[p] += pp[c * kOut + p];
      fn += pp[c * kOut + kPairs];
    }
  }
  auto pidx = [](int i, int j) { return i * N - i * (i - 1) / 2 + (j - i); };  // i <= j, row-major triangle
  if (res != nullptr) {
    float dl = 0.f;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (i == last) dl = g[pidx(i, i)];
    __shared__ float red[2][16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float s1 = wave_sum(dl), s2 = wave_sum(fn);
    if (lane == 0) {
      red[0][wave] = s1;
      red[1][wave] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a1 = 0.f, a2 = 0.f;
      for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) {
        a1 += red[0][w];
        a2 += red[1][w];
      }
      res[0] = sqrtf(a1) / (1e-5f + sqrtf(a2));
    }
  }
  if (b >= bsz) return;
  float H[M][M], y[M];
#pragma unroll
  for (int r = 0; r < M; ++r) {
    y[r] = r == 0 ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < M; ++c) {
      float v;
      if (r == 0 && c == 0) v = 0.f;
      else if (r == 0 || c == 0) v = 1.f;
      else v = g[r <= c ? pidx(r - 1, c - 1) : pidx(c - 1, r - 1)] + (r == c ? lam : 0.f);
      H[r][c] = v;
    }
  }
#pragma unroll
  for (int k = 0; k < M; ++k) {
    int piv = k;
    float best = fabsf(H[k][k]);
#pragma unroll
    for (int r = k + 1; r < M; ++r) {
      const float a = fabsf(H[r][k]);
      if (a > best) {
        best = a;
        piv = r;
      }
    }
#pragma unroll
    for (int r = k + 1; r < M; ++r) {
      if (r == piv) {
#pragma unroll
        for (int c = 0; c < M; ++c) {
          const float t = H[k][c];
          H[k][c] = H[r][c];
          H[r][c] = t;
        }
        const float t = y[k];
        y[k] = y[r];
        y[r] = t;
      }
    }
    const float inv = 1.f / H[k][k];
#pragma unroll
    for (int r = k + 1; r < M; ++r) {
      const float f = H[r][k] * inv;
#pragma unroll
      for (int c = k + 1; c < M; ++c) H[r][c] = fmaf(-f, H[k][c], H[r][c]);
      y[r] = fmaf(-f, y[k], y[r]);
    }
  }
  float x[M];
#pragma unroll
  for (int k = M - 1; k >= 0; --k) {
    float sacc = y[k];
#pragma unroll
    for (int c = k + 1; c < M; ++c) sacc = fmaf(-H[k][c], x[c], sacc);
    x[k] = sacc / H[k][k];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) alpha[static_cast<int64_t>(b) * N + i] = x[i + 1];
}

// DEQ adjoint fixed-point step, one pass: u_new = vjp + grad (model dtype, rounded like the
// PyTorch add) and per-workgroup partial sums of (u_new - u)^2 in fp32 (the convergence test;
// summed by gemm_splitk_reduce) — instead of an add, a subtract and a norm pass (7 tensor
// passes -> 4).
template <typename T>
__global__ __launch_bounds__(kThreads) void adjoint_step_kernel(const T* __restrict__ vjp, const T* __restrict__ grad,
                                                                const T* __restrict__ u, T* __restrict__ u_new,
                                                                float* __restrict__ part, int64_t n8) {
  float acc = 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; v < n8; v += stride) {
    T a[8], g[8], o[8], r[8];
    load8(vjp + v * 8, a);
    load8(grad + v * 8, g);
    load8(u + v * 8, o);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r[j] = static_cast<T>(static_cast<float>(a[j]) + static_cast<float>(g[j]));
      const float dlt = static_cast<float>(r[j]) - static_cast<float>(o[j]);
      acc = fmaf(dlt, dlt, acc);
    }
    store8(u_new + v * 8, r);
  }
  __shared__ float red[kThreads / 64];
  const float s = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) t += red[w];
    part[blockIdx.x] = t;
  }
}

// X / G (fp32 or bf16) and F (fp32 or bf16) share one element layout: [bsz][rows of row_stride][d]
void check_layout(const void* X, const void* F, int64_t d, int64_t row_stride, int64_t batch_stride, int n) {
  if (n < 1 || n > kMaxRows) throw std::runtime_error("anderson: need 1 <= n <= 8 (got " + std::to_string(n) + ")");
  if (d % 4 != 0 || row_stride % 4 != 0 || batch_stride % 4 != 0 || row_stride < d)
    throw std::runtime_error("anderson: d and strides must be multiples of 4 elements");
  if (((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(F)) & 15u) != 0)
    throw std::runtime_error("anderson: X and F must be 16-byte aligned");
}

}  // namespace

int anderson_gram_chunks(int64_t bsz, int64_t d) {
  // >= ~2048 workgroups over the batch, >= 4 float4 per lane per chunk
  const int64_t d4 = d / 4;
  int64_t chunks = (2048 + bsz - 1) / (bsz > 0 ? bsz : 1);
  const int64_t max_chunks = (d4 + 4 * kThreads - 1) / (4 * kThreads);
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks < 1) chunks = 1;
  return static_cast<int>(chunks);
}

template <int N, bool ONE, typename HT>
void gram_launch(const HT* X, const void* F, int fdt, HT* G, float* part, dim3 grid, int64_t d4, int64_t rs,
                 int64_t bs, int64_t chunk4, int last, int fr, hipStream_t s) {
  if (fdt == kBF16)
    gram_kernel<N, ONE, bf16, HT><<<grid, kThreads, 0, s>>>(X, static_cast<const bf16*>(F), G, part, d4, rs, bs, chunk4,
                                                            last, fr);
  else
    gram_kernel<N, ONE, float, HT><<<grid, kThreads, 0, s>>>(X, static_cast<const float*>(F), G, part, d4, rs, bs,
                                                             chunk4, last, fr);
}

template <typename HT>
void gram_dispatch(const HT* X, const void* F, int f_dtype, HT* G, bool one, float* partials, dim3 grid, int64_t d4,
                   int64_t row_stride, int64_t batch_stride, int64_t chunk4, int n, int last, hipStream_t stream) {
#define GRAM_CASE(NN)                                                                                              \
  case NN:                                                                                                         \
    if (one) gram_launch<NN, true>(X, F, f_dtype, G, partials, grid, d4, row_stride, batch_stride, chunk4, last,  \
                                   last, stream);                                                                  \
    else gram_launch<NN, false>(X, F, f_dtype, G, partials, grid, d4, row_stride, batch_stride, chunk4, last, 0,  \
                                stream);                                                                           \
    break;
  switch (n) {
    GRAM_CASE(1) GRAM_CASE(2) GRAM_CASE(3) GRAM_CASE(4) GRAM_CASE(5) GRAM_CASE(6) GRAM_CASE(7) GRAM_CASE(8)
  }
#undef GRAM_CASE
}

void anderson_gram(const void* X, const void* F, int f_dtype, void* G, unsigned fresh, float* partials, int64_t bsz,
                   int64_t d, int64_t row_stride, int64_t batch_stride, int n, int last, int chunks, hipStream_t stream,
                   int h_dtype) {
  check_layout(X, F, d, row_stride, batch_stride, n);
  if (f_dtype != kF32 && f_dtype != kBF16) throw std::runtime_error("anderson_gram: F must be fp32 or bf16");
  if (h_dtype != kF32 && h_dtype != kBF16) throw std::runtime_error("anderson_gram: X / G must be fp32 or bf16");
  if (G != nullptr && (reinterpret_cast<uintptr_t>(G) & 15u) != 0)
    throw std::runtime_error("anderson_gram: G must be 16-byte aligned");
  if (last < 0 || last >= n) throw std::runtime_error("anderson_gram: last row out of range");
  if (bsz > 65535) throw std::runtime_error("anderson_gram: bsz > 65535");
  const int64_t d4 = d / 4;
  const int64_t chunk4 = (d4 + chunks - 1) / chunks;
  dim3 grid(chunks, static_cast<unsigned>(bsz));
  // one new row (the steady state): the others come from G; otherwise every row from F - X
  const bool one = G != nullptr && fresh == (1u << last);
  if (h_dtype == kBF16)
    gram_dispatch(static_cast<const bf16*>(X), F, f_dtype, static_cast<bf16*>(G), one, partials, grid, d4, row_stride,
                  batch_stride, chunk4, n, last, stream);
  else
    gram_dispatch(static_cast<const float*>(X), F, f_dtype, static_cast<float*>(G), one, partials, grid, d4,
                  row_stride, batch_stride, chunk4, n, last, stream);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

template <int N, bool MIXX, typename FT, typename HT>
void mix_launch(HT* X, const FT* F, const float* alpha, void* z, int zdt, int64_t bsz, int64_t d4, int64_t rs,
                int64_t bs, int slot, float beta, hipStream_t s) {
  dim3 grid(static_cast<unsigned>((d4 + kThreads - 1) / kThreads), static_cast<unsigned>(bsz));
  switch (zdt) {
    case kBF16: mix_kernel<N, MIXX, bf16, FT, HT><<<grid, kThreads, 0, s>>>(X, F, alpha, static_cast<bf16*>(z), d4, rs, bs, slot, beta); break;
    case kF16: mix_kernel<N, MIXX, f16, FT, HT><<<grid, kThreads, 0, s>>>(X, F, alpha, static_cast<f16*>(z), d4, rs, bs, slot, beta); break;
    case kF32: mix_kernel<N, MIXX, float, FT, HT><<<grid, kThreads, 0, s>>>(X, F, alpha, static_cast<float*>(z), d4, rs, bs, slot, beta); break;
    default: throw std::runtime_error("anderson_mix: unsupported z dtype");
  }
}

template <typename HT>
void mix_dispatch(HT* X, const void* F, int f_dtype, const float* alpha, void* z, int zdt, int64_t bsz, int64_t d4,
                  int64_t row_stride, int64_t batch_stride, int n, int slot, float beta, hipStream_t stream) {
  const bool mixx = beta != 1.f;
  const bf16* fh = static_cast<const bf16*>(F);
  const float* ff = static_cast<const float*>(F);
#define MIX_CASE(NN)                                                                                              \
  case NN:                                                                                                        \
    if (f_dtype == kBF16) {                                                                                       \
      if (mixx) mix_launch<NN, true>(X, fh, alpha, z, zdt, bsz, d4, row_stride, batch_stride, slot, beta, stream); \
      else mix_launch<NN, false>(X, fh, alpha, z, zdt, bsz, d4, row_stride, batch_stride, slot, beta, stream);    \
    } else {                                                                                                      \
      if (mixx) mix_launch<NN, true>(X, ff, alpha, z, zdt, bsz, d4, row_stride, batch_stride, slot, beta, stream); \
      else mix_launch<NN, false>(X, ff, alpha, z, zdt, bsz, d4, row_stride, batch_stride, slot, beta, stream);    \
    }                                                                                                             \
    break;
  switch (n) {
    MIX_CASE(1) MIX_CASE(2) MIX_CASE(3) MIX_CASE(4) MIX_CASE(5) MIX_CASE(6) MIX_CASE(7) MIX_CASE(8)
  }
#undef MIX_CASE
}

void anderson_mix(void* X, const void* F, int f_dtype, const float* alpha, void* z, int z_dtype, int64_t bsz,
                  int64_t d, int64_t row_stride, int64_t batch_stride, int n, int slot, float beta, hipStream_t stream,
                  int h_dtype) {
  check_layout(X, F, d, row_stride, batch_stride, n);
  if (f_dtype != kF32 && f_dtype != kBF16) throw std::runtime_error("anderson_mix: F must be fp32 or bf16");
  if (h_dtype != kF32 && h_dtype != kBF16) throw std::runtime_error("anderson_mix: X must be fp32 or bf16");
  if (slot < 0 || slot * row_stride + d > batch_stride) throw std::runtime_error("anderson_mix: slot out of range");
  if (bsz > 65535) throw std::runtime_error("anderson_mix: bsz > 65535");
  if (z != nullptr && (reinterpret_cast<uintptr_t>(z) & 7u) != 0)
    throw std::runtime_error("anderson_mix: z must be 8-byte aligned");
  const int64_t d4 = d / 4;
  const int zdt = z != nullptr ? z_dtype : kF32;
  if (h_dtype == kBF16)
    mix_dispatch(static_cast<bf16*>(X), F, f_dtype, alpha, z, zdt, bsz, d4, row_stride, batch_stride, n, slot, beta,
                 stream);
  else
    mix_dispatch(static_cast<float*>(X), F, f_dtype, alpha, z, zdt, bsz, d4, row_stride, batch_stride, n, slot, beta,
                 stream);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void anderson_solve(const float* partials, int chunks, int64_t bsz, int n, int last, float lam, float* alpha,
                    float* res, hipStream_t stream) {
  if (n < 1 || n > kMaxRows) throw std::runtime_error("anderson_solve: need 1 <= n <= 8");
  if (bsz < 1 || bsz > 1024) throw std::runtime_error("anderson_solve: need 1 <= bsz <= 1024 (one workgroup)");
  if (chunks < 1 || last < 0 || last >= n) throw std::runtime_error("anderson_solve: bad chunks / last row");
  const unsigned threads = static_cast<unsigned>((bsz + 63) / 64 * 64);
#define SOLVE_CASE(NN) \
  case NN: solve_kernel<NN><<<1, threads, 0, stream>>>(partials, chunks, static_cast<int>(bsz), last, lam, alpha, res); break;
  switch (n) {
    SOLVE_CASE(1) SOLVE_CASE(2) SOLVE_CASE(3) SOLVE_CASE(4) SOLVE_CASE(5) SOLVE_CASE(6) SOLVE_CASE(7) SOLVE_CASE(8)
  }
#undef SOLVE_CASE
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

int adjoint_step_blocks(int64_t n) {
  int64_t b = (n / 8 + kThreads * 4 - 1) / (kThreads * 4);  // >= 4 vectors per lane
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

void adjoint_step(const void* vjp, const void* grad, const void* u, void* u_new, float* partials, int blocks,
                  int64_t n, int dtype, hipStream_t stream) {
  if (n % 8 != 0 || blocks < 1) throw std::runtime_error("adjoint_step: need n % 8 == 0 and blocks >= 1");
  if (((reinterpret_cast<uintptr_t>(vjp) | reinterpret_cast<uintptr_t>(grad) | reinterpret_cast<uintptr_t>(u) |
        reinterpret_cast<uintptr_t>(u_new)) & 15u) != 0)
    throw std::runtime_error("adjoint_step: tensors must be 16-byte aligned");
  switch (dtype) {
    case kBF16:
      adjoint_step_kernel<bf16><<<blocks, kThreads, 0, stream>>>(static_cast<const bf16*>(vjp), static_cast<const bf16*>(grad),
                                                                  static_cast<const bf16*>(u), static_cast<bf16*>(u_new),
                                                                  partials, n / 8);
      break;
    case kF16:
      adjoint_step_kernel<f16><<<blocks, kThreads, 0, stream>>>(static_cast<const f16*>(vjp), static_cast<const f16*>(grad),
                                                                 static_cast<const f16*>(u), static_cast<f16*>(u_new),
                                                                 partials, n / 8);
      break;
    case kF32:
      adjoint_step_kernel<float><<<blocks, kThreads, 0, stream>>>(static_cast<const float*>(vjp), static_cast<const float*>(grad),
                                                                   static_cast<const float*>(u), static_cast<float*>(u_new),
                                                                   partials, n / 8);
      break;
    default:
      throw std::runtime_error("adjoint_step: bf16 / fp16 / fp32 only");
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
