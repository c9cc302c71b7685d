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

// wave sums by DPP + readlane (common.h): no LDS round trips (the ds_bpermute butterfly was 6
// dependent LDS ops per reduction, on every row's critical path)
__device__ __forceinline__ float wave_sum(float v) { return wave_sum_dpp(v); }

__device__ __forceinline__ void ld8w(const float* __restrict__ p, int c0, float (&v)[8]) {
  const float4 a0 = *reinterpret_cast<const float4*>(p + c0);
  const float4 a1 = *reinterpret_cast<const float4*>(p + c0 + 4);
  v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w;
  v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
}

// the affine in the activation dtype (a bf16 model's LayerNorm parameters as they are: no
// per-call fp32 copies of w and b, two tiny cast kernels per LayerNorm per step)
template <typename A>
__device__ __forceinline__ void ld8w(const A* __restrict__ p, int c0, float (&v)[8]) {
  A t[8];
  load8(p + c0, t);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = static_cast<float>(t[j]);
}

// A lane's vectors i = lane + 64 * i of a row; lanes past the row (D/8 not a multiple of 64)
// load vector 0 and are masked in the math: every load is unconditional (a load under
// `if (v < nv)` is waited for at the branch join, one exposed latency per vector).
template <int VPL>
struct LnLanes {
  int vc[VPL];
  bool act[VPL];
  __device__ __forceinline__ LnLanes(int lane, int nv) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int v = lane + i * 64;
      act[i] = v < nv;
      vc[i] = act[i] ? v : 0;
    }
  }
};

// Forward: a persistent grid (one full round of resident workgroups); each wave walks rows
// row, row + step, ... with the NEXT row's x (and residual) loads issued before the current
// row's reductions, and the affine w/b held in registers for the whole kernel (16-byte
// loads, once). (The one-row-per-wave version had only one row's loads in flight: 141-155 us
// per ViT-B LayerNorm (50432 x 768 bf16) on MI355X, ~2-3x its HBM time, s48 trace.)
template <typename T, bool ADD, int VPL, typename A>
__global__ __launch_bounds__(kThreads) void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                          T* __restrict__ h, T* __restrict__ y,
                                                          const A* __restrict__ w, const A* __restrict__ b,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int64_t rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const LnLanes<VPL> L(lane, D / 8);
  const float inv_d = 1.f / static_cast<float>(D);
  float wv[VPL][8], bv[VPL][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    ld8w(w, L.vc[i] * 8, wv[i]);
    ld8w(b, L.vc[i] * 8, bv[i]);
  }
  const int64_t step = static_cast<int64_t>(gridDim.x) * kWaves;
  int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;  // no block-level synchronisation below
  T rx[VPL][8], rr[VPL][8];
  auto load = [&](int64_t rw, T (&ox)[VPL][8], T (&orr)[VPL][8]) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      load8(x + rw * D + L.vc[i] * 8, ox[i]);
      if (ADD) load8(r + rw * D + L.vc[i] * 8, orr[i]);
    }
  };
  // one row: (h,) the statistics, y
  auto process = [&](int64_t rw, const T (&cx)[VPL][8], const T (&cr)[VPL][8]) {
    float f[VPL][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[i][j] = static_cast<float>(cx[i][j]);
      if (ADD) {
        T o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = static_cast<T>(f[i][j] + static_cast<float>(cr[i][j]));
          f[i][j] = static_cast<float>(o[j]);  // normalise exactly the stored (rounded) h
        }
        if (L.act[i]) store8(h + rw * D + L.vc[i] * 8, o);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += L.act[i] ? f[i][j] : 0.f;
    }
    const float mean = wave_sum(s) * inv_d;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = f[i][j] - mean;
        q = fmaf(L.act[i] ? d : 0.f, d, q);
      }
    const float rstd = rsqrtf(wave_sum(q) * inv_d + eps);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      T o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = static_cast<T>(fmaf((f[i][j] - mean) * rstd, wv[i][j], bv[i][j]));
      if (L.act[i]) store8(y + rw * D + L.vc[i] * 8, o);
    }
    if (lane == 0) {
      mean_out[rw] = mean;
      rstd_out[rw] = rstd;
    }
  };
  // PF (up to 4 vectors per lane): the next row's loads in flight during this row's
  // reductions and stores (unconditional: the last row re-reads itself); wider rows would
  // spill the second buffer
  constexpr bool PF = VPL <= 4;
  load(row, rx, rr);
  while (true) {
    const int64_t nrow = row + step;
    const bool more = nrow < rows;
    if (PF) {
      T nx[VPL][8], nr[VPL][8];
      load(more ? nrow : row, nx, nr);
      process(row, rx, rr);
      if (!more) break;
#pragma unroll
      for (int i = 0; i < VPL; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          rx[i][j] = nx[i][j];
          if (ADD) rr[i][j] = nr[i][j];
        }
    } else {
      process(row, rx, rr);
      if (!more) break;
      load(nrow, rx, rr);
    }
    row = nrow;
  }
}

// Backward: same persistent walk, the next row's (dy, x[, dh_ext], mean, rstd) in flight
// during the current row's two reductions and its dx stores (PF: up to 4 vectors per lane;
// wider rows would spill the second buffer). dy and xhat are recomputed from the raw row in
// the second pass rather than kept as fp32 arrays.
// CS (with DH): also the column sums of dx — in a pre-LN block dx is the gradient of h = x + p
// where p is the previous Linear's output, so these are that Linear's bias gradient (no colsum
// pass over dx afterwards); the partial row is then [3][D].
template <typename T, bool DH, int VPL, typename A, bool CS = false>
__global__ __launch_bounds__(kThreads) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ dh_ext,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in,
                                                          const A* __restrict__ w, T* __restrict__ dx,
                                                          float* __restrict__ part, int64_t rows, int D) {
  constexpr bool PF = VPL <= 4;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2 or 3][D]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = D / 8;
  const LnLanes<VPL> L(lane, nv);
  const float inv_d = 1.f / static_cast<float>(D);
  float wv[VPL][8], dwp[VPL][8], dbp[VPL][8], csp[CS ? VPL : 1][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    ld8w(w, L.vc[i] * 8, wv[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) dwp[i][j] = dbp[i][j] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < (CS ? VPL : 1); ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) csp[i][j] = 0.f;
  struct Buf {
    T d[VPL][8], x[VPL][8], e[DH ? VPL : 1][8];
    float mean, rstd;
  };
  auto load = [&](int64_t rw, Buf& o) {
    o.mean = mean_in[rw];
    o.rstd = rstd_in[rw];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      load8(dy + rw * D + L.vc[i] * 8, o.d[i]);
      load8(x + rw * D + L.vc[i] * 8, o.x[i]);
      if (DH) load8(dh_ext + rw * D + L.vc[i] * 8, o.e[i]);
    }
  };
  auto process = [&](int64_t rw, const Buf& c) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = L.act[i] ? static_cast<float>(c.d[i][j]) : 0.f;
        const float xh = (static_cast<float>(c.x[i][j]) - c.mean) * c.rstd;
        const float g = d * wv[i][j];
        s1 += g;
        s2 = fmaf(g, xh, s2);
        dwp[i][j] = fmaf(d, xh, dwp[i][j]);
        dbp[i][j] += d;
      }
    const float m1 = wave_sum(s1) * inv_d, m2 = wave_sum(s2) * inv_d;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      T o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (static_cast<float>(c.x[i][j]) - c.mean) * c.rstd;
        float g = c.rstd * (static_cast<float>(c.d[i][j]) * wv[i][j] - m1 - xh * m2);
        if (DH) g += static_cast<float>(c.e[i][j]);
        o[j] = static_cast<T>(g);
        if (CS) csp[CS ? i : 0][j] += L.act[i] ? static_cast<float>(o[j]) : 0.f;  // of the stored (rounded) dx
      }
      if (L.act[i]) store8(dx + rw * D + L.vc[i] * 8, o);
    }
  };
  const int64_t step = static_cast<int64_t>(gridDim.x) * kWaves;
  int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wave;
  if (row < rows) {  // (every wave reaches the block reduction below)
    Buf cur;
    load(row, cur);
    while (true) {
      const int64_t nrow = row + step;
      const bool more = nrow < rows;
      if (PF) {
        Buf nxt;
        load(more ? nrow : row, nxt);  // unconditional: the last row re-reads itself
        process(row, cur);
        if (!more) break;
        cur = nxt;
      } else {
        process(row, cur);
        if (!more) break;
        load(nrow, cur);
      }
      row = nrow;
    }
  }
  // block partial of dw / db: the waves add their register partials into one [2][D] LDS
  // row in turn (8*D bytes of LDS whatever the wave count)
  for (int k = 0; k < kWaves; ++k) {
    if (wave == k) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        if (L.act[i])
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int c = L.vc[i] * 8 + j;
            red[c] = k == 0 ? dwp[i][j] : red[c] + dwp[i][j];
            red[D + c] = k == 0 ? dbp[i][j] : red[D + c] + dbp[i][j];
            if (CS) red[2 * D + c] = k == 0 ? csp[CS ? i : 0][j] : red[2 * D + c] + csp[CS ? i : 0][j];
          }
      }
    }
    __syncthreads();
  }
  constexpr int NP = CS ? 3 : 2;
  float* out = part + static_cast<int64_t>(blockIdx.x) * NP * D;
  for (int c = threadIdx.x; c < NP * D; c += kThreads) out[c] = red[c];
}

int vpl_for(int64_t D) {
  if (D % 8 != 0 || D < 8 || D > 8192)
    throw std::runtime_error("fused layernorm: need D % 8 == 0 and 8 <= D <= 8192 (got " + std::to_string(D) + ")");
  const int v = static_cast<int>((D / 8 + 63) / 64);  // vectors per lane actually needed
  for (int c : {1, 2, 3, 4, 6, 8, 12, 16})
    if (c >= v) return c;
  return 16;
}

template <typename T, bool ADD, int VPL, typename A>
void fwd_launch(const void* x, const void* r, void* h, void* y, const void* w, const void* b, float* mean,
                float* rstd, int64_t rows, int64_t D, float eps, hipStream_t s) {
  auto k = ln_fwd_kernel<T, ADD, VPL, A>;
  int64_t blocks = resident_blocks(reinterpret_cast<const void*>(k), kThreads, 0);
  const int64_t need = (rows + kWaves - 1) / kWaves;
  if (blocks > need) blocks = need;
  if (blocks < 1) blocks = 1;
  k<<<(unsigned)blocks, kThreads, 0, s>>>(
      static_cast<const T*>(x), static_cast<const T*>(r), static_cast<T*>(h), static_cast<T*>(y),
      static_cast<const A*>(w), static_cast<const A*>(b), mean, rstd,
      rows, static_cast<int>(D), eps);
}

template <typename T, bool DH, int VPL, typename A, bool CS = false>
int bwd_launch(const void* dy, const void* x, const void* dh, const float* mean, const float* rstd, const void* w,
               void* dx, float* part, int max_blocks, int64_t rows, int64_t D, hipStream_t s) {
  auto k = ln_bwd_kernel<T, DH, VPL, A, CS>;
  const size_t lds = static_cast<size_t>(CS ? 3 : 2) * D * sizeof(float);
  int64_t blocks = resident_blocks(reinterpret_cast<const void*>(k), kThreads, lds);
  const int64_t need = (rows + kWaves - 1) / kWaves;
  if (blocks > need) blocks = need;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  k<<<(unsigned)blocks, kThreads, lds, s>>>(static_cast<const T*>(dy), static_cast<const T*>(x),
                                            static_cast<const T*>(dh), mean, rstd, static_cast<const A*>(w),
                                            static_cast<T*>(dx), part, rows,
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

// the affine is fp32 or in the activation dtype (wdtype == dtype)
static void check_affine(int dtype, int wdtype, const char* who) {
  if (wdtype != static_cast<int>(kF32) && wdtype != dtype)
    throw std::runtime_error(std::string(who) + ": w / b must be fp32 or in the activation dtype");
}

void layernorm_fwd(const void* x, const void* residual, void* h, void* y, const void* w, const void* b, float* mean,
                   float* rstd, int64_t rows, int64_t D, float eps, int dtype, int wdtype, hipStream_t stream) {
  const int vpl = vpl_for(D);
  const bool add = residual != nullptr;
  if (w == nullptr || b == nullptr || (reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(b)) % 16 != 0)
    throw std::runtime_error("fused layernorm: w and b must be 16-byte aligned (ones / zeros when absent)");
  check_affine(dtype, wdtype, "fused layernorm");
  const bool wt = wdtype != static_cast<int>(kF32);
#define CALL_ADD(V) fwd_launch<TT, true, V, AT>(x, residual, h, y, w, b, mean, rstd, rows, D, eps, stream)
#define CALL_NOADD(V) fwd_launch<TT, false, V, AT>(x, residual, h, y, w, b, mean, rstd, rows, D, eps, stream)
#define CALL_ALL                                                                \
  if (add) { LN_VPL_SWITCH(vpl, CALL_ADD) } else { LN_VPL_SWITCH(vpl, CALL_NOADD) }
  switch (dtype) {
    case kBF16: {
      using TT = bf16;
      if (wt) { using AT = bf16; CALL_ALL } else { using AT = float; CALL_ALL }
      break;
    }
    case kF16: {
      using TT = f16;
      if (wt) { using AT = f16; CALL_ALL } else { using AT = float; CALL_ALL }
      break;
    }
    case kF32: {
      using TT = float;
      using AT = float;
      CALL_ALL
      break;
    }
    default:
      throw std::runtime_error("fused layernorm: unsupported dtype");
  }
#undef CALL_ALL
#undef CALL_ADD
#undef CALL_NOADD
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

int layernorm_bwd(const void* dy, const void* x, const void* dh_ext, const float* mean, const float* rstd,
                  const void* w, void* dx, float* partials, int max_blocks, int64_t rows, int64_t D, int dtype,
                  int wdtype, bool colsum, hipStream_t stream) {
  const int vpl = vpl_for(D);
  const bool dh = dh_ext != nullptr;
  if (colsum && !dh) throw std::runtime_error("fused layernorm backward: colsum needs the residual-stream input");
  if (w == nullptr || reinterpret_cast<uintptr_t>(w) % 16 != 0)
    throw std::runtime_error("fused layernorm backward: w must be 16-byte aligned (ones when absent)");
  check_affine(dtype, wdtype, "fused layernorm backward");
  const bool wt = wdtype != static_cast<int>(kF32);
  int blocks = 0;
#define CALL_DH(V) blocks = bwd_launch<TT, true, V, AT>(dy, x, dh_ext, mean, rstd, w, dx, partials, max_blocks, rows, D, stream)
#define CALL_NODH(V) blocks = bwd_launch<TT, false, V, AT>(dy, x, dh_ext, mean, rstd, w, dx, partials, max_blocks, rows, D, stream)
#define CALL_DHCS(V) blocks = bwd_launch<TT, true, V, AT, true>(dy, x, dh_ext, mean, rstd, w, dx, partials, max_blocks, rows, D, stream)
#define CALL_ALL                                                                \
  if (dh && colsum) { LN_VPL_SWITCH(vpl, CALL_DHCS) } else if (dh) { LN_VPL_SWITCH(vpl, CALL_DH) }      \
  else { LN_VPL_SWITCH(vpl, CALL_NODH) }
  switch (dtype) {
    case kBF16: {
      using TT = bf16;
      if (wt) { using AT = bf16; CALL_ALL } else { using AT = float; CALL_ALL }
      break;
    }
    case kF16: {
      using TT = f16;
      if (wt) { using AT = f16; CALL_ALL } else { using AT = float; CALL_ALL }
      break;
    }
    case kF32: {
      using TT = float;
      using AT = float;
      CALL_ALL
      break;
    }
    default:
      throw std::runtime_error("fused layernorm: unsupported dtype");
  }
#undef CALL_ALL
#undef CALL_DH
#undef CALL_DHCS
#undef CALL_NODH
  FLUXMPI_HIP_CHECK(hipGetLastError());
  return blocks;
}

}  // namespace fluxmpi
