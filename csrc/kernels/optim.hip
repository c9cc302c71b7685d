// Fused multi-tensor optimiser steps for gfx950 (K3/K4 of SURVEY §2.4).
//
// The reference delegates to Optimisers.jl, i.e. one broadcast kernel per
// expression per leaf (src/optimizer.jl:22). Adam alone is ~4 passes over
// g, x, m, v per leaf. Here one launch updates every leaf of a bucket in a
// single pass: read g, x (or the fp32 master), m, v once; write x, m, v once.
//
// Numerics follow Optimisers.jl exactly, in the element type's precision
// (fp32 math for bf16/fp16/fp32, fp64 math for fp64):
//   Adam:     m = b1*m + (1-b1)*g ; v = b2*v + (1-b2)*g^2
//             dx = m / (1-b1^t) / (sqrt(v / (1-b2^t)) + eps) * lr   [+ wd*x: AdamW chain]
//             x -= dx
//   Descent:  x -= lr*g
//   Momentum: v = rho*v + lr*g ; x -= v
//   Nesterov: dx = -rho^2*v + (1+rho)*lr*g ; v = rho*v - lr*g ; x -= dx
//
// Optional fp32 master weights give the mixed-precision layout (bf16 param +
// fp32 master/m/v); without them the state dtype equals the parameter dtype,
// which is Optimisers.jl's `zero(x)` layout (bit-compatible state trees).
#include <stdexcept>
#include <string>
#include <vector>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;
constexpr int kIters = 2;
constexpr int kChunk = kThreads * kVec * kIters;  // 4096 elements per workgroup
constexpr int kMaxT = 24;

struct OptArgs {
  uintptr_t p[kMaxT];
  uintptr_t g[kMaxT];
  uintptr_t s1[kMaxT];
  uintptr_t s2[kMaxT];
  uintptr_t w[kMaxT];  // fp32 master (or 0)
  int64_t numel[kMaxT];
  int32_t start[kMaxT + 1];
  int n;
};

template <typename P> struct Comp { using type = float; };
template <> struct Comp<double> { using type = double; };

template <typename P, typename G, typename S, bool MASTER>
struct AdamElem {
  using C = typename Comp<P>::type;
  C lr, b1, b2, eps, bc1, bc2, wd, gs;
  __device__ __forceinline__ void operator()(P& p, G g_in, S& m_io, S& v_io, float& w) const {
    const C g = static_cast<C>(g_in) * gs;
    const C m = b1 * static_cast<C>(m_io) + (C(1) - b1) * g;
    const C v = b2 * static_cast<C>(v_io) + (C(1) - b2) * (g * g);
    C x = MASTER ? static_cast<C>(w) : static_cast<C>(p);
    C dx = m / bc1 / (sqrt(v / bc2) + eps) * lr;
    if (wd != C(0)) dx += wd * x;
    x -= dx;
    m_io = static_cast<S>(m);
    v_io = static_cast<S>(v);
    if (MASTER) w = static_cast<float>(x);
    p = static_cast<P>(x);
  }
};

template <typename P, typename G, typename S, bool MASTER>
__global__ __launch_bounds__(kThreads) void mt_adam_kernel(OptArgs a, AdamHyper h) {
  using C = typename Comp<P>::type;
  const int b = blockIdx.x;
  const int t = find_tensor(a.start, a.n, b);
  const int64_t base = static_cast<int64_t>(b - a.start[t]) * kChunk;
  const int64_t n = a.numel[t];
  const int64_t end = base + kChunk < n ? base + kChunk : n;

  AdamElem<P, G, S, MASTER> op;
  C lr = h.lr, bc1 = h.bc1, bc2 = h.bc2;
  if (h.dev != nullptr) {  // graph mode: step-dependent scalars live on the device
    lr = h.dev[0];
    bc1 = C(1) - static_cast<C>(h.dev[1]);
    bc2 = C(1) - static_cast<C>(h.dev[2]);
  }
  op.lr = lr; op.bc1 = bc1; op.bc2 = bc2;
  op.b1 = h.beta1; op.b2 = h.beta2; op.eps = h.eps; op.wd = h.weight_decay;
  op.gs = h.grad_scale * (h.dev_gscale ? *h.dev_gscale : 1.f);

  P* __restrict__ p = reinterpret_cast<P*>(a.p[t]);
  const G* __restrict__ g = reinterpret_cast<const G*>(a.g[t]);
  S* __restrict__ m = reinterpret_cast<S*>(a.s1[t]);
  S* __restrict__ v = reinterpret_cast<S*>(a.s2[t]);
  float* __restrict__ w = reinterpret_cast<float*>(a.w[t]);
  const int tid = threadIdx.x;
  const bool vec = aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v) && (!MASTER || aligned16(w));
  int64_t scalar_from = base;
  if (vec) {
    const int64_t nvec = (end - base) / kVec;
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const int64_t vi = tid + k * kThreads;
      if (vi < nvec) {
        const int64_t off = base + vi * kVec;
        P pv[kVec]; G gv[kVec]; S mv[kVec]; S vv[kVec]; float wv[kVec];
        load8(g + off, gv);
        load8(m + off, mv);
        load8(v + off, vv);
        if (MASTER) load8(w + off, wv); else load8(p + off, pv);
#pragma unroll
        for (int j = 0; j < kVec; ++j) op(pv[j], gv[j], mv[j], vv[j], wv[j]);
        store8(m + off, mv);
        store8(v + off, vv);
        if (MASTER) store8(w + off, wv);
        store8(p + off, pv);
      }
    }
    scalar_from = base + nvec * kVec;
  }
  for (int64_t i = scalar_from + tid; i < end; i += kThreads) {
    P pv = p[i];
    S mv = m[i], vv = v[i];
    float wv = MASTER ? w[i] : 0.f;
    op(pv, g[i], mv, vv, wv);
    m[i] = mv; v[i] = vv;
    if (MASTER) w[i] = wv;
    p[i] = pv;
  }
}

template <typename P, typename G, typename S, bool MASTER>
struct SgdElem {
  using C = typename Comp<P>::type;
  C lr, rho, wd, gs;
  int mode;  // 0 descent, 1 momentum, 2 nesterov
  __device__ __forceinline__ void operator()(P& p, G g_in, S& buf, float& w) const {
    C x = MASTER ? static_cast<C>(w) : static_cast<C>(p);
    C g = static_cast<C>(g_in) * gs;
    if (wd != C(0)) g += wd * x;
    C dx;
    if (mode == 0) {
      dx = g * lr;
    } else if (mode == 1) {
      const C vel = rho * static_cast<C>(buf) + lr * g;
      buf = static_cast<S>(vel);
      dx = vel;
    } else {
      const C vel0 = static_cast<C>(buf);
      dx = -(rho * rho) * vel0 + (C(1) + rho) * lr * g;
      buf = static_cast<S>(rho * vel0 - lr * g);
    }
    x -= dx;
    if (MASTER) w = static_cast<float>(x);
    p = static_cast<P>(x);
  }
};

template <typename P, typename G, typename S, bool MASTER>
__global__ __launch_bounds__(kThreads) void mt_sgd_kernel(OptArgs a, SgdHyper h) {
  const int b = blockIdx.x;
  const int t = find_tensor(a.start, a.n, b);
  const int64_t base = static_cast<int64_t>(b - a.start[t]) * kChunk;
  const int64_t n = a.numel[t];
  const int64_t end = base + kChunk < n ? base + kChunk : n;
  SgdElem<P, G, S, MASTER> op;
  op.lr = h.dev_lr ? *h.dev_lr : h.lr;
  op.rho = h.momentum; op.wd = h.weight_decay; op.gs = h.grad_scale;
  op.mode = h.momentum == 0.f ? 0 : (h.nesterov ? 2 : 1);
  P* __restrict__ p = reinterpret_cast<P*>(a.p[t]);
  const G* __restrict__ g = reinterpret_cast<const G*>(a.g[t]);
  S* __restrict__ buf = reinterpret_cast<S*>(a.s1[t]);
  float* __restrict__ w = reinterpret_cast<float*>(a.w[t]);
  const bool has_buf = op.mode != 0;
  const int tid = threadIdx.x;
  const bool vec = aligned16(p) && aligned16(g) && (!has_buf || aligned16(buf)) && (!MASTER || aligned16(w));
  int64_t scalar_from = base;
  if (vec) {
    const int64_t nvec = (end - base) / kVec;
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const int64_t vi = tid + k * kThreads;
      if (vi < nvec) {
        const int64_t off = base + vi * kVec;
        P pv[kVec]; G gv[kVec]; S bv[kVec]; float wv[kVec];
        load8(g + off, gv);
        if (has_buf) load8(buf + off, bv);
        if (MASTER) load8(w + off, wv); else load8(p + off, pv);
#pragma unroll
        for (int j = 0; j < kVec; ++j) op(pv[j], gv[j], bv[j], wv[j]);
        if (has_buf) store8(buf + off, bv);
        if (MASTER) store8(w + off, wv);
        store8(p + off, pv);
      }
    }
    scalar_from = base + nvec * kVec;
  }
  for (int64_t i = scalar_from + tid; i < end; i += kThreads) {
    P pv = p[i];
    S bv = has_buf ? buf[i] : S(0);
    float wv = MASTER ? w[i] : 0.f;
    op(pv, g[i], bv, wv);
    if (has_buf) buf[i] = bv;
    if (MASTER) w[i] = wv;
    p[i] = pv;
  }
}

__global__ void adam_advance_kernel(float* dev, float b1, float b2) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    dev[1] *= b1;
    dev[2] *= b2;
  }
}

template <typename F>
void for_each_group(const std::vector<uintptr_t>& p, const std::vector<uintptr_t>& g,
                    const std::vector<uintptr_t>& s1, const std::vector<uintptr_t>& s2,
                    const std::vector<uintptr_t>& w, const std::vector<int64_t>& numel, F&& launch) {
  const size_t N = numel.size();
  if (p.size() != N || g.size() != N) throw std::runtime_error("optimizer kernel: list length mismatch");
  if ((!s1.empty() && s1.size() != N) || (!s2.empty() && s2.size() != N) || (!w.empty() && w.size() != N))
    throw std::runtime_error("optimizer kernel: state list length mismatch");
  OptArgs a{};
  int n = 0;
  int32_t blocks = 0;
  auto flush = [&]() {
    if (n == 0) return;
    a.n = n;
    a.start[n] = blocks;
    launch(a, blocks);
    a = OptArgs{};
    n = 0;
    blocks = 0;
  };
  for (size_t i = 0; i < N; ++i) {
    if (numel[i] <= 0) continue;
    const int64_t nb = (numel[i] + kChunk - 1) / kChunk;
    if (n == kMaxT || int64_t(blocks) + nb > (int64_t(1) << 30)) flush();
    a.p[n] = p[i];
    a.g[n] = g[i];
    a.s1[n] = s1.empty() ? 0 : s1[i];
    a.s2[n] = s2.empty() ? 0 : s2[i];
    a.w[n] = w.empty() ? 0 : w[i];
    a.numel[n] = numel[i];
    a.start[n] = blocks;
    blocks += static_cast<int32_t>(nb);
    ++n;
  }
  flush();
}

#define OPT_DTYPE_COMBOS(X)            \
  X(float, float, float, false)          \
  X(float, bf16, float, false)           \
  X(bf16, bf16, bf16, false)             \
  X(bf16, bf16, float, false)            \
  X(bf16, bf16, float, true)             \
  X(bf16, float, float, true)            \
  X(f16, f16, f16, false)                \
  X(f16, f16, float, false)              \
  X(f16, f16, float, true)               \
  X(f16, float, float, true)             \
  X(double, double, double, false)

template <typename T> constexpr int code_of();
template <> constexpr int code_of<float>() { return kF32; }
template <> constexpr int code_of<bf16>() { return kBF16; }
template <> constexpr int code_of<f16>() { return kF16; }
template <> constexpr int code_of<double>() { return kF64; }

}  // namespace

void mt_adam(const std::vector<uintptr_t>& param, const std::vector<uintptr_t>& grad,
             const std::vector<uintptr_t>& m, const std::vector<uintptr_t>& v,
             const std::vector<uintptr_t>& master, const std::vector<int64_t>& numel,
             int p_dtype, int g_dtype, int s_dtype, const AdamHyper& h, hipStream_t stream) {
  const bool has_master = !master.empty();
  if (m.size() != numel.size() || v.size() != numel.size()) throw std::runtime_error("mt_adam: need m and v");
  for_each_group(param, grad, m, v, master, numel, [&](const OptArgs& a, int blocks) {
    bool done = false;
#define X(P, G, S, M)                                                                            \
  if (!done && p_dtype == code_of<P>() && g_dtype == code_of<G>() && s_dtype == code_of<S>() && \
      has_master == M) {                                                                         \
    mt_adam_kernel<P, G, S, M><<<blocks, kThreads, 0, stream>>>(a, h);                           \
    done = true;                                                                                 \
  }
    OPT_DTYPE_COMBOS(X)
#undef X
    if (!done)
      throw std::runtime_error("mt_adam: unsupported dtype combination p=" + std::to_string(p_dtype) +
                               " g=" + std::to_string(g_dtype) + " s=" + std::to_string(s_dtype) +
                               " master=" + std::to_string(has_master));
    FLUXMPI_HIP_CHECK(hipGetLastError());
  });
}

void adam_advance(float* dev, float beta1, float beta2, hipStream_t stream) {
  adam_advance_kernel<<<1, 64, 0, stream>>>(dev, beta1, beta2);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void mt_sgd(const std::vector<uintptr_t>& param, const std::vector<uintptr_t>& grad,
            const std::vector<uintptr_t>& buf, const std::vector<uintptr_t>& master,
            const std::vector<int64_t>& numel, int p_dtype, int g_dtype, int s_dtype,
            const SgdHyper& h, hipStream_t stream) {
  const bool has_master = !master.empty();
  if (h.momentum != 0.f && buf.size() != numel.size())
    throw std::runtime_error("mt_sgd: momentum needs buffers");
  for_each_group(param, grad, buf, {}, master, numel, [&](const OptArgs& a, int blocks) {
    bool done = false;
#define X(P, G, S, M)                                                                            \
  if (!done && p_dtype == code_of<P>() && g_dtype == code_of<G>() && s_dtype == code_of<S>() && \
      has_master == M) {                                                                         \
    mt_sgd_kernel<P, G, S, M><<<blocks, kThreads, 0, stream>>>(a, h);                            \
    done = true;                                                                                 \
  }
    OPT_DTYPE_COMBOS(X)
#undef X
    if (!done) throw std::runtime_error("mt_sgd: unsupported dtype combination");
    FLUXMPI_HIP_CHECK(hipGetLastError());
  });
}

}  // namespace fluxmpi
