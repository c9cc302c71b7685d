// tanh-form GELU, NNlib's `gelu` (the activation of the reference's Lux / Metalhead ViT) and
// hipBLASLt's GELU epilogue: gelu(x) = x/2 (1 + tanh(u)), u = sqrt(2/pi) (x + 0.044715 x^3).
// tanh(u) = 1 - 2 / (1 + exp(2u)): one v_exp_f32 + one v_rcp_f32, saturating to +-1 without
// branches (exp2 -> inf gives 1, -> 0 gives -1).
#pragma once
#include <hip/hip_runtime.h>

namespace fluxmpi {

__device__ __forceinline__ float gelu_tanh_t(float x) {
  constexpr float kK0 = 0.79788456080286536f, kK1 = 0.044715f, k2Log2e = 2.8853900817779268f;
  const float u = kK0 * x * fmaf(kK1 * x, x, 1.f);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(k2Log2e * u));
}

__device__ __forceinline__ float gelu_tanh(float x) { return 0.5f * x * (1.f + gelu_tanh_t(x)); }

// d gelu / dx = (1 + t) / 2 + x/2 (1 - t^2) sqrt(2/pi) (1 + 3 * 0.044715 x^2)
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  constexpr float kK0 = 0.79788456080286536f, kK3 = 3.f * 0.044715f;
  const float t = gelu_tanh_t(x);
  return fmaf(0.5f * x * fmaf(-t, t, 1.f), kK0 * fmaf(kK3 * x, x, 1.f), 0.5f * (1.f + t));
}

}  // namespace fluxmpi
