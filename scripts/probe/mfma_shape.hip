// MFMA shape under load on MI355X: v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 in bare
// loops on random bf16 operands held in registers, every CU issuing (1 or 2 waves per SIMD).
// Prints achieved TFLOP/s and the implied clock for each shape: the answer to "would gemm_nt's
// wave tiles gain from the 32x32x16 instruction" (same cycles per FLOP by the ISA tables; the chip
// clock under load can differ by shape). Build: hipcc --offload-arch=gfx950 -O3 mfma_shape.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// SHAPE 0: 16x16x32 on 4 accumulators; 1: 32x32x16 on 2 accumulators (the same FLOPs per loop trip)
template <int SHAPE>
__global__ __launch_bounds__(512) void mfma_loop(const bf16x8* __restrict__ src, float* __restrict__ out, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 a0 = src[(tid * 4 + 0) & 65535], a1 = src[(tid * 4 + 1) & 65535];
  bf16x8 b0 = src[(tid * 4 + 2) & 65535], b1 = src[(tid * 4 + 3) & 65535];
  float s = 0.f;
  if constexpr (SHAPE == 0) {
    f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
      // 8 MFMAs x 16384 FLOP per trip
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, c3, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, c3, 0, 0, 0);
    }
    for (int j = 0; j < 4; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  } else {
    f32x16 c0 = {}, c1 = {};
    for (int i = 0; i < iters; ++i) {
      // 4 MFMAs x 32768 FLOP per trip
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c1, 0, 0, 0);
    }
    for (int j = 0; j < 16; ++j) s += c0[j] + c1[j];
  }
  out[tid] = s;  // vector store: keeps the loop alive
}

template <int SHAPE>
double run(const bf16x8* src, float* out, int cus, int waves_per_simd, int iters) {
  const int threads = 64 * 4 * waves_per_simd;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  mfma_loop<SHAPE><<<cus, threads>>>(src, out, iters / 10);  // warm-up (clocks settle)
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e0));
  mfma_loop<SHAPE><<<cus, threads>>>(src, out, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double flop = static_cast<double>(cus) * (threads / 64) * iters * 8.0 * 16384.0;
  return flop / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200000;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint16_t> h(65536 * 8);
  srand(1);
  for (auto& v : h) {  // random bf16 in [-1, 1): sign, exponent 120..126, random mantissa
    const uint16_t sign = (rand() & 1) << 15, ex = static_cast<uint16_t>(120 + rand() % 7) << 7;
    v = sign | ex | static_cast<uint16_t>(rand() & 127);
  }
  bf16x8* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, static_cast<size_t>(cus) * 512 * 4));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  for (int w = 1; w <= 2; ++w)
    for (int rep = 0; rep < 2; ++rep) {
      const double t16 = run<0>(src, out, cus, w, iters);
      const double t32 = run<1>(src, out, cus, w, iters);
      // 16x16x32: 16 cycles per MFMA, 32x32x16: 32 cycles (per SIMD) -> implied clock
      printf("{\"waves_per_simd\": %d, \"rep\": %d, \"mfma16x16x32_tflops\": %.1f, \"mfma32x32x16_tflops\": %.1f, "
             "\"ratio_16_over_32\": %.3f, \"implied_ghz_16\": %.3f, \"implied_ghz_32\": %.3f}\n",
             w, rep, t16, t32, t16 / t32, t16 * 1e12 / (cus * 4 * 16384.0 / 16.0) / 1e9,
             t32 * 1e12 / (cus * 4 * 32768.0 / 32.0) / 1e9);
    }
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
