// Token-major Linear GEMMs on 256 x 256 tiles with fused epilogues — gfx950.
//
//   forward      C[m][n] = sum_k A[m][k] W[n][k]  (+ bias[n])           B_T = false (W k-contiguous)
//   input grad   C[m][n] = sum_k A[m][k] B[k][n]                         B_T = true  (W [k][n] rows)
//
// ViT-B/16 at batch 256 runs these on M = 50432 tokens (197 x 256) with N, K in {768, 2304,
// 3072}: 25 TFLOP of the step's 27. hipBLASLt's 256x256 kernels reach ~1.0 PF/s there, but
// every fusion around them costs a full pass over a [50432 x 3072] activation: the fc1 bias +
// GELU (a separate elementwise kernel, 115 us per block) and, in the backward, the GELU
// derivative + fc1's bias gradient (gelu_bwd_bias, 197 us per block). Here those live in
// the epilogue:
//   EPI 0: C = acc (+ bias)                                  -> bf16
//   EPI 1: h = acc + bias -> C (bf16), g = gelu(h) -> C2      (fc1 forward; tanh or erf GELU, gelu_set_form)
//   EPI 2: dh = bf16(acc) * gelu'(H[m][n]) -> C (bf16), and the column sums of dh over the
//          tile's rows -> colpart[2 * tile_m + wave_m][n] (fp32, no atomics; fc1's bias
//          gradient after gemm_splitk_reduce)                (fc2's input gradient)
//
// Main loop: wgrad256.hip's pipeline. One 512-thread workgroup per CU, 8 waves as 2 (M) x 4 (N)
// with 128 x 64 outputs each (8 x 4 tiles of v_mfma_f32_16x16x32_bf16); BK = 32 k per step,
// four LDS stages of [A 256 x 32 | B 256 x 32] (128 KiB), filled by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction) with three steps in flight: one counted
// vmcnt wait for the oldest step, a raw s_barrier, the DMA of step t + 3, 32 MFMAs per wave.
// k-contiguous operands use gemm_glds.hip's image ([rows][32], chunk slot q ^ f(row), f = [0,3,2,1][(row >> 2) & 3])
// read by ds_read_b128; the [k][n] B of the input gradient uses wgrad256.hip's ([32 k][256],
// transposed reads). Every per-step address is hoisted out of the loop (a lane's DMA pieces
// keep their row and chunk: pointers advance by 32 elements / 32 rows).
// B goes first in the MFMA (D = C^T): a lane's four accumulators are four consecutive columns
// of one row, so the epilogue stores 8 B per lane per tile straight from registers.
// Tile order: 1-D grid, XCD-aware — the workgroups of one XCD take a contiguous range of tiles
// in N-fastest order, so they share A row panels (and W) in that XCD's L2.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"
#include "gelu_tanh.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4v;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void gl_void;

constexpr int kThreads = 512;
constexpr int kTile = 256;
constexpr int kSmem = 128 * 1024;  // BK 32 x 4 stages or BK 64 x 2 stages of [A | B] images

__device__ __attribute__((aligned(16))) uint4 g_zero_g256[4];

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// [BK k][256] image swizzle of wgrad256.hip (the 8 k-rows of a half-wave's transposed read land
// on 8 distinct 32-B bank groups)
__device__ __forceinline__ int swz_tr(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }

// [256][BK] k-contiguous image: slot of chunk q in row r is q ^ swz_k(r); every 16-lane bank group
// of a ds_read_b128 fragment read covers the 64 banks once (scripts/lds_banks.py)
template <int BK>
__device__ __forceinline__ int swz_k(int row) {
  return BK == 32 ? ((-(row >> 2)) & 3) : ((row >> 1) & 7);
}

// Phi(x) = 0.5 (1 + erf(x / sqrt 2)) and exp(-x^2 / 2): Abramowitz-Stegun 7.1.26 erf
// (|error| <= 1.5e-7), the exponential shared with the derivative (gelu.hip)
__device__ __forceinline__ void gelu_parts(float x, float& cdf, float& e) {
  constexpr float kP0 = 0.3275911f, kA1 = 0.254829592f, kA2 = -0.284496736f, kA3 = 1.421413741f,
                  kA4 = -1.453152027f, kA5 = 1.061405429f;
  constexpr float kInvSqrt2 = 0.70710678118654752f;
  constexpr float kNegHalfLog2e = -0.72134752044448170f;
  e = __builtin_amdgcn_exp2f(kNegHalfLog2e * x * x);
  const float t = __builtin_amdgcn_rcpf(fmaf(kP0 * kInvSqrt2, fabsf(x), 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, kA5, kA4), kA3), kA2), kA1);
  const float tail = 0.5f * poly * e;
  cdf = x >= 0.f ? 1.f - tail : tail;
}

struct G256Args {
  const bf16* a;       // [M][lda]
  const bf16* b;       // B_T: [K][ldb] (N contiguous); else [N][ldb] (K contiguous)
  bf16* c;             // [M][ldc]
  bf16* c2;            // EPI 1: gelu output [M][ldc]
  const void* bias;    // [N] fp32 / bf16 (bias_f32), or nullptr
  const bf16* h;       // EPI 2: GELU input [M][ldc]
  float* colpart;      // EPI 2: [2 * tiles_m][N]
  int64_t lda, ldb, ldc;
  int64_t M, N, K;
  int tiles_m, tiles_n;
  int bias_f32;
  int gelu_tanh;  // EPI 1 / 2: tanh-form GELU (gelu_set_form), else exact erf
};

// VAR bit 0: the next step's LDS-DMA is issued spread through this step's MFMAs (one piece per
// four MFMAs) instead of in one burst after the barrier, so its issue cost (~60 cycles a piece)
// overlaps the partner wave's matrix work; bit 1: waves 4-7 at s_setprio 1 for the whole loop
// (the static form of cdna_hip_programming.md T5: the younger half stops losing arbitration);
// bit 2: s_setprio 1 around each MFMA cluster; bit 3 (kST == 2 only): the A operand of the next
// step goes global -> VGPRs (4 x 16 B per lane, issued after the barrier) and is written to LDS
// with ds_write_b128 after this step's MFMAs — half the bytes leave the LDS-DMA path, whose
// chip-wide rate (~6.4 TB/s measured for streams, MI355X_MICROARCH.md ldsdma-fill) caps the
// all-DMA loop near 0.8 PF/s at 128 FLOP per staged byte.
template <bool B_T, int EPI, int kBK, int kST, int VAR = 0>
__global__ __launch_bounds__(kThreads, 2) void gemm256_kernel(G256Args p) {
  constexpr int kImg = kTile * kBK * 2;   // bytes per operand image (16 / 32 KiB)
  constexpr int kStage = 2 * kImg;
  static_assert(kST * kStage <= kSmem, "LDS ring");
  constexpr int kP = kImg / 1024 / 8;     // DMA pieces per wave per operand (2 / 4)
  constexpr int kG = 2 * kP;              // DMA instructions per wave per step
  constexpr int kCPR = kBK / 8;           // 16-B chunks per k-contiguous row
  constexpr int kRPP = 64 / kCPR;         // k-contiguous rows per 1 KiB piece
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nt = p.tiles_m * p.tiles_n;
  int lid = blockIdx.x;
  {  // bijective XCD-aware order: XCD x gets a contiguous range of tile ids (N fastest)
    const int q = nt / 8, r = nt % 8, xcd = lid % 8, pos = lid / 8;
    lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int tm = lid / p.tiles_n, tn = lid - tm * p.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * kTile, n0 = static_cast<int64_t>(tn) * kTile;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;
  const int nk = static_cast<int>((p.K + kBK - 1) / kBK);

  // ---- DMA pieces of this lane (fixed row / chunk, pointers advance each step)
  // k-contiguous image: piece = kRPP rows x kCPR chunks; lane -> row piece*kRPP + lane/kCPR, slot lane%kCPR
  const bf16* pa[kP];
  const bf16* pb[kP];
  int kq[kP];  // k offset of this lane's chunk in the current step (k-contiguous operands)
  int kr[kP];  // B_T: k row of this lane's piece in the current step
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const int piece = wave * kP + j;
    const int row = piece * kRPP + lane / kCPR;
    const int q = (lane % kCPR) ^ swz_k<kBK>(row);
    kq[j] = q * 8;
    pa[j] = p.a + (m0 + row) * p.lda + q * 8;
    if (B_T) {
      const int krow = 2 * piece + (lane >> 5);
      const int chunk = (lane & 31) ^ swz_tr(krow);
      kr[j] = krow;
      pb[j] = p.b + static_cast<int64_t>(krow) * p.ldb + n0 + chunk * 8;
    } else {
      pb[j] = p.b + (n0 + row) * p.ldb + q * 8;
    }
  }
  const int64_t stepB = B_T ? static_cast<int64_t>(kBK) * p.ldb : kBK;
  // DMA instruction q (0 .. kG-1) of step t: even q = A piece q/2, odd q = B piece q/2
  auto issue_piece = [&](int t, int q) {
    char* st = smem + (t % kST) * kStage;
    const int j = q >> 1;
    // K tail (K % 32 != 0): chunks past K read zeros (both operands, so the products vanish)
    if ((q & 1) == 0) {
      const bool oka = t * kBK + kq[j] < p.K;
      const void* sa = oka ? static_cast<const void*>(pa[j]) : static_cast<const void*>(g_zero_g256);
      __builtin_amdgcn_global_load_lds((gl_void*)(sa), (lds_char*)(st + (wave * kP + j) * 1024), 16, 0, 0);
      pa[j] += kBK;
    } else {
      const bool okb = B_T ? t * kBK + kr[j] < p.K : t * kBK + kq[j] < p.K;
      const void* sb = okb ? static_cast<const void*>(pb[j]) : static_cast<const void*>(g_zero_g256);
      __builtin_amdgcn_global_load_lds((gl_void*)(sb), (lds_char*)(st + kImg + (wave * kP + j) * 1024), 16, 0, 0);
      pb[j] += stepB;
    }
  };
  auto issue = [&](int t) {
#pragma unroll
    for (int q = 0; q < kG; ++q) issue_piece(t, q);
  };
  // AREG: A of a step as 4 x 16 B per lane (chunk c = tid + 512 i: row c / kCPR, k chunk c % kCPR;
  // 8 lanes per 128-B row, coalesced), written to the same swizzled image the DMA would fill
  constexpr bool AREG = (VAR & 8) && kST == 2;
  constexpr int kAR = AREG ? kImg / 16 / kThreads : 1;
  uint4 areg[kAR];
  auto load_a_regs = [&](int t) {
#pragma unroll
    for (int i = 0; i < kAR; ++i) {
      const int c = threadIdx.x + kThreads * i, row = c / kCPR, kc = c % kCPR;
      const int64_t k = static_cast<int64_t>(t) * kBK + kc * 8;
      const bf16* src = k < p.K ? p.a + (m0 + row) * p.lda + k : reinterpret_cast<const bf16*>(g_zero_g256);
      areg[i] = *reinterpret_cast<const uint4*>(src);
    }
  };
  auto store_a_regs = [&](int t) {
    char* img = smem + (t % kST) * kStage;
#pragma unroll
    for (int i = 0; i < kAR; ++i) {
      const int c = threadIdx.x + kThreads * i, row = c / kCPR, kc = c % kCPR;
      *reinterpret_cast<uint4*>(img + row * (kBK * 2) + ((kc ^ swz_k<kBK>(row)) << 4)) = areg[i];
    }
  };

  // ---- fragment offsets (bytes within an image)
  // k-contiguous: lane reads row r0 + (lane & 15), k chunk (lane >> 4) + 4 kh at slot chunk ^ swz_k(row);
  // r0 is a multiple of 16, so the slot depends on the lane (and kh, by an XOR with 4) only
  const int rl = lane & 15;
  int slot[kBK / 32];
#pragma unroll
  for (int kh = 0; kh < kBK / 32; ++kh) slot[kh] = (((lane >> 4) + 4 * kh) ^ swz_k<kBK>(rl)) * 16;
  const int offA0 = (wm * 128 + rl) * (kBK * 2);
  const int offBk0 = (wn * 64 + rl) * (kBK * 2);
  // transposed [32 k][256] image (B_T): wgrad256h's per-lane constants
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int ktr = 8 * g4 + qq;
  const int swt = swz_tr(ktr);
  int offBt[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wn * 64 + j * 16 + 4 * pp;
    offBt[j] = ktr * (kTile * 2) + (((col >> 3) ^ swt) << 4) + (col & 7) * 2;
  }
  auto frag_k = [&](const char* __restrict__ img, int off) {
    return *reinterpret_cast<const bf16x8*>(img + off);
  };
  auto frag_t = [&](const char* __restrict__ img, int off) {
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off + 4 * kTile * 2));
    bf16x8 out;
    __builtin_memcpy(&out, &lo, 8);
    __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
    return out;
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < kST - 1; ++t)
    if (t < nk) issue(t);
  if ((VAR & 2) && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  // VAR & 1: piece g (0 .. kG-1) of the next step's DMA goes out before i-group g of the MFMAs
  constexpr int kGroups = (kBK / 32) * 8;  // (kh, i) fragment groups of 4 MFMAs per step
  for (int t = 0; t < nk; ++t) {
    const int ahead = nk - 1 - t;
    if (kST >= 4 && ahead >= 2) wait_vm<(kST >= 4 ? 2 : 0) * kG>();
    else if (kST >= 3 && ahead >= 1) wait_vm<(kST >= 3 ? 1 : 0) * kG>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const bool pre = t + kST - 1 < nk;
    if (AREG) {
      if (pre) {
#pragma unroll
        for (int q = 0; q < kP; ++q) issue_piece(t + 1, 2 * q + 1);  // B by LDS-DMA
        load_a_regs(t + 1);
      }
    } else if (!(VAR & 1) && pre) {
      issue(t + kST - 1);
    }
    const char* ta = smem + (t % kST) * kStage;
    const char* tb = ta + kImg;
#pragma unroll
    for (int kh = 0; kh < kBK / 32; ++kh) {
      bf16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = B_T ? frag_t(tb, offBt[j] + kh * 32 * kTile * 2) : frag_k(tb, offBk0 + j * 16 * (kBK * 2) + slot[kh]);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 fa = frag_k(ta, offA0 + i * 16 * (kBK * 2) + slot[kh]);
        if (VAR & 1) {
          const int g = kh * 8 + i;  // spread the kG pieces evenly over the kGroups groups
          if (pre && (g * kG) % kGroups < kG) issue_piece(t + kST - 1, (g * kG) / kGroups);
        }
        if (VAR & 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa, acc[i][j], 0, 0, 0);
        if (VAR & 4) __builtin_amdgcn_s_setprio(0);
      }
    }
    if (AREG && pre) {
      __builtin_amdgcn_s_waitcnt(0);  // the A registers (and B's DMA) of step t + 1 have landed
      store_a_regs(t + 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the writes are in LDS before the barrier
    }
  }

  // ---- epilogue: acc[i][j][r] = C[m0 + wm*128 + i*16 + (lane & 15)][n0 + wn*64 + j*16 + 4*(lane >> 4) + r]
  const int cq = 4 * (lane >> 4);
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + wn * 64 + j * 16 + cq;
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = 0.f;
    if (EPI != 2 && p.bias != nullptr) {
      if (p.bias_f32) {
        const float4 v = *reinterpret_cast<const float4*>(static_cast<const float*>(p.bias) + n);
        bias[j][0] = v.x, bias[j][1] = v.y, bias[j][2] = v.z, bias[j][3] = v.w;
      } else {
        bf16 v[4];
        __builtin_memcpy(v, static_cast<const bf16*>(p.bias) + n, 8);
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[j][r] = static_cast<float>(v[r]);
      }
    }
  }
  float cs[4][4];  // EPI 2: column sums over this lane's 8 rows
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t m = m0 + wm * 128 + i * 16 + rl;
    uint2 hv[4];
    if (EPI == 2) {  // all four loads of the row issued before any use
#pragma unroll
      for (int j = 0; j < 4; ++j) hv[j] = *reinterpret_cast<const uint2*>(p.h + m * p.ldc + n0 + wn * 64 + j * 16 + cq);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t off = m * p.ldc + n0 + wn * 64 + j * 16 + cq;
      bf16 o[4];
      if (EPI == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = static_cast<bf16>(acc[i][j][r] + bias[j][r]);
      } else if (EPI == 1) {
        bf16 g[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = static_cast<bf16>(acc[i][j][r] + bias[j][r]);
          const float x = static_cast<float>(o[r]);  // GELU of the bf16 pre-activation, as F.gelu(h)
          if (p.gelu_tanh) {
            g[r] = static_cast<bf16>(gelu_tanh(x));
          } else {
            float cdf, e;
            gelu_parts(x, cdf, e);
            g[r] = static_cast<bf16>(x * cdf);
          }
        }
        uint2 gv;
        __builtin_memcpy(&gv, g, 8);
        *reinterpret_cast<uint2*>(p.c2 + off) = gv;
      } else {
        bf16 hh[4];
        __builtin_memcpy(hh, &hv[j], 8);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dg = static_cast<float>(static_cast<bf16>(acc[i][j][r]));  // the bf16 dg, as autograd sees it
          const float x = static_cast<float>(hh[r]);
          float d;
          if (p.gelu_tanh) {
            d = gelu_tanh_grad(x);
          } else {
            float cdf, e;
            gelu_parts(x, cdf, e);
            d = fmaf(x * 0.39894228040143268f, e, cdf);
          }
          o[r] = static_cast<bf16>(dg * d);
          cs[j][r] += static_cast<float>(o[r]);  // the bias gradient of the rounded dh
        }
      }
      uint2 ov;
      __builtin_memcpy(&ov, o, 8);
      *reinterpret_cast<uint2*>(p.c + off) = ov;
    }
  }
  if (EPI == 2) {
    // sum the 16 lanes of equal (lane >> 4) (same columns, different rows): DPP within the row
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] = row_sum16(cs[j][r]);
    if (rl == 0) {
      float* dst = p.colpart + static_cast<int64_t>(2 * tm + wm) * p.N + n0 + wn * 64 + cq;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<float4*>(dst + j * 16) = float4{cs[j][0], cs[j][1], cs[j][2], cs[j][3]};
    }
  }
}

template <bool B_T, int EPI, int BK, int VAR>
void launch_v(const G256Args& p, hipStream_t stream) {
  constexpr int ST = BK == 32 ? 4 : 2;
  static bool attr = false;
  if (!attr) {
    FLUXMPI_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_kernel<B_T, EPI, BK, ST, VAR>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, kSmem));
    attr = true;
  }
  gemm256_kernel<B_T, EPI, BK, ST, VAR><<<p.tiles_m * p.tiles_n, kThreads, kSmem, stream>>>(p);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

int g_var = -1;
int var() {
  if (g_var < 0) {
    const char* e = std::getenv("FLUXMPI_GEMM256_VAR");
    g_var = e != nullptr ? (std::atoi(e) & 15) : 2;  // 2: measured best (+0.5-3 %, rd3f/rd3g)
  }
  return g_var;
}

template <bool B_T, int EPI, int BK>
void launch_bk(const G256Args& p, hipStream_t stream) {
  switch (var()) {
    case 1: launch_v<B_T, EPI, BK, 1>(p, stream); break;
    case 2: launch_v<B_T, EPI, BK, 2>(p, stream); break;
    case 3: launch_v<B_T, EPI, BK, 3>(p, stream); break;
    case 5: launch_v<B_T, EPI, BK, 5>(p, stream); break;
    case 8: launch_v<B_T, EPI, BK, 8>(p, stream); break;
    case 10: launch_v<B_T, EPI, BK, 10>(p, stream); break;
    default: launch_v<B_T, EPI, BK, 0>(p, stream); break;
  }
}

// pipeline: FLUXMPI_GEMM256_BK = 32 (four 32-deep stages, three in flight) or 64 (default: two
// 64-deep stages, 128-B rows per DMA lane group)
int g_bk = 0;
int bk() {
  if (g_bk == 0) {
    const char* e = std::getenv("FLUXMPI_GEMM256_BK");
    g_bk = (e != nullptr && std::atoi(e) == 32) ? 32 : 64;
  }
  return g_bk;
}

template <bool B_T, int EPI>
void launch(const G256Args& p, hipStream_t stream) {
  if (bk() == 32) launch_bk<B_T, EPI, 32>(p, stream);
  else launch_bk<B_T, EPI, 64>(p, stream);
}

}  // namespace

bool gemm256_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, bool b_t) {
  // the tile grid covers M and N exactly (no row / column guards in the loaders or the epilogue)
  return M > 0 && N > 0 && K > 0 && M % kTile == 0 && N % kTile == 0 && K % 8 == 0 && lda % 8 == 0 &&
         ldb % 8 == 0 && ldc % 8 == 0 && lda >= K && ldc >= N && (b_t ? ldb >= N : ldb >= K) &&
         M / kTile * (N / kTile) < (int64_t(1) << 31) && K < (int64_t(1) << 30);
}

int gemm256_colpart_rows(int64_t M) { return static_cast<int>(2 * (M / kTile)); }

void gemm256_set_bk(int bk_) { g_bk = bk_ == 32 ? 32 : 64; }
void gemm256_set_var(int v) { g_var = v & 15; }

void gemm256(const void* a, const void* b, void* c, void* c2, const void* bias, int bias_f32, const void* h,
             float* colpart, int64_t lda, int64_t ldb, int64_t ldc, int64_t M, int64_t N, int64_t K, bool b_t,
             int epi, hipStream_t stream) {
  if (!gemm256_supported(M, N, K, lda, ldb, ldc, b_t))
    throw std::runtime_error("gemm256: unsupported shape (M, N multiples of 256, K / leading dims multiples of 8; M=" +
                             std::to_string(M) + " N=" + std::to_string(N) + " K=" + std::to_string(K) + ")");
  if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15u) != 0)
    throw std::runtime_error("gemm256: operands must be 16-byte aligned");
  if (epi == 1 && c2 == nullptr) throw std::runtime_error("gemm256: GELU epilogue needs the second output");
  if (epi == 2 && (h == nullptr || colpart == nullptr || b_t == false))
    throw std::runtime_error("gemm256: GELU-backward epilogue needs h, colpart and the [k][n] B layout");
  if (bias != nullptr && (reinterpret_cast<uintptr_t>(bias) & (bias_f32 ? 15u : 7u)) != 0)
    throw std::runtime_error("gemm256: bias must be 16-byte (fp32) / 8-byte (bf16) aligned");
  G256Args p{static_cast<const bf16*>(a), static_cast<const bf16*>(b), static_cast<bf16*>(c), static_cast<bf16*>(c2),
             bias, static_cast<const bf16*>(h), colpart, lda, ldb, ldc, M, N, K,
             static_cast<int>(M / kTile), static_cast<int>(N / kTile), bias_f32, gelu_form()};
  if (b_t) {
    if (epi == 2) launch<true, 2>(p, stream);
    else if (epi == 1) launch<true, 1>(p, stream);
    else launch<true, 0>(p, stream);
  } else {
    if (epi == 1) launch<false, 1>(p, stream);
    else launch<false, 0>(p, stream);
  }
}

}  // namespace fluxmpi
