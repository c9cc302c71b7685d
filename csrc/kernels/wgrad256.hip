// Weight gradient C[m][n] = sum_k A[k][m] * B[k][n] on 256 x 256 tiles — gfx950.
//
// The long-K / small-output GEMM of every token-major Linear's backward (ViT-B/16: K = 50432
// tokens, M x N = 768..3072 squared) and of the large 1x1 convolutions. gemm_glds.hip's
// 128 x 128 / 4-wave weight-gradient kernel moves 16 KB per 128x128x32 step through L2 ->
// LDS (64 FLOP per staged byte) and tops out near 700 TF/s on these shapes
// (scripts/bench_vit_gemm.py); a 256 x 256 tile halves the staged bytes per FLOP.
//
// Structure (one workgroup per CU: 8 waves, 128 KiB of LDS):
//   * BK = 32 k-rows per step, four LDS stages (FLUXMPI_WGRAD256_VARIANT=1: BK = 64, two
//     stages); a stage holds both operand tiles as [BK k][256 cols] bf16 images (512-B rows)
//     filled by LDS-DMA (global_load_lds_dwordx4: each wave-instruction writes 1 KiB = two
//     k-rows);
//   * one barrier per step: a counted vmcnt wait for the OLDEST outstanding step only (the
//     younger ones stay in flight), raw s_barrier, issue the DMA of step t + 3 into the stage
//     step t - 1 used, then 32 MFMAs per wave — three steps of DMA run under the MFMAs;
//   * fragments by ds_read_b64_tr_b16 (both operands are k-major in memory, the MFMA wants k
//     along the lane's 8 elements). Chunk-slot swizzle slot = chunk ^ ((k & 3) << 1 |
//     ((k >> 3) & 1) << 3), applied on the per-lane GLOBAL source address (the DMA image is
//     lane-linear): the 8 k-rows a half-wave's transposed read touches land on 8 distinct
//     32-B bank groups;
//   * waves 2 (M) x 4 (N), 128 x 64 outputs each: 8 x 4 accumulator tiles of
//     v_mfma_f32_16x16x32_bf16;
//   * split-K over a 1-D grid, XCD-aware: the workgroups of one split (which read the same
//     A / B rows) run on one XCD and share its L2; fp32 partials [split][M][N], summed (and
//     cast) by gemm_splitk_reduce.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;
constexpr int kTile = 256;  // BM = BN

__device__ __attribute__((aligned(16))) uint4 g_zero256[4];

__device__ __forceinline__ int swz(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

struct W256Args {
  const bf16* a;  // [K][lda], M contiguous
  const bf16* b;  // [K][ldb], N contiguous
  float* c;       // [splits][M][N]
  int64_t lda, ldb;
  int64_t M, N, K;
  int64_t k_per_split;
  int tiles_m, tiles_n;
};

// LDS-DMA of this wave's pieces of one [BK k][256] operand image for k-rows [k0, k0 + BK)
template <int BK>
__device__ __forceinline__ void issue_img(char* img, const bf16* __restrict__ g, int64_t ld, int64_t col0, int64_t k0,
                                          int64_t kend) {
  constexpr int kPieces = BK * kTile * 2 / 1024 / 8;  // 1-KiB pieces per wave (two k-rows each)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < kPieces; ++j) {
    const int piece = wave * kPieces + j;
    const int row = 2 * piece + (lane >> 5);
    const int chunk = (lane & 31) ^ swz(row);
    const int64_t k = k0 + row;
    const void* src = k < kend ? static_cast<const void*>(g + k * ld + col0 + chunk * 8)
                               : static_cast<const void*>(g_zero256);
    typedef __attribute__((address_space(3))) char lds_char;
    typedef __attribute__((address_space(1))) void gl_void;
    __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(img + piece * 1024), 16, 0, 0);
  }
}

// lane l: tile[k = 32 kh + 8 (l >> 4) + j][r0 + (l & 15)], j = 0..7 (two transposed reads)
__device__ __forceinline__ bf16x8 frag(const bf16* __restrict__ img, int r0, int kh) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, li = l & 15, q = li >> 2, p = li & 3;
  const int col = r0 + 4 * p;
  const int k0 = 32 * kh + 8 * g + q, k1 = k0 + 4;
  const bf16* a0 = img + k0 * kTile + (((col >> 3) ^ swz(k0)) << 3) + (col & 7);
  const bf16* a1 = img + k1 * kTile + (((col >> 3) ^ swz(k1)) << 3) + (col & 7);
  typedef short short4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4v lds_short4v;
  short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(a0));
  short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(a1));
  bf16x8 out;
  __builtin_memcpy(&out, &lo, 8);
  __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
  return out;
}

// BK k-rows per step, ST LDS stages (ST - 1 steps of DMA in flight). Stage images are
// [BK][256] bf16 for A and for B; ST * BK * 2 KiB of LDS in all.
template <int BK, int ST, bool PRIO = false>
__global__ __launch_bounds__(kThreads, 1) void wgrad256_kernel(W256Args p) {
  constexpr int kImgBytes = BK * kTile * 2;
  constexpr int kStageBytes = 2 * kImgBytes;
  constexpr int kG = 2 * (kImgBytes / 1024 / 8);  // DMA instructions per wave per step (both operands)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nt = p.tiles_m * p.tiles_n;
  const int total = static_cast<int>(gridDim.x);
  int lid = blockIdx.x;
  if (total >= 8) {  // bijective XCD-aware order: an XCD gets a contiguous (split-major) id range
    const int q = total / 8, r = total % 8, xcd = lid % 8, pos = lid / 8;
    lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int split = lid / nt, bid = lid - split * nt;
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * kTile, n0 = static_cast<int64_t>(tn) * kTile;
  const int64_t kbeg = static_cast<int64_t>(split) * p.k_per_split;
  const int64_t kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  const int nk = kend > kbeg ? static_cast<int>((kend - kbeg + BK - 1) / BK) : 0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* st = smem + (t % ST) * kStageBytes;
    const int64_t k0 = kbeg + static_cast<int64_t>(t) * BK;
    issue_img<BK>(st, p.a, p.lda, m0, k0, kend);
    issue_img<BK>(st + kImgBytes, p.b, p.ldb, n0, k0, kend);
  };
#pragma unroll
  for (int t = 0; t < ST - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    // this wave's DMA of step t has landed once at most min(ST - 2, steps issued after t) steps
    // are outstanding; then the barrier publishes every wave's pieces (raw s_barrier: a
    // __syncthreads() fence would drain the younger DMAs too)
    const int ahead = nk - 1 - t;
    if (ST >= 4 && ahead >= 2) wait_vm<(ST >= 4 ? 2 : 0) * kG>();
    else if (ST >= 3 && ahead >= 1) wait_vm<(ST >= 3 ? 1 : 0) * kG>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    // stage (t + ST - 1) % ST was last read in step t - 1, which every wave finished
    if (t + ST - 1 < nk) issue(t + ST - 1);
    const bf16* ta = reinterpret_cast<const bf16*>(smem + (t % ST) * kStageBytes);
    const bf16* tb = reinterpret_cast<const bf16*>(smem + (t % ST) * kStageBytes + kImgBytes);
    if (PRIO) __builtin_amdgcn_s_setprio(1);  // MFMA-issuing waves first (T5)
#pragma unroll
    for (int kh = 0; kh < BK / 32; ++kh) {
      bf16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag(tb, wn * 64 + j * 16, kh);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 fa = frag(ta, wm * 128 + i * 16, kh);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
      }
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  // fp32 partial: acc[i][j][r] is (row wm*128 + i*16 + 4*(lane>>4) + r, col wn*64 + j*16 + lane&15)
  float* c = p.c + static_cast<int64_t>(split) * p.M * p.N;
  const int col_in = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + j * 16 + col_in;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 128 + i * 16 + rq + r;
        c[m * p.N + n] = acc[i][j][r];
      }
    }
}

// Variant 3: the same pipeline with every per-step address computation hoisted out of the
// k-loop (PMC: 2.2 VALU instructions per MFMA in variant 0, mostly 64-bit DMA source
// addresses and the swizzled fragment offsets recomputed each step). A lane's DMA pieces
// keep their (row, chunk) for the whole loop, so their source pointers just advance by BK
// rows; a fragment's swizzle term depends only on the lane (k rows 32 kh + 8 g + q and
// + 4 share it), so its LDS offset is one per-lane constant per fragment plus immediates.
template <int BK, int ST>
__global__ __launch_bounds__(kThreads, 1) void wgrad256h_kernel(W256Args p) {
  constexpr int kImgBytes = BK * kTile * 2;
  constexpr int kStageBytes = 2 * kImgBytes;
  constexpr int kP = kImgBytes / 1024 / 8;  // DMA pieces per wave per operand
  constexpr int kG = 2 * kP;                // DMA instructions per wave per step
  constexpr int kRow = kTile * 2;           // bytes per k-row of an image
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nt = p.tiles_m * p.tiles_n;
  const int total = static_cast<int>(gridDim.x);
  int lid = blockIdx.x;
  if (total >= 8) {
    const int q = total / 8, r = total % 8, xcd = lid % 8, pos = lid / 8;
    lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int split = lid / nt, bid = lid - split * nt;
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * kTile, n0 = static_cast<int64_t>(tn) * kTile;
  const int64_t kbeg = static_cast<int64_t>(split) * p.k_per_split;
  const int64_t kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  const int nk = kend > kbeg ? static_cast<int>((kend - kbeg + BK - 1) / BK) : 0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;

  // DMA: this lane's pieces (row 2 * piece + lane / 32, chunk slot lane % 32)
  const bf16* pa[kP];
  const bf16* pb[kP];
  int krow[kP];  // k row relative to kbeg
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const int row = 2 * (wave * kP + j) + (lane >> 5);
    const int chunk = (lane & 31) ^ swz(row);
    krow[j] = row;
    pa[j] = p.a + (kbeg + row) * p.lda + m0 + chunk * 8;
    pb[j] = p.b + (kbeg + row) * p.ldb + n0 + chunk * 8;
  }
  const int64_t stepA = static_cast<int64_t>(BK) * p.lda, stepB = static_cast<int64_t>(BK) * p.ldb;
  const int klim = static_cast<int>(kend - kbeg);
  auto issue = [&](int t) {
    char* st = smem + (t % ST) * kStageBytes;
    typedef __attribute__((address_space(3))) char lds_char;
    typedef __attribute__((address_space(1))) void gl_void;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const bool ok = krow[j] < klim;
      const void* sa = ok ? static_cast<const void*>(pa[j]) : static_cast<const void*>(g_zero256);
      const void* sb = ok ? static_cast<const void*>(pb[j]) : static_cast<const void*>(g_zero256);
      __builtin_amdgcn_global_load_lds((gl_void*)(sa), (lds_char*)(st + (wave * kP + j) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gl_void*)(sb), (lds_char*)(st + kImgBytes + (wave * kP + j) * 1024), 16,
                                       0, 0);
      pa[j] += stepA;
      pb[j] += stepB;
      krow[j] += BK;
    }
  };

  // fragment offsets within an image (kh = 0, first transposed read)
  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int k0 = 8 * g + qq;
  const int sw = swz(k0);
  int offA[8], offB[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int col = wm * 128 + i * 16 + 4 * pp;
    offA[i] = k0 * kRow + ((((col >> 3) ^ sw)) << 4) + (col & 7) * 2;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wn * 64 + j * 16 + 4 * pp;
    offB[j] = k0 * kRow + ((((col >> 3) ^ sw)) << 4) + (col & 7) * 2;
  }
  typedef short short4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4v lds_short4v;
  // __restrict__ matters: it gives the reads alias scopes, without which the waitcnt pass
  // assumes they may read the DMA just issued and drains vmcnt(0) before them
  auto frag_at = [&](const char* __restrict__ img, int off) {
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off + 4 * kRow));
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
  for (int t = 0; t < ST - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    const int ahead = nk - 1 - t;
    if (ST >= 4 && ahead >= 2) wait_vm<(ST >= 4 ? 2 : 0) * kG>();
    else if (ST >= 3 && ahead >= 1) wait_vm<(ST >= 3 ? 1 : 0) * kG>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (t + ST - 1 < nk) issue(t + ST - 1);
    const char* ta = smem + (t % ST) * kStageBytes;
    const char* tb = ta + kImgBytes;
#pragma unroll
    for (int kh = 0; kh < BK / 32; ++kh) {
      bf16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_at(tb, offB[j] + kh * 32 * kRow);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 fa = frag_at(ta, offA[i] + kh * 32 * kRow);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  float* c = p.c + static_cast<int64_t>(split) * p.M * p.N;
  const int col_in = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + j * 16 + col_in;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 128 + i * 16 + rq + r;
        c[m * p.N + n] = acc[i][j][r];
      }
    }
}

// Variant 4: wgrad256h's operands, addressing and 4-stage ring in gemm_nt.hip's ping-pong
// schedule. A 32-deep step is two PHASES (the wave's rows 0..63, then 64..127 of its 128: 16
// MFMAs each); a phase is a LOAD segment (phase 0: the step's 4 B fragments + the first 4 A
// fragments, phase 1: the other 4 A fragments, all by ds_read_b64_tr_b16; phase 0 issues the
// LDS-DMA of A three steps ahead, phase 1 that of B; lgkmcnt(0), and in phase 1 the counted
// vmcnt(8) that retires step t + 1) then a COMPUTE segment (16 MFMAs between s_setprio 1 / 0),
// separated by raw s_barriers. Waves 4-7 run one barrier behind waves 0-3, so the two waves of a
// SIMD alternate compute and load (MI355X_MICROARCH.md "Two waves per SIMD"). The stage a DMA
// refills was last read one step earlier, before a barrier that follows its readers' lgkmcnt(0).
__global__ __launch_bounds__(kThreads, 2) void wgrad256pp_kernel(W256Args p) {
  constexpr int BK = 32, ST = 4;
  constexpr int kImgBytes = BK * kTile * 2;  // 16 KiB
  constexpr int kStageBytes = 2 * kImgBytes;
  constexpr int kP = kImgBytes / 1024 / 8;    // 2 DMA pieces per wave per operand per step
  constexpr int kRow = kTile * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nt = p.tiles_m * p.tiles_n;
  const int total = static_cast<int>(gridDim.x);
  int lid = blockIdx.x;
  if (total >= 8) {
    const int q = total / 8, r = total % 8, xcd = lid % 8, pos = lid / 8;
    lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int split = lid / nt, bid = lid - split * nt;
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * kTile, n0 = static_cast<int64_t>(tn) * kTile;
  const int64_t kbeg = static_cast<int64_t>(split) * p.k_per_split;
  const int64_t kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  const int nk = kend > kbeg ? static_cast<int>((kend - kbeg + BK - 1) / BK) : 0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;

  const bf16* pa[kP];
  const bf16* pb[kP];
  int krow[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const int row = 2 * (wave * kP + j) + (lane >> 5);
    const int chunk = (lane & 31) ^ swz(row);
    krow[j] = row;
    pa[j] = p.a + (kbeg + row) * p.lda + m0 + chunk * 8;
    pb[j] = p.b + (kbeg + row) * p.ldb + n0 + chunk * 8;
  }
  const int64_t stepA = static_cast<int64_t>(BK) * p.lda, stepB = static_cast<int64_t>(BK) * p.ldb;
  const int klim = static_cast<int>(kend - kbeg);
  typedef __attribute__((address_space(3))) char lds_char;
  typedef __attribute__((address_space(1))) void gl_void;
  // the DMA of one operand of step t (rows past the split's end read a zero line: same count)
  auto issue = [&](int t, bool b_op) {
    char* img = smem + (t % ST) * kStageBytes + (b_op ? kImgBytes : 0);
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const int kr = krow[j] + t * BK;
      const void* src = kr < klim ? static_cast<const void*>((b_op ? pb[j] + t * stepB : pa[j] + t * stepA))
                                  : static_cast<const void*>(g_zero256);
      __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(img + (wave * kP + j) * 1024), 16, 0, 0);
    }
  };

  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int k0 = 8 * g + qq;
  const int sw = swz(k0);
  int offA[8], offB[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int col = wm * 128 + i * 16 + 4 * pp;
    offA[i] = k0 * kRow + ((((col >> 3) ^ sw)) << 4) + (col & 7) * 2;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wn * 64 + j * 16 + 4 * pp;
    offB[j] = k0 * kRow + ((((col >> 3) ^ sw)) << 4) + (col & 7) * 2;
  }
  typedef short short4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4v lds_short4v;
  auto frag_at = [&](const char* __restrict__ img, int off) {
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off + 4 * kRow));
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
  // prologue: steps 0, 1, 2 (A then B each); step 0 retired with the 8 younger in flight
#pragma unroll
  for (int t = 0; t < ST - 1; ++t) {
    issue(t, false);
    issue(t, true);
  }
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();  // the stagger

  bf16x8 fb[4];
  for (int t = 0; t < nk; ++t) {
    const char* ta = smem + (t % ST) * kStageBytes;
    const char* tb = ta + kImgBytes;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      // ---------- load segment
      if (ph == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = frag_at(tb, offB[j]);
      }
      bf16x8 fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_at(ta, offA[4 * ph + i]);
      issue(t + ST - 1, ph == 1);
      if (ph == 1) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---------- compute segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 * ph + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[4 * ph + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* c = p.c + static_cast<int64_t>(split) * p.M * p.N;
  const int col_in = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + j * 16 + col_in;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 128 + i * 16 + rq + r;
        c[m * p.N + n] = acc[i][j][r];
      }
    }
}

// pipeline variant: 0 = BK 32 x 4 stages, 1 = BK 64 x 2 stages, 2 = variant 0 with s_setprio(1)
// around each step's MFMAs, 3 = variant 0 with the addressing hoisted out of the loop,
// 4 (default) = the ping-pong schedule (wgrad256pp_kernel): +1-3 % on three of the four ViT-B/16
// shapes, equal on the fourth (profiles/rd4c_bench_wgrad_v3_v4.jsonl)
int g_variant = -1;
int variant() {
  if (g_variant < 0) {
    const char* e = std::getenv("FLUXMPI_WGRAD256_VARIANT");
    g_variant = e != nullptr ? std::atoi(e) : 4;
    if (g_variant < 0 || g_variant > 4) g_variant = 4;
  }
  return g_variant;
}
int bk_of(int v) { return v == 1 ? 64 : 32; }

}  // namespace

void wgrad256_set_variant(int v) { g_variant = v >= 0 && v <= 4 ? v : 4; }

bool wgrad256_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  return M % kTile == 0 && N % kTile == 0 && M > 0 && N > 0 && K > 0 && K < (int64_t(1) << 31) && lda % 8 == 0 &&
         ldb % 8 == 0 && lda >= M && ldb >= N;
}

void gemm_wgrad256(const void* a, const void* b, float* ws, int64_t lda, int64_t ldb, int64_t M, int64_t N, int64_t K,
                   int splits, hipStream_t stream) {
  if (!wgrad256_supported(M, N, K, lda, ldb))
    throw std::runtime_error("gemm_wgrad256: need M, N multiples of 256, lda/ldb multiples of 8 (M=" +
                             std::to_string(M) + ", N=" + std::to_string(N) + ")");
  if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15u) != 0)
    throw std::runtime_error("gemm_wgrad256: operands must be 16-byte aligned");
  if (splits < 1) splits = 1;
  const int v = variant();
  const int bk = bk_of(v);
  const int64_t nk = (K + bk - 1) / bk;
  const int64_t kps = (nk + splits - 1) / splits * bk;
  const int s = static_cast<int>((K + kps - 1) / kps);  // splits actually used (every one non-empty)
  W256Args p{static_cast<const bf16*>(a), static_cast<const bf16*>(b), ws, lda, ldb, M, N, K, kps,
             static_cast<int>(M / kTile), static_cast<int>(N / kTile)};
  const int64_t grid = static_cast<int64_t>(s) * p.tiles_m * p.tiles_n;
  if (grid > 0x7fffffff) throw std::runtime_error("gemm_wgrad256: grid too large");
  constexpr int kSmem = 128 * 1024;  // both variants: 4 x 32 KiB / 2 x 64 KiB
  static bool attr[5] = {false, false, false, false, false};
  const void* fn = v == 1   ? reinterpret_cast<const void*>(&wgrad256_kernel<64, 2>)
                   : v == 2 ? reinterpret_cast<const void*>(&wgrad256_kernel<32, 4, true>)
                   : v == 3 ? reinterpret_cast<const void*>(&wgrad256h_kernel<32, 4>)
                   : v == 4 ? reinterpret_cast<const void*>(&wgrad256pp_kernel)
                            : reinterpret_cast<const void*>(&wgrad256_kernel<32, 4>);
  if (!attr[v]) {
    FLUXMPI_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kSmem));
    attr[v] = true;
  }
  if (v == 1) wgrad256_kernel<64, 2><<<static_cast<unsigned>(grid), kThreads, kSmem, stream>>>(p);
  else if (v == 2) wgrad256_kernel<32, 4, true><<<static_cast<unsigned>(grid), kThreads, kSmem, stream>>>(p);
  else if (v == 3) wgrad256h_kernel<32, 4><<<static_cast<unsigned>(grid), kThreads, kSmem, stream>>>(p);
  else if (v == 4) wgrad256pp_kernel<<<static_cast<unsigned>(grid), kThreads, kSmem, stream>>>(p);
  else wgrad256_kernel<32, 4><<<static_cast<unsigned>(grid), kThreads, kSmem, stream>>>(p);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

int wgrad256_actual_splits(int64_t K, int splits) {
  if (splits < 1) splits = 1;
  const int bk = bk_of(variant());
  const int64_t nk = (K + bk - 1) / bk;
  const int64_t kps = (nk + splits - 1) / splits * bk;
  return static_cast<int>((K + kps - 1) / kps);
}

}  // namespace fluxmpi
