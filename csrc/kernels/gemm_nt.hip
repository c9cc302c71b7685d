// Token-major Linear GEMMs, "NT": C[m][n] = sum_k A[m][k] B[n][k], both operands k-contiguous —
// gfx950, 256 x 256 tiles, ping-pong 8-wave schedule.
//
//   forward      A = x [M][K], B = W [N][K]             (nn.Linear weight as stored)
//   input grad   A = dy [M][N_out], B = W^T [N_in][N_out] (transpose_bf16 once per call: the
//                weight is 0.6-4.7 MB, the activation 77-310 MB, so both operands stay
//                k-contiguous and every fragment is one ds_read_b128)
//
// Epilogues (the registers of the accumulator, no extra pass):
//   EPI 0: C = acc (+ bias)                                 -> bf16
//   EPI 1: h = bf16(acc + bias) -> C, g = gelu(h) -> C2     (fc1 forward, tanh or erf GELU)
//   EPI 2: dh = bf16(acc) * gelu'(H[m][n]) -> C, and the column sums of dh over the wave's 128
//          rows -> colpart[2 * tile_m + wave_m][n] (fp32; fc1's bias gradient after one reduce)
//
// Main loop (reference: /root/reference has no kernels — this is the compute under
// DistributedOptimizer's per-leaf work, src/optimizer.jl:20-23, for the ViT-B/16 config of
// BASELINE.json). One 512-thread workgroup per CU, 8 waves as 2 (M) x 4 (N), 128 x 64 outputs
// per wave (8 x 4 accumulators of v_mfma_f32_16x16x32_bf16). K advances 64 per tile; a tile is
// four PHASES, phase p computing the wave's rows 32p .. 32p + 31 (2 x 4 accumulators, K = 64:
// 16 MFMAs). Each phase is a LOAD segment (the phase's A fragments by ds_read_b128, in phase 0
// also the 8 B fragments kept in registers for the whole tile; the phase's LDS-DMA issues;
// one s_waitcnt vmcnt(7) lgkmcnt(0)) and a COMPUTE segment (16 MFMAs between s_setprio 1/0),
// separated by raw s_barriers. Waves 4-7 (wave_m = 1) run one barrier behind waves 0-3, so the
// two waves sharing a SIMD alternate: one computes while its partner loads (MI355X_MICROARCH.md
// "Two waves per SIMD"; cdna_hip_programming.md T3+T4).
//
// LDS: two buffers of [A 256 x 64 | B 256 x 64] bf16 images with 128-B rows (128 KiB), chunk
// slot q ^ ((row >> 1) & 7): every 16-lane group of a fragment read hits 16 distinct 16-B bank
// slots. Filled by global_load_lds_dwordx4, a wave-instruction = 8 full 128-B rows (full cache
// lines, not fragment-shaped pieces). Per tile each wave issues 8 DMA instructions:
//   phase p: the A rows of phase p of tile t+1 (1), and B of tile t+2 (phases 1..3: 2, 1, 1)
// B of a tile is read once (phase 0) and then lives in registers, so its slot is refilled a
// tile ahead; every group is read >= 4 phases after issue, and the wait that retires it is
// ALWAYS vmcnt(7) (every group is needed exactly 8 issues after its own). Issues past the last
// tile load a 16-B zero line into a dead slot, so the count never changes. A slot is restaged
// only after a barrier that follows its readers' lgkmcnt(0).
//
// Tile order: 1-D grid, XCD-aware (bijective): the workgroups of one XCD take a contiguous
// range of tile ids in N-fastest order, so they share A row panels in that XCD's L2.
#include <cstdint>
#include <stdexcept>
#include <type_traits>
#include <string>

#include "../api.h"
#include "common.h"
#include "gelu_tanh.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void gl_void;

constexpr int kT = 256;                // tile rows / columns
constexpr int kBK = 64;                // k per tile
constexpr int kThreads = 512;
constexpr int kRow = kBK * 2;          // 128-B image rows
constexpr int kImg = kT * kRow;        // 32 KiB per operand image
constexpr int kBuf = 2 * kImg;         // [A | B]
constexpr int kBiasOff = 2 * kBuf;     // 2 x 1 KiB bias slots (tile parity)
constexpr int kSmem = kBiasOff + 2048;  // 130 KiB

__device__ __attribute__((aligned(64))) uint4 g_zero_nt[4];

struct NTArgs {
  const bf16* a;       // [M][lda]
  const bf16* b;       // [N][ldb]
  bf16* c;             // [M][ldc]
  bf16* c2;            // EPI 1: GELU output [M][ldc]
  const void* bias;    // [N] fp32 / bf16 (bias_f32), or nullptr
  const bf16* h;       // EPI 2: GELU input [M][ldc]
  float* colpart;      // EPI 2: [2 * tiles_m][N]
  int64_t lda, ldb, ldc;
  int64_t N;
  int nk;              // K / 64
  int tiles_m, tiles_n;
  int bias_f32;
  int gelu_tanh;
};

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// Phi(x) and exp(-x^2/2) for the erf GELU (Abramowitz-Stegun 7.1.26, |error| <= 1.5e-7)
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

__device__ __forceinline__ void glds16(const void* src, char* dst) {
  __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(dst), 16, 0, 0);
}

__device__ __forceinline__ bf16x8 frag(const char* __restrict__ p) { return *reinterpret_cast<const bf16x8*>(p); }

// Tile list of workgroup g (grid G, persistent): rounds i = 0, 1, ... with g + i G < nt; round i
// covers tile ids [i G, i G + cnt), cnt = min(G, nt - i G), and g takes id i G + xcd_order(g, cnt)
// (bijective: the workgroups of one XCD take a contiguous range of ids, N fastest).
struct TileInfo {
  int64_t aoff, boff;  // m0 * lda, n0 * ldb
  int64_t m0, n0;
  int tm;
};

__device__ __forceinline__ TileInfo tile_info(const NTArgs& p, int g, int G, int i) {
  const int nt = p.tiles_m * p.tiles_n;
  const int base = i * G;
  const int cnt = min(G, nt - base);
  const int q = cnt / 8, r = cnt % 8, xcd = g % 8, pos = g / 8;
  const int lid = base + (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  TileInfo t;
  t.tm = lid / p.tiles_n;
  const int tn = lid - t.tm * p.tiles_n;
  t.m0 = static_cast<int64_t>(t.tm) * kT;
  t.n0 = static_cast<int64_t>(tn) * kT;
  t.aoff = t.m0 * p.lda;
  t.boff = t.n0 * p.ldb;
  return t;
}

// Persistent: the k-tiles of all of this workgroup's output tiles form ONE stream (stream slot
// s uses LDS buffer s & 1); the DMA of the next tile's first k-tiles is in flight while a tile's
// epilogue stores, so a tile costs its main loop plus its epilogue's issue time, no prologue.
// After an epilogue the first k-tile's waits count its vector-memory instructions (kEpiVm):
// they are younger than the DMA groups those waits retire.
// BIAS: 0 none, 1 fp32, 2 bf16 (EPI 0 / 1). The bias of a tile is loaded at the start of its
// last k-tile: loaded in the epilogue, its wait would also retire the next tile's DMA.
template <int EPI, int BIAS>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[kSmem];
  constexpr int kEpiVm = EPI == 0 ? 32 : 56;  // vector-memory instructions per wave in an epilogue (lower bound)
  const int G = gridDim.x, g = blockIdx.x;
  const int nt = p.tiles_m * p.tiles_n;
  const int nmine = (nt - g + G - 1) / G;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave-uniform
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = p.nk;  // >= 2

  // ---- LDS-DMA lanes: a wave-instruction fills 8 rows x 8 chunks; lane -> row lane >> 3, slot lane & 7
  const int lrow = lane >> 3, lslot = lane & 7;
  // A rows of phase p: waves 0-3 rows 32p + 8w, waves 4-7 rows 128 + 32p + 8(w-4) (+ lrow);
  // the swizzle of row + 32p equals that of row
  const int arow = (wave & 4) * 32 + (wave & 3) * 8 + lrow;
  const int laneA = arow * static_cast<int>(p.lda) + ((lslot ^ swz(arow)) << 3);  // < 2^31: lda < 2^23
  const int64_t aPhase = 32 * p.lda;
  const int dstA = (arow - lrow) * kRow;
  // B rows of piece j: 32w + 8j + lrow
  int laneB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 32 * wave + 8 * j + lrow;
    laneB[j] = row * static_cast<int>(p.ldb) + ((lslot ^ swz(row)) << 3);
  }
  const int dstB = kImg + 32 * wave * kRow;
  const void* zero = g_zero_nt;

  // DMA of stream slot s (LDS buffer s & 1): k-tile tk of the current tile (nxt = false) or of
  // the next one (nxt = true; a zero line into the dead slot when there is none)
  TileInfo cur = tile_info(p, g, G, 0);
  TileInfo nxt = tile_info(p, g, G, nmine > 1 ? 1 : 0);
  bool has_nxt = nmine > 1;
  auto issueA = [&](int s, bool n, int tk, int ph) {
    const int64_t base = n ? nxt.aoff : cur.aoff;
    const void* src = (!n || has_nxt) ? static_cast<const void*>(p.a + base + laneA + ph * aPhase + tk * kBK) : zero;
    glds16(src, smem + (s & 1) * kBuf + dstA + ph * 32 * kRow);
  };
  auto issueB = [&](int s, bool n, int tk, int j) {
    const int64_t base = n ? nxt.boff : cur.boff;
    const void* src = (!n || has_nxt) ? static_cast<const void*>(p.b + base + laneB[j] + tk * kBK) : zero;
    glds16(src, smem + (s & 1) * kBuf + dstB + j * 8 * kRow);
  };

  // ---- fragment reads: lane row (lane & 15), chunk (lane >> 4) + 4 kh at slot chunk ^ swz(row)
  const int fr = lane & 15;
  const int slot0 = ((lane >> 4) ^ (fr >> 1)) << 4;  // byte slot of chunk lane >> 4; kh = 1: slot0 ^ 64
  int offA[2], offB[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    offA[kh] = (wr * 128 + fr) * kRow + (slot0 ^ (kh << 6));  // + (32p + 16i) rows
    offB[kh] = kImg + (wc * 64 + fr) * kRow + (slot0 ^ (kh << 6));
  }

  f32x4 acc[4][2][4];
  bf16x8 fb[4][2];
  int s = 0;  // stream slot of the current k-tile

  // ---- prologue: B(0), A(0) phases 0..3, B(1)
#pragma unroll
  for (int j = 0; j < 4; ++j) issueB(0, false, 0, j);
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) issueA(0, false, 0, ph);
#pragma unroll
  for (int j = 0; j < 4; ++j) issueB(1, false, 1, j);
  asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // the stagger: waves 4-7 one barrier behind

  const int cq = 4 * (lane >> 4);
  int tile_i = 0;

  // one k-tile (4 phases) of the current tile; FIRST: the accumulators start from zero (and wave 0
  // stages the tile's bias); XV: vector-memory instructions issued since the DMA groups this
  // k-tile's first three waits retire
  auto ktile = [&](int t, auto first_c, auto last_c, auto xv_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr bool LAST = decltype(last_c)::value;
    constexpr int XV = decltype(xv_c)::value;
    if (FIRST && BIAS != 0 && wave == 0) {
      // the tile's 256 bias values (fp32 1 KiB / bf16 512 B) into its parity's LDS slot by one
      // LDS-DMA of wave 0; read in the epilogue, after many barriers and wave 0's vmcnt waits
      const char* src = BIAS == 1 ? reinterpret_cast<const char*>(static_cast<const float*>(p.bias) + cur.n0) + 16 * lane
                                  : (lane < 32 ? reinterpret_cast<const char*>(static_cast<const bf16*>(p.bias) + cur.n0) + 16 * lane
                                               : reinterpret_cast<const char*>(zero));
      glds16(src, smem + kBiasOff + (tile_i & 1) * 1024);
    }
    const char* buf = smem + (s & 1) * kBuf;
    // DMA targets: A of stream slot s + 1, B of slot s + 2
    const bool an = t + 1 >= nk;
    const int at = an ? t + 1 - nk : t + 1;
    const bool bn = t + 2 >= nk;
    const int bt = bn ? t + 2 - nk : t + 2;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      // ---------- load segment
      if (ph == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) fb[j][kh] = frag(buf + offB[kh] + j * 16 * kRow);
      }
      bf16x8 fa[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) fa[i][kh] = frag(buf + offA[kh] + (32 * ph + 16 * i) * kRow);
      issueA(s + 1, an, at, ph);
      if (ph == 1) {
        issueB(s + 2, bn, bt, 0);
        issueB(s + 2, bn, bt, 1);
      } else if (ph >= 2) {
        issueB(s + 2, bn, bt, ph);
      }
      if (ph < 3 && XV > 0) {
        if constexpr (7 + XV >= 63) asm volatile("s_waitcnt vmcnt(63) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(7 + XV) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---------- compute segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[ph][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fb[j][kh], fa[i][kh], (FIRST && kh == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[ph][i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    ++s;
  };

  using Z = std::integral_constant<int, 0>;
  for (int i = 0;;) {
    if (i == 0) ktile(0, std::true_type{}, std::false_type{}, Z{});
    else ktile(0, std::true_type{}, std::false_type{}, std::integral_constant<int, kEpiVm>{});
    for (int t = 1; t < nk; ++t) ktile(t, std::false_type{}, std::false_type{}, Z{});

    // ---- epilogue: acc[ph][i][j][r] = C[m0 + wr*128 + 32ph + 16i + (lane & 15)][n0 + wc*64 + 16j + 4(lane >> 4) + r]
    const int64_t ncol = cur.n0 + wc * 64 + cq;
    float bias[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const char* bl = smem + kBiasOff + (tile_i & 1) * 1024;
      const int col = wc * 64 + 16 * j + cq;
      if (BIAS == 1) {
        const float4 v = *reinterpret_cast<const float4*>(bl + 4 * col);
        bias[j][0] = v.x, bias[j][1] = v.y, bias[j][2] = v.z, bias[j][3] = v.w;
      } else if (BIAS == 2) {
        const uint2 v = *reinterpret_cast<const uint2*>(bl + 2 * col);
        bias[j][0] = __builtin_bit_cast(float, v.x << 16), bias[j][1] = __builtin_bit_cast(float, v.x & 0xFFFF0000u);
        bias[j][2] = __builtin_bit_cast(float, v.y << 16), bias[j][3] = __builtin_bit_cast(float, v.y & 0xFFFF0000u);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[j][r] = 0.f;
      }
    }
    float cs[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
    uint2 hv[4][2][4];  // EPI 2: every GELU input of the tile's lane issued before the first use (one round trip)
    if (EPI == 2) {
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            hv[ph][ii][j] = *reinterpret_cast<const uint2*>(
                p.h + (cur.m0 + wr * 128 + 32 * ph + 16 * ii + fr) * p.ldc + ncol + 16 * j);
    }
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int64_t m = cur.m0 + wr * 128 + 32 * ph + 16 * ii + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t off = m * p.ldc + ncol + 16 * j;
          bf16 o[4];
          if (EPI == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = static_cast<bf16>(acc[ph][ii][j][r] + bias[j][r]);
          } else if (EPI == 1) {
            bf16 gg[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              o[r] = static_cast<bf16>(acc[ph][ii][j][r] + bias[j][r]);
              const float x = static_cast<float>(o[r]);  // GELU of the bf16 pre-activation, as F.gelu(h)
              if (p.gelu_tanh) {
                gg[r] = static_cast<bf16>(gelu_tanh(x));
              } else {
                float cdf, e;
                gelu_parts(x, cdf, e);
                gg[r] = static_cast<bf16>(x * cdf);
              }
            }
            uint2 gv;
            __builtin_memcpy(&gv, gg, 8);
            *reinterpret_cast<uint2*>(p.c2 + off) = gv;
          } else {
            bf16 hh[4];
            __builtin_memcpy(hh, &hv[ph][ii][j], 8);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float dg = static_cast<float>(static_cast<bf16>(acc[ph][ii][j][r]));  // the bf16 dg autograd sees
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
    }
    if (EPI == 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[j][r] = row_sum16(cs[j][r]);
      if (fr == 0) {
        float* dst = p.colpart + static_cast<int64_t>(2 * cur.tm + wr) * p.N + ncol;
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<float4*>(dst + 16 * j) = float4{cs[j][0], cs[j][1], cs[j][2], cs[j][3]};
      }
    }
    if (++i >= nmine) break;
    tile_i = i;
    cur = nxt;
    has_nxt = i + 1 < nmine;
    nxt = tile_info(p, g, G, has_nxt ? i + 1 : i);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dead-slot DMAs
}

// dst[c][r] = src[r][c] (bf16), 64 x 64 tiles through LDS, 16-B global accesses both ways
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                             int64_t rows, int64_t cols, int64_t lds, int64_t ldd) {
  __shared__ bf16 tile[64][64 + 8];
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * 64, c0 = static_cast<int64_t>(blockIdx.x) * 64;
  const int tid = threadIdx.x;
  // load: 64 rows x 8 chunks of 8 elements; thread -> (row tid / 8 + 32 s, chunk tid % 8)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int r = tid / 8 + 32 * s, ch = tid % 8;
    uint4 v = uint4{0, 0, 0, 0};
    if (r0 + r < rows && c0 + ch * 8 < cols) v = *reinterpret_cast<const uint4*>(src + (r0 + r) * lds + c0 + ch * 8);
    bf16 e[8];
    __builtin_memcpy(e, &v, 16);
#pragma unroll
    for (int q = 0; q < 8; ++q) tile[r][ch * 8 + q] = e[q];
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = tid / 8 + 32 * s, ch = tid % 8;
    bf16 e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) e[q] = tile[ch * 8 + q][c];
    if (c0 + c < cols && r0 + ch * 8 < rows) {
      uint4 v;
      __builtin_memcpy(&v, e, 16);
      *reinterpret_cast<uint4*>(dst + (c0 + c) * ldd + r0 + ch * 8) = v;
    }
  }
}

int g_cus = 0;

template <int EPI, int BIAS>
void launch(const NTArgs& p, hipStream_t stream) {
  if (g_cus == 0) {
    int dev = 0;
    FLUXMPI_HIP_CHECK(hipGetDevice(&dev));
    FLUXMPI_HIP_CHECK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int nt = p.tiles_m * p.tiles_n;
  gemm_nt_kernel<EPI, BIAS><<<nt < g_cus ? nt : g_cus, kThreads, 0, stream>>>(p);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
  // the tile grid covers M, N and K exactly (no guards in the loaders or the epilogue)
  return M > 0 && N > 0 && K >= 2 * kBK && M % kT == 0 && N % kT == 0 && K % kBK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % 8 == 0 && lda >= K && ldb >= K && ldc >= N && lda < (int64_t(1) << 23) && ldb < (int64_t(1) << 23) && M / kT * (N / kT) < (int64_t(1) << 31) &&
         K / kBK < (int64_t(1) << 30);
}

int gemm_nt_colpart_rows(int64_t M) { return static_cast<int>(2 * (M / kT)); }

void gemm_nt(const void* a, const void* b, void* c, void* c2, const void* bias, int bias_f32, const void* h,
             float* colpart, int64_t lda, int64_t ldb, int64_t ldc, int64_t M, int64_t N, int64_t K, int epi,
             hipStream_t stream) {
  if (!gemm_nt_supported(M, N, K, lda, ldb, ldc))
    throw std::runtime_error("gemm_nt: unsupported shape (M, N multiples of 256, K of 64, leading dims of 8; M=" +
                             std::to_string(M) + " N=" + std::to_string(N) + " K=" + std::to_string(K) + ")");
  if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15u) != 0)
    throw std::runtime_error("gemm_nt: operands must be 16-byte aligned");
  if (epi == 1 && c2 == nullptr) throw std::runtime_error("gemm_nt: the GELU epilogue needs the second output");
  if (epi == 2 && (h == nullptr || colpart == nullptr))
    throw std::runtime_error("gemm_nt: the GELU-backward epilogue needs h and colpart");
  if (bias != nullptr && (reinterpret_cast<uintptr_t>(bias) & (bias_f32 ? 15u : 7u)) != 0)
    throw std::runtime_error("gemm_nt: bias must be 16-byte (fp32) / 8-byte (bf16) aligned");
  NTArgs p{static_cast<const bf16*>(a), static_cast<const bf16*>(b), static_cast<bf16*>(c), static_cast<bf16*>(c2),
           bias, static_cast<const bf16*>(h), colpart, lda, ldb, ldc, N, static_cast<int>(K / kBK),
           static_cast<int>(M / kT), static_cast<int>(N / kT), bias_f32, gelu_form()};
  const int bk = bias == nullptr ? 0 : bias_f32 ? 1 : 2;
  if (epi == 2) {
    launch<2, 0>(p, stream);
  } else if (epi == 1) {
    if (bk == 1) launch<1, 1>(p, stream);
    else if (bk == 2) launch<1, 2>(p, stream);
    else launch<1, 0>(p, stream);
  } else {
    if (bk == 1) launch<0, 1>(p, stream);
    else if (bk == 2) launch<0, 2>(p, stream);
    else launch<0, 0>(p, stream);
  }
}

void transpose_bf16(const void* src, void* dst, int64_t rows, int64_t cols, int64_t lds, int64_t ldd,
                    hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return;
  if (cols % 8 != 0 || rows % 8 != 0 || lds % 8 != 0 || ldd % 8 != 0 ||
      ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) != 0)
    throw std::runtime_error("transpose_bf16: rows, cols and leading dims must be multiples of 8, pointers 16-B aligned");
  dim3 grid(static_cast<unsigned>((cols + 63) / 64), static_cast<unsigned>((rows + 63) / 64));
  transpose_bf16_kernel<<<grid, 256, 0, stream>>>(static_cast<const bf16*>(src), static_cast<bf16*>(dst), rows, cols,
                                                    lds, ldd);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
