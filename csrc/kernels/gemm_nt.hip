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
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
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
  float* ws;           // stream-K partials: [grid][32][512] float4 (gemm_nt_workspace_bytes)
  int* flags;          // [grid][8] per-wave publish flags, zero between launches
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

// Stream-K over the whole problem: the U = tiles x nk (tile, k-tile) units are dealt to the G
// persistent workgroups as equal contiguous ranges (workgroups of one XCD take neighbouring
// ranges: the tiles of one XCD share their A row panels in its L2). Tiles are N-fastest, a
// tile's k-tiles consecutive. A workgroup's range is ONE stream of k-tiles (stream slot s uses
// LDS buffer s & 1): the DMA of a tile's first k-tiles is in flight while the previous tile's
// epilogue stores, and because the ranges start at different points of their tiles the
// workgroups' epilogues (bandwidth bursts) do not all land at once, and no round is partial.
// A range that starts inside a tile writes that segment's fp32 partial to its slot of the
// workspace (each wave its own 32 x 16 B per lane, then an agent-scope release and a per-wave
// flag); the workgroup whose range covers the tile's FIRST k-tile finishes it: at the end of
// its range it polls the flags of the following workgroups whose ranges start inside the tile
// (relaxed agent-scope loads), acquires, adds their partials and runs the epilogue (flags reset
// to 0 for the next launch). Contributors publish at the START of their ranges and never wait,
// so the wait is deadlock-free whatever the residency (MI355X_MICROARCH.md "Workgroup dispatch
// ... inter-workgroup visibility", cdna_hip_programming.md Guideline 16).
// After an epilogue the first k-tile's waits count its vector-memory instructions (kEpiVm):
// they are younger than the DMA groups those waits retire.
// BIAS: 0 none, 1 fp32, 2 bf16 (EPI 0 / 1), staged into LDS by one LDS-DMA of wave 0 at the
// first k-tile of the finishing segment.
struct TileInfo {
  int64_t aoff, boff;  // m0 * lda, n0 * ldb
  int64_t m0, n0;
  int tm;
};

__device__ __forceinline__ int64_t uni64(int64_t v) {  // provably wave-uniform (SGPRs)
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32));
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}

__device__ __forceinline__ TileInfo tile_of(const NTArgs& p, int T) {
  TileInfo t;
  T = __builtin_amdgcn_readfirstlane(T);
  t.tm = __builtin_amdgcn_readfirstlane(T / p.tiles_n);
  const int tn = T - t.tm * p.tiles_n;
  t.m0 = uni64(static_cast<int64_t>(t.tm) * kT);
  t.n0 = uni64(static_cast<int64_t>(tn) * kT);
  t.aoff = uni64(t.m0 * p.lda);
  t.boff = uni64(t.n0 * p.ldb);
  return t;
}

// first unit of workgroup (range) r
__device__ __forceinline__ int range_start(int U, int G, int r) {
  return static_cast<int>(static_cast<int64_t>(U) * r / G);
}

template <int EPI, int BIAS>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[kSmem];
  constexpr int kEpiVm = EPI == 0 ? 32 : 56;  // vector-memory instructions per wave in an epilogue (lower bound)
  const int G = gridDim.x;
  int gi = blockIdx.x;
  {  // bijective XCD-aware range order: the workgroups of one XCD take neighbouring ranges
    const int q = G / 8, r = G % 8, xcd = gi % 8, pos = gi / 8;
    gi = __builtin_amdgcn_readfirstlane((xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos);
  }
  const int nk = p.nk;  // >= 2
  const int U = p.tiles_m * p.tiles_n * nk;  // < 2^31 (gemm_nt_supported)
  const int u0 = __builtin_amdgcn_readfirstlane(range_start(U, G, gi));
  const int u1 = __builtin_amdgcn_readfirstlane(range_start(U, G, gi + 1));
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave-uniform
  const int wr = wave >> 2, wc = wave & 3;

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

  // DMA into stream slot s (LDS buffer s & 1) of k-tile tk of tile `ti`. Source = a wave-uniform
  // base (SGPRs: readfirstlane) + the lane's 32-bit byte offset, so no 64-bit per-lane address is
  // kept live across the loop. Past the range's end (`ok` false) the slot is dead and the DMA just
  // re-reads valid bytes (the caller passes the current unit), keeping the vmcnt count fixed.
  const uint32_t laneAb = static_cast<uint32_t>(laneA) * 2u;
  uint32_t laneBb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) laneBb[j] = static_cast<uint32_t>(laneB[j]) * 2u;
  auto sbase = [](const bf16* base, int64_t elems) {
    const uint64_t a = reinterpret_cast<uint64_t>(base + elems);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
    return reinterpret_cast<const char*>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  auto issueA = [&](int s, const TileInfo& ti, int tk, int ph) {
    glds16(sbase(p.a, ti.aoff + ph * aPhase + tk * kBK) + laneAb, smem + (s & 1) * kBuf + dstA + ph * 32 * kRow);
  };
  auto issueB = [&](int s, const TileInfo& ti, int tk, int j) {
    glds16(sbase(p.b, ti.boff + tk * kBK) + laneBb[j], smem + (s & 1) * kBuf + dstB + j * 8 * kRow);
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
  const int cq = 4 * (lane >> 4);
  int seg = 0;  // segments (tile pieces) started so far: parity of the bias slot

  // ---- prologue: B(u0), A(u0) phases 0..3, B(u0 + 1)
  {
    const int T0 = u0 / nk, t0 = u0 - T0 * nk;
    const TileInfo a0 = tile_of(p, T0);
    const TileInfo a1 = t0 + 1 < nk ? a0 : tile_of(p, T0 + 1);
    const int t1 = t0 + 1 < nk ? t0 + 1 : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) issueB(0, a0, t0, j);
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) issueA(0, a0, t0, ph);
    const bool ok1 = u0 + 1 < u1;
#pragma unroll
    for (int j = 0; j < 4; ++j) issueB(1, ok1 ? a1 : a0, ok1 ? t1 : t0, j);
  }
  asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // the stagger: waves 4-7 one barrier behind

  // one k-tile (4 phases) of unit u; FIRST: the accumulators start from zero (and wave 0 stages
  // the tile's bias when the segment will finish the tile); XV: vector-memory instructions
  // issued since the DMA groups this k-tile's first three waits retire
  auto ktile = [&](int u, int t, const TileInfo& cur, const TileInfo& nxt, bool stage_bias, auto first_c,
                   auto xv_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr int XV = decltype(xv_c)::value;
    if (FIRST && BIAS != 0 && wave == 0 && stage_bias) {
      // the tile's 256 bias values (fp32 1 KiB / bf16 512 B) into the segment's parity LDS slot
      const char* src = BIAS == 1 ? reinterpret_cast<const char*>(static_cast<const float*>(p.bias) + cur.n0) + 16 * lane
                                  : (lane < 32 ? reinterpret_cast<const char*>(static_cast<const bf16*>(p.bias) + cur.n0) + 16 * lane
                                               : reinterpret_cast<const char*>(zero));
      glds16(src, smem + kBiasOff + (seg & 1) * 1024);
    }
    const int sl = u - u0;  // stream slot
    const char* buf = smem + (sl & 1) * kBuf;
    // DMA targets: A of unit u + 1, B of unit u + 2 (the next tile's first k-tiles at the end;
    // the current unit again past the range's end)
    const bool an = t + 1 >= nk, bn = t + 2 >= nk;
    const bool aok = u + 1 < u1, bok = u + 2 < u1;
    const int at = !aok ? t : (an ? t + 1 - nk : t + 1), bt = !bok ? t : (bn ? t + 2 - nk : t + 2);
    const TileInfo& ta = aok && an ? nxt : cur;
    const TileInfo& tb = bok && bn ? nxt : cur;
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
      issueA(sl + 1, ta, at, ph);
      if (ph == 1) {
        issueB(sl + 2, tb, bt, 0);
        issueB(sl + 2, tb, bt, 1);
      } else if (ph >= 2) {
        issueB(sl + 2, tb, bt, ph);
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
  };

  // partial slots through a buffer resource: the lane offset is one VGPR (threadIdx.x * 16), the
  // slot + element offset a wave-uniform SGPR (soffset), so the 32 stores / loads of a slot keep
  // no per-instruction 64-bit address live next to the 128 accumulator VGPRs
  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(p.ws, 0, 0x7fffffff, 0x00020000);
  const int wlane = threadIdx.x * 16;
  auto slot_off = [&](int r, int idx) { return __builtin_amdgcn_readfirstlane((r * 32 + idx) * (kThreads * 16)); };
  using Z = std::integral_constant<int, 0>;
  bool after_epi = false;
  int T = u0 / nk;
  TileInfo cur = tile_of(p, T);
  for (int u = u0; u < u1;) {
    const int ts = u - T * nk;
    const int tile_end = (T + 1) * nk;
    const int te = (u1 < tile_end ? u1 : tile_end) - T * nk;
    const TileInfo nxt = tile_of(p, T + 1 < p.tiles_m * p.tiles_n ? T + 1 : T);
    const bool finish = ts == 0;  // this segment owns the tile's first k-tile: it runs the epilogue
    if (after_epi) ktile(u, ts, cur, nxt, finish, std::true_type{}, std::integral_constant<int, kEpiVm>{});
    else ktile(u, ts, cur, nxt, finish, std::true_type{}, Z{});
    for (int t = ts + 1; t < te; ++t) ktile(u + (t - ts), t, cur, nxt, finish, std::false_type{}, Z{});
    u += te - ts;
    after_epi = false;
    if (!finish) {
      // ---- contributor: publish this segment's partial for the workgroup that finishes the tile
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, acc[ph][i][j]), wsr, wlane,
                                                   slot_off(gi, (ph * 2 + i) * 4 + j), 0);
          }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep the fence's wait (ROCm 7.2 may drop it)
      if (lane == 0) __hip_atomic_store(p.flags + gi * 8 + wave, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ++seg;
      ++T;
      cur = nxt;
      continue;  // its waits drained every older transfer: no epilogue count for the next k-tile
    }
    if (te < nk) {
      // ---- finisher of a tile the following ranges complete: add their partials (in order)
      for (int r = gi + 1; r < G && range_start(U, G, r) < (T + 1) * nk; ++r) {
        int* flag = p.flags + r * 8 + wave;
        if (lane == 0) {
          while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {  // 8 loads in flight at a time (the accumulators hold 128 VGPRs)
          i32x4 v[2][4];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[i][j] = __builtin_amdgcn_raw_buffer_load_b128(wsr, wlane, slot_off(r, (ph * 2 + i) * 4 + j), 0);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[ph][i][j] += __builtin_bit_cast(f32x4, v[i][j]);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (lane == 0) __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }

    // ---- epilogue: acc[ph][i][j][r] = C[m0 + wr*128 + 32ph + 16i + (lane & 15)][n0 + wc*64 + 16j + 4(lane >> 4) + r]
    float bias[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const char* bl = smem + kBiasOff + (seg & 1) * 1024;
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
    // outputs through buffer resources based at the tile's first element (wave-uniform SGPRs):
    // voffset = the lane's (row, column) byte offset in the tile (one VGPR), soffset = the
    // (ph, ii) row block, the j column block an immediate
    auto tile_rsrc = [&](const void* base) {
      const uint64_t a = reinterpret_cast<uint64_t>(static_cast<const bf16*>(base) + cur.m0 * p.ldc + cur.n0);
      const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
      const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
      return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0,
                                               0x7fffffff, 0x00020000);
    };
    const int ldcb = static_cast<int>(p.ldc) * 2;  // < 2^23 (gemm_nt_supported)
    const int vo = (wr * 128 + fr) * ldcb + (wc * 64 + cq) * 2;
    auto rowblk = [&](int ph, int ii) { return __builtin_amdgcn_readfirstlane((32 * ph + 16 * ii) * ldcb); };
    const __amdgpu_buffer_rsrc_t crs = tile_rsrc(p.c);
    i32x2 hv[4][2][4];  // EPI 2: every GELU input of the tile's lane issued before the first use (one round trip)
    if (EPI == 2) {
      const __amdgpu_buffer_rsrc_t hrs = tile_rsrc(p.h);
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j) hv[ph][ii][j] = __builtin_amdgcn_raw_buffer_load_b64(hrs, vo + 32 * j, rowblk(ph, ii), 0);
    }
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
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
            i32x2 gv;
            __builtin_memcpy(&gv, gg, 8);
            __builtin_amdgcn_raw_buffer_store_b64(gv, tile_rsrc(p.c2), vo + 32 * j, rowblk(ph, ii), 0);
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
          i32x2 ov;
          __builtin_memcpy(&ov, o, 8);
          __builtin_amdgcn_raw_buffer_store_b64(ov, crs, vo + 32 * j, rowblk(ph, ii), 0);
        }
      }
    }
    if (EPI == 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[j][r] = row_sum16(cs[j][r]);
      if (fr == 0) {
        float* dst = p.colpart + static_cast<int64_t>(2 * cur.tm + wr) * p.N + cur.n0 + wc * 64 + cq;
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<float4*>(dst + 16 * j) = float4{cs[j][0], cs[j][1], cs[j][2], cs[j][3]};
      }
    }
    ++seg;
    after_epi = true;
    ++T;
    cur = nxt;
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

int cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    FLUXMPI_HIP_CHECK(hipGetDevice(&dev));
    FLUXMPI_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return n;
}

// one persistent workgroup per CU (fewer when there are fewer units than CUs)
int grid_of(const NTArgs& p) {
  const int64_t U = static_cast<int64_t>(p.tiles_m) * p.tiles_n * p.nk;
  return static_cast<int>(U < cus() ? U : cus());
}

template <int EPI, int BIAS>
void launch(const NTArgs& p, hipStream_t stream) {
  gemm_nt_kernel<EPI, BIAS><<<grid_of(p), kThreads, 0, stream>>>(p);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
  // the tile grid covers M, N and K exactly (no guards in the loaders or the epilogue)
  return M > 0 && N > 0 && K >= 2 * kBK && M % kT == 0 && N % kT == 0 && K % kBK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % 8 == 0 && lda >= K && ldb >= K && ldc >= N && lda < (int64_t(1) << 23) && ldb < (int64_t(1) << 23) &&
         ldc < (int64_t(1) << 22) &&  // the epilogue's 32-bit byte offsets within a tile
         M / kT * (N / kT) * (K / kBK) < (int64_t(1) << 31);
}

int gemm_nt_colpart_rows(int64_t M) { return static_cast<int>(2 * (M / kT)); }

// stream-K workspace for one stream: fp32 partial slots [CUs][32][512] float4 and [CUs][8] int flags
// (zero-initialised once; every launch leaves them zero)
int64_t gemm_nt_ws_floats() { return static_cast<int64_t>(cus()) * 32 * kThreads * 4; }
int64_t gemm_nt_flag_ints() { return static_cast<int64_t>(cus()) * 8; }

void gemm_nt(const void* a, const void* b, void* c, void* c2, const void* bias, int bias_f32, const void* h,
             float* colpart, float* ws, int* flags, int64_t lda, int64_t ldb, int64_t ldc, int64_t M, int64_t N,
             int64_t K, int epi, hipStream_t stream) {
  if (ws == nullptr || flags == nullptr || (reinterpret_cast<uintptr_t>(ws) & 15u) != 0)
    throw std::runtime_error("gemm_nt: needs its stream-K workspace (gemm_nt_ws_floats / gemm_nt_flag_ints)");
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
           bias, static_cast<const bf16*>(h), colpart, ws, flags, lda, ldb, ldc, N, static_cast<int>(K / kBK),
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
