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
//   EPI 1: h = bf16(acc + bias): gelu'(h) -> C, gelu(h) -> C2 (fc1 forward, tanh or erf GELU;
//          the derivative is what the backward needs, so no GELU math is left for it)
//   EPI 2: dh = bf16(acc) * D[m][n] (D = EPI 1's gelu'(h)) -> C, and the column sums of dh over the wave's 128
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
// Tile order: 1-D grid, XCD-aware (bijective): the workgroups of one XCD take a contiguous block
// of tile ids round-robin in N-fastest order, so they share A row / B column panels in its L2.
// Split-K tail: the last, partial round of each XCD's block is cut into even k-tile ranges over
// all its workgroups (stream-K on the tail only: the K = 3072 ViT shapes have 591 tiles = 2.3
// rounds of 256 CUs, a third of the last round's CUs were idle); the pieces of a tile meet in a
// write-through fp32 workspace and the last arriving workgroup runs the epilogue (TailPlan).
#include <cstdint>
#include <cstdlib>
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
constexpr int kFlagOff = kBiasOff + 2048;  // split tiles: the arrival ticket's verdict
constexpr int kSmem = kFlagOff + 16;      // 130 KiB

__device__ __attribute__((aligned(64))) uint4 g_zero_nt[4];

struct NTArgs {
  const bf16* a;       // [M][lda]
  const bf16* b;       // [N][ldb]
  bf16* c;             // [M][ldc]
  bf16* c2;            // EPI 1: GELU output [M][ldc]
  const void* bias;    // [N] fp32 / bf16 (bias_f32), or nullptr
  const bf16* h;       // EPI 2: the GELU derivative gelu'(h) [M][ldc] (EPI 1's C)
  float* colpart;      // EPI 2: [2 * tiles_m][N]
  float* stats;        // EPI 3: BatchNorm statistics shards [kShards][2][N] (sum, sum of squares)
  int64_t lda, ldb, ldc;
  int64_t N;
  int nk;              // K / 64
  int tiles_m, tiles_n;
  int bias_f32;
  int gelu_tanh;
  // CONV: A is the implicit im2col of a 3x3 / stride 1 / pad 1 convolution over the NHWC image
  // batch p.a [pixels][conv_c] (K = 9 conv_c, k = tap * conv_c + channel, conv_c % 64 == 0)
  int conv_h, conv_w, conv_c;
  int conv_cpt;        // k-tiles per tap (conv_c / 64)
  float conv_inv_cpt;  // 1 / conv_cpt
  uint32_t a_bytes;    // bytes of the image (the buffer resource's range: taps outside read zeros)
  // split-K tail (stream-K on the last, partial round of each XCD's block of tiles): 0 off
  int split;
  int split_min;       // fewest k-tiles of a WG's share of the tail (even; fewer WGs take part below it)
  int max_q;           // partial-tile jobs per workgroup (workspace slots per workgroup)
  float* ws;           // fp32 partial accumulators: [G * max_q] slots of kSlotBytes
  int* counters;       // [tiles] arrival tickets of split tiles (zero between launches: the last arriver resets)
};

constexpr int kShards = 64;  // BatchNorm statistics shards (== batchnorm.hip)
constexpr int kSlotBytes = 8 * 32 * 64 * 16;  // one partial tile: 8 waves x 32 f32x4 accumulators x 64 lanes

// The tile schedule, identical on host and device (host: workspace size, max_q). The tiles
// (N-fastest) are dealt to the XCDs as G contiguous ranges (workgroup b runs on XCD b % 8, a
// speed assumption only); inside an XCD's block [tb, te) its nx workgroups take the tiles
// round-robin (workgroup pos: tb + pos, tb + pos + nx, ...) for the F = (te - tb) / nx full rounds.
// The R = (te - tb) % nx tiles of the last round: without split, one each for workgroups 0..R-1;
// with split (stream-K tail), their R * nk k-tiles are cut into nw equal, even-length ranges, one
// per workgroup (nw = min(nx, units / split_min)), so the tail takes ~R / nx of a round instead
// of a whole one. A range may cover parts of several tiles: a partial-tile job; the pieces of a
// tile are summed by whichever workgroup arrives last (below).
struct TailPlan {
  int tb, nx, pos;
  int nfull;     // full-tile jobs of this workgroup
  int tt0;       // first tail tile (split)
  int u2, nw;    // tail units in k-tile PAIRS, workgroups sharing it (0 if no split tail)
  int s, e;      // this workgroup's tail k-tile range [s, e) (split and pos < nw), else s = e = 0
  __host__ __device__ int bnd(int w) const { return 2 * static_cast<int>(static_cast<int64_t>(u2) * w / nw); }
  // workgroup (position) whose range holds tail k-tile x
  __host__ __device__ int wg_of(int x) const {
    return static_cast<int>((static_cast<int64_t>(x / 2 + 1) * nw - 1) / u2);
  }
};

__host__ __device__ inline int range_start_hd(int tiles, int G, int r) {
  return static_cast<int>(static_cast<int64_t>(tiles) * r / G);
}

__host__ __device__ inline TailPlan tail_plan(int tiles, int G, int nk, int split, int split_min, int b) {
  TailPlan t{};
  const int q = G / 8, r = G % 8, xcd = b % 8, pos = b / 8;
  const int gx0 = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, nx = q + (xcd < r ? 1 : 0);
  const int tb = range_start_hd(tiles, G, gx0), te = range_start_hd(tiles, G, gx0 + nx);
  t.tb = tb, t.nx = nx, t.pos = pos;
  const int T = te - tb, F = nx > 0 ? T / nx : 0, R = T - F * nx;
  t.tt0 = tb + F * nx;
  if (split && R > 0) {
    t.u2 = R * nk / 2;
    const int want = (2 * t.u2) / (split_min > 2 ? split_min : 2);
    t.nw = want < 1 ? 1 : (want > nx ? nx : want);
    t.nfull = F;
    if (pos < t.nw) t.s = t.bnd(pos), t.e = t.bnd(pos + 1);
  } else {
    t.u2 = 0, t.nw = 0;
    t.nfull = F + (pos < R ? 1 : 0);
  }
  return t;
}

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

// After an epilogue's 16-B store: a scheduling fence and STORE_GUARD_NOPS + 1 wait states before
// any later instruction may overwrite the store's data registers. hipcc (ROCm 7.2) lets a VALU
// rewrite them 1-2 states after a buffer_store_dwordx4, which gfx950 does not tolerate under a full
// store queue: the fc2 input-gradient epilogue (EPI 2) wrote ~20 wrong elements per launch, always
// the lanes of two rows of one 16-row block, on the split tiles (whose epilogue runs while other
// workgroups store), and the same build with a wait after each store, or with its loads reordered,
// was clean over 40 launches (profiles/rd5c_gemm_nt_store_hazard.md). The earlier "SLP build gives
// NaNs in EPI 1" (round 4) is the same hazard: packed VALU moved closer to the stores.
#ifndef STORE_GUARD_NOPS
#define STORE_GUARD_NOPS 3
#endif
__device__ __forceinline__ void store_guard() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop %0" ::"n"(STORE_GUARD_NOPS));
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf16x8 frag(const char* __restrict__ p) { return *reinterpret_cast<const bf16x8*>(p); }

// Persistent, tile-granular: the tiles (N-fastest) are dealt to the G = min(tiles, CUs)
// workgroups as equal contiguous ranges (the workgroups of one XCD take neighbouring ranges, so
// they share A row panels in its L2). A workgroup's tiles are ONE stream of k-tile units (slot s
// uses LDS buffer s & 1): the DMA of the next tile's first k-tiles is in flight while this tile's
// epilogue stores. (A stream-K split with fp32 partials handed between workgroups measured
// 1.5x slower on the ViT shapes: a hand-off across the XCDs' non-coherent L2s costs an L2
// write-back + invalidate or write-through traffic per tile — MI355X_MICROARCH.md price list,
// "publish-large" / "splitk-seam"; profiles/rd4d_bench_gemm_nt_streamk_first.jsonl.)
// After an epilogue the first k-tile's waits count its vector-memory instructions (kEpiVm):
// they are younger than the DMA groups those waits retire.
// BIAS: 0 none, 1 fp32, 2 bf16 (EPI 0 / 1), staged into LDS by one LDS-DMA of wave 0 at the
// tile's first k-tile (slot = tile parity).
struct TileInfo {  // one job, wave-uniform (SGPRs); every offset below fits 32 bits (gemm_nt_supported)
  int tm, tn;
  int id;       // tile id (N-fastest)
  int k0, k1;   // the job's k-tiles [k0, k1) (a full tile: [0, nk)); always >= 2 of them
  int r;        // split tail: the tile's index in the tail (-1: a full-tile job)
  __device__ __forceinline__ int m0() const { return tm * kT; }
  __device__ __forceinline__ int n0() const { return tn * kT; }
};

__device__ __forceinline__ TileInfo tile_of(const NTArgs& p, int T) {
  TileInfo t;
  T = __builtin_amdgcn_readfirstlane(T);
  t.id = T;
  t.tm = __builtin_amdgcn_readfirstlane(T / p.tiles_n);
  t.tn = T - t.tm * p.tiles_n;
  t.k0 = 0, t.k1 = p.nk, t.r = -1;
  return t;
}

// an opaque copy: values derived from it are recomputed where they are used instead of being
// hoisted out of the tile loop by LICM and kept live (spilled) across the whole k-tile stream
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <int EPI, int BIAS, bool CONV, int GF = 1>  // GF (EPI 1 / 2): 1 tanh GELU, 0 erf GELU
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[kSmem];
  // vector-memory instructions per wave in an epilogue (lower bound: unconditional ones)
  constexpr int kEpiVm = EPI == 1 || EPI == 2 || EPI == 4 ? 32 : 16;
  const int G = gridDim.x;
  const int nk = p.nk;  // >= 2
  const int tiles = p.tiles_m * p.tiles_n;
  // The schedule (TailPlan): workgroup `pos` of an XCD takes tiles tb + pos, tb + pos + nx, ... — at
  // any moment the XCD's workgroups work on neighbouring tiles (N-fastest), which share A row
  // panels and B column panels in its L2 (contiguous per-workgroup ranges re-read a panel from
  // beyond L2 for each tile: L2 hit rate 48 % on qkv, profiles/rd4ab_gemm_nt_pmc.md) — then, with
  // the split tail, its share of the last round's k-tiles as partial-tile jobs.
  const TailPlan tp = tail_plan(tiles, G, nk, p.split, p.split_min, blockIdx.x);
  const int ntail = tp.e > tp.s ? (tp.e - 1) / nk - tp.s / nk + 1 : 0;
  const int nJ = __builtin_amdgcn_readfirstlane(tp.nfull + ntail);
  if (nJ <= 0) return;  // workgroup-uniform, before any DMA or barrier
  auto job_of = [&](int jj) -> TileInfo {
    if (jj < tp.nfull) return tile_of(p, tp.tb + tp.pos + jj * tp.nx);
    const int r = tp.s / nk + (jj - tp.nfull);
    TileInfo t = tile_of(p, tp.tt0 + r);
    const int a = tp.s - r * nk, b = tp.e - r * nk;
    t.k0 = __builtin_amdgcn_readfirstlane(a > 0 ? a : 0);
    t.k1 = __builtin_amdgcn_readfirstlane(b < nk ? b : nk);
    t.r = __builtin_amdgcn_readfirstlane(r);
    return t;
  };
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave-uniform
  const int wr = wave >> 2, wc = wave & 3;

  // ---- LDS-DMA lanes: a wave-instruction fills 8 rows x 8 chunks; lane -> row lane >> 3, slot lane & 7
  const int lrow = lane >> 3, lslot = lane & 7;
  // A rows of phase p: waves 0-3 rows 32p + 8w, waves 4-7 rows 128 + 32p + 8(w-4) (+ lrow);
  // the swizzle of row + 32p equals that of row
  const int arow = (wave & 4) * 32 + (wave & 3) * 8 + lrow;
  const int laneA = arow * static_cast<int>(p.lda) + ((lslot ^ swz(arow)) << 3);  // < 2^31: lda < 2^23
  const int lda2 = static_cast<int>(p.lda) * 2, ldb2 = static_cast<int>(p.ldb) * 2;  // bytes per row
  const int dstA = (arow - lrow) * kRow;
  // B rows of piece j: 32w + 8j + lrow
  // B rows of piece j: 32w + 8j + lrow; the swizzle of row + 8j is that of row ^ 4 (j odd), so
  // two lane offsets (j even / odd) + a wave-uniform 8j rows
  uint32_t laneBb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 32 * wave + 8 * j + lrow;
    laneBb[j] = static_cast<uint32_t>(lrow * static_cast<int>(p.ldb) + ((lslot ^ swz(row)) << 3)) * 2u;
  }
  const int bwave = 32 * wave * static_cast<int>(p.ldb) * 2;
  const int dstB = kImg + 32 * wave * kRow;
  const void* zero = g_zero_nt;

  // DMA into stream slot s (LDS buffer s & 1) of k-tile tk of tile `ti`. Source = a wave-uniform
  // base (SGPRs: readfirstlane) + the lane's 32-bit byte offset, so no 64-bit per-lane address is
  // kept live across the loop. Past the range's end (`ok` false) the slot is dead and the DMA just
  // re-reads valid bytes (the caller passes the current unit), keeping the vmcnt count fixed.
  const uint32_t laneAb = static_cast<uint32_t>(laneA) * 2u;
  // CONV: the A rows a lane stages are output pixels m = m0 + arow + 32 ph of the tile whose
  // info is loaded (conv_info: at the prologue and when the issues move on to the next tile);
  // pixb = phase 0's pixel byte offset + the lane's chunk, vmask = its in-image taps (9 bits per
  // phase, phases 2k / 2k+1 in halves of word k). A k-tile lies inside one tap (conv_c % 64 == 0):
  // the tap's pixel shift and the channel offset are wave-uniform, and an out-of-image tap's
  // offset is past the buffer's range, which the LDS-DMA reads as zeros (the padding).
  struct ConvRows {
    uint32_t pixb = 0;      // phase 0's pixel byte offset + the lane's chunk (phase ph adds 32 ph pixels)
    uint32_t vmask[2] = {};  // in-image taps: 9 bits per phase, phases 2k / 2k+1 in halves of word k
  };
  ConvRows crow, crow_n;  // the current tile's rows, the next tile's (computed once per segment)
  const __amdgpu_buffer_rsrc_t arsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.a), 0, CONV ? p.a_bytes : 0x7fffffffu, 0x00020000);
  auto conv_info = [&](const TileInfo& ti, ConvRows& cr) {
    const uint32_t chunkb = static_cast<uint32_t>((lslot ^ swz(arow)) << 4);
    const int H = p.conv_h, W = p.conv_w, HW = H * W;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int m = ti.m0() + arow + 32 * ph;  // < 2^31 (gemm_nt_conv_supported)
      const int hw = m % HW, h = hw / W, w = hw - h * W;
      if (ph == 0) cr.pixb = static_cast<uint32_t>(m) * static_cast<uint32_t>(p.conv_c) * 2u + chunkb;
      const uint32_t rm = (h > 0 ? 1u : 0u) | 2u | (h < H - 1 ? 4u : 0u);
      const uint32_t cm = (w > 0 ? 1u : 0u) | 2u | (w < W - 1 ? 4u : 0u);
      const uint32_t m9 = ((rm & 1u) ? cm : 0u) | ((rm & 2u) ? cm << 3 : 0u) | ((rm & 4u) ? cm << 6 : 0u);
      if (ph & 1) cr.vmask[ph >> 1] |= m9 << 16;
      else cr.vmask[ph >> 1] = m9;
    }
  };
  auto issueA = [&](int s, const TileInfo& ti, int tk, int ph, bool next_tile) {
    if constexpr (CONV) {
      const int tap = __builtin_amdgcn_readfirstlane(static_cast<int>((static_cast<float>(tk) + 0.5f) * p.conv_inv_cpt));
      const int r3 = (tap * 11) >> 5;  // tap / 3 for tap < 9
      const int c0 = (tk - tap * p.conv_cpt) * kBK;
      const int sh =
          __builtin_amdgcn_readfirstlane((((r3 - 1) * p.conv_w + (tap - 3 * r3 - 1) + 32 * ph) * p.conv_c + c0) * 2);
      const uint32_t vm = next_tile ? crow_n.vmask[ph >> 1] : crow.vmask[ph >> 1];
      const uint32_t pb = next_tile ? crow_n.pixb : crow.pixb;
      const uint32_t vo = (vm >> (tap + 16 * (ph & 1))) & 1u ? pb + static_cast<uint32_t>(sh) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_char*)(smem + (s & 1) * kBuf + dstA + ph * 32 * kRow), 16,
                                               vo, 0, 0, 0);
    } else {
      const int so = __builtin_amdgcn_readfirstlane((ti.m0() + 32 * ph) * lda2 + tk * kRow);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_char*)(smem + (s & 1) * kBuf + dstA + ph * 32 * kRow), 16,
                                               laneAb, so, 0, 0);
    }
  };
  // B through a buffer resource: the lane's 32-bit byte offset (voffset) + the tile / k-tile
  // offset (soffset, wave-uniform) — no 64-bit per-lane address is formed or kept
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.b), 0, 0x7fffffff, 0x00020000);
  auto issueB = [&](int s, const TileInfo& ti, int tk, int j) {
    const int so = __builtin_amdgcn_readfirstlane((ti.n0() + 8 * j) * ldb2 + tk * kRow + bwave);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_char*)(smem + (s & 1) * kBuf + dstB + j * 8 * kRow), 16,
                                             laneBb[j & 1], so, 0, 0);
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
  int seg = 0;  // tiles started so far: parity of the bias slot

  // ---- prologue: B(u0), A(u0) phases 0..3, B(u0 + 1)
  TileInfo cur = job_of(0);
  {  // a job has >= 2 k-tiles, so unit 1 is the first job's second k-tile
    if constexpr (CONV) conv_info(cur, crow);
#pragma unroll
    for (int j = 0; j < 4; ++j) issueB(0, cur, cur.k0, j);
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) issueA(0, cur, cur.k0, ph, false);
#pragma unroll
    for (int j = 0; j < 4; ++j) issueB(1, cur, cur.k0 + 1, j);
  }
  asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // the stagger: waves 4-7 one barrier behind

  // one k-tile (4 phases) of stream unit u (k-tile t of job `cur`; `nxt` the next job, if
  // has_next); FIRST: the accumulators start from zero (and wave 0 stages the tile's bias);
  // XV: vector-memory instructions issued since the DMA groups this k-tile's first three waits retire
  auto ktile = [&](int u, int t, const TileInfo& cur, const TileInfo& nxt, bool has_next, auto first_c, auto xv_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr int XV = decltype(xv_c)::value;
    if (FIRST && BIAS != 0 && wave == 0) {
      // the tile's 256 bias values (fp32 1 KiB / bf16 512 B) into the segment's parity LDS slot
      const char* src = BIAS == 1 ? reinterpret_cast<const char*>(static_cast<const float*>(p.bias) + cur.n0()) + 16 * lane
                                  : (lane < 32 ? reinterpret_cast<const char*>(static_cast<const bf16*>(p.bias) + cur.n0()) + 16 * lane
                                               : reinterpret_cast<const char*>(zero));
      glds16(src, smem + kBiasOff + (seg & 1) * 1024);
    }
    const int sl = u;  // stream slot
    const char* buf = smem + (sl & 1) * kBuf;
    // DMA targets: A of unit u + 1, B of unit u + 2 (the next job's first k-tiles at the end — it
    // has >= 2; the current unit again past the last job's end)
    const bool an = t + 1 >= cur.k1, bn = t + 2 >= cur.k1;
    const bool aok = !an || has_next, bok = !bn || has_next;
    const int at = !aok ? t : (an ? nxt.k0 : t + 1), bt = !bok ? t : (bn ? nxt.k0 + (t + 2 - cur.k1) : t + 2);
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
      issueA(sl + 1, ta, at, ph, aok && an);
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

  using Z = std::integral_constant<int, 0>;
  bool after_epi = false;
  bool staggered = true;  // waves 4-7 one barrier behind (undone around a split tile's fix-up)
  int* const lds_flag = reinterpret_cast<int*>(smem + kFlagOff);
  int u = 0;
  for (int jb = 0; jb < nJ; ++jb) {
    const bool has_next = jb + 1 < nJ;
    const TileInfo nxt = job_of(has_next ? jb + 1 : jb);
    if constexpr (CONV) conv_info(nxt, crow_n);  // for the A issues of this job's last k-tile
    if (!staggered) {  // re-stagger after a fix-up: waves 4-7 fall one barrier behind again
      if (wr == 1) __builtin_amdgcn_s_barrier();
      staggered = true;
    }
    if (after_epi) ktile(u, cur.k0, cur, nxt, has_next, std::true_type{}, std::integral_constant<int, kEpiVm>{});
    else ktile(u, cur.k0, cur, nxt, has_next, std::true_type{}, Z{});
    ++u;
    for (int t = cur.k0 + 1; t < cur.k1; ++t, ++u) ktile(u, t, cur, nxt, has_next, std::false_type{}, Z{});

    // ---- split tile: every piece stores its fp32 accumulators write-through (sc1) into its
    // workspace slot; after every wave's stores have completed (vmcnt(0) + barrier) one lane takes
    // an arrival ticket (agent-scope atomic); the workgroup that arrives last sums ALL pieces'
    // slots in piece order (deterministic: the same sum whichever arrives last; its own piece
    // re-read too) with sc1 loads and runs the epilogue; the others move on. No workgroup ever
    // waits for another (no residency assumption). Hand-off form: MI355X_MICROARCH.md
    // "Valid forms" table, row 1 (sc1 stores + drained waits + last-add ticket + sc1 loads).
    bool do_epi = true;
    if (cur.r >= 0) {
      const int x0 = cur.r * nk;
      const int wlo = __builtin_amdgcn_readfirstlane(tp.wg_of(x0)), whi = __builtin_amdgcn_readfirstlane(tp.wg_of(x0 + nk - 1));
      const int P = whi - wlo + 1;
      if (P > 1) {
        if (wr == 0) __builtin_amdgcn_s_barrier();  // unstagger: all 8 waves at the same barrier count
        staggered = false;
        const int xcd = blockIdx.x % 8;
        auto slot_rsrc = [&](int w) {
          const int qw = cur.r - tp.bnd(w) / nk;
          const int64_t slot = static_cast<int64_t>(w * 8 + xcd) * p.max_q + qw;
          const uint64_t a = reinterpret_cast<uint64_t>(reinterpret_cast<char*>(p.ws) + slot * kSlotBytes);
          const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
          const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
          return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0,
                                                   kSlotBytes, 0x00020000);
        };
        // + 1 KiB per accumulator register (opaque: not hoisted out of the job loop, no VGPR kept live)
        const int pvo = (wave * 32 * 64 + opaque(lane)) * 16;
        {
          const __amdgpu_buffer_rsrc_t ms = slot_rsrc(tp.pos);
#pragma unroll
          for (int ph = 0; ph < 4; ++ph)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int jj = 0; jj < 4; ++jj)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, acc[ph][i][jj]), ms,
                                                       pvo + 1024 * (8 * ph + 4 * i + jj), 0, 16 /* sc1 */);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (threadIdx.x == 0) {
          const int tk = __hip_atomic_fetch_add(p.counters + cur.id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const int last = tk == P - 1 ? 1 : 0;
          if (last) __hip_atomic_store(p.counters + cur.id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(lds_flag, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        do_epi = __builtin_amdgcn_readfirstlane(__hip_atomic_load(lds_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
        if (do_epi) {
          for (int pc = 0; pc < P; ++pc) {  // piece order
            const __amdgpu_buffer_rsrc_t rs = slot_rsrc(wlo + pc);
            if (pc == 0) {
#pragma unroll
              for (int ph = 0; ph < 4; ++ph)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                  for (int jj = 0; jj < 4; ++jj)
                    acc[ph][i][jj] = __builtin_bit_cast(
                        f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, pvo + 1024 * (8 * ph + 4 * i + jj), 0, 16));
            } else {
#pragma unroll
              for (int ph = 0; ph < 4; ++ph) {  // 8 loads in flight per batch (32 VGPRs)
                f32x4 tmp[2][4];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                  for (int jj = 0; jj < 4; ++jj)
                    tmp[i][jj] = __builtin_bit_cast(
                        f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, pvo + 1024 * (8 * ph + 4 * i + jj), 0, 16));
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                  for (int jj = 0; jj < 4; ++jj) acc[ph][i][jj] += tmp[i][jj];
              }
            }
          }
        }
      }
    }
    if (do_epi) {

    // ---- epilogue. acc[ph][i][j][r] = C[m0 + wr*128 + 32ph + 16i + (lane & 15)][n0 + wc*64 + 16j + 4(lane >> 4) + r].
    // The rounded values are exchanged between lane rows g and g ^ 1 (v_permlane16_swap: row 2k
    // keeps its own 4 columns of block 2p and receives row 2k+1's, row 2k+1 likewise for block
    // 2p + 1), so each lane holds 8 consecutive columns: 16-B stores / GELU-input loads instead
    // of 8-B ones (half the instructions, whole 64-B segments). Lane row g holds, for pair p,
    // columns 32p + 16 (g & 1) + 8 (g >> 1) .. + 7 of the wave's 64.
    const int lane_e = opaque(lane), fr_e = lane_e & 15, g_e = lane_e >> 4, cq_e = 4 * g_e;
    float bias[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const char* bl = smem + kBiasOff + (seg & 1) * 1024;
      const int col = wc * 64 + 16 * j + cq_e;
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
    const int colx = wc * 64 + 16 * (g_e & 1) + 8 * (g_e >> 1);  // the lane's first column (pair 0)
    float cs[2][8], cq2[EPI == 3 ? 2 : 1][8];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[q][e] = 0.f;
        if (EPI == 3) cq2[q][e] = 0.f;
      }
    // outputs through buffer resources based at the tile's first element (wave-uniform SGPRs):
    // voffset = the lane's (row, column) byte offset in the tile (one VGPR), soffset = the
    // (ph, ii) row block, the column pair an immediate
    auto tile_rsrc = [&](const void* base) {
      const uint64_t a = reinterpret_cast<uint64_t>(static_cast<const bf16*>(base) +
                                                    static_cast<int64_t>(cur.m0()) * p.ldc + cur.n0());
      const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
      const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
      return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0,
                                               0x7fffffff, 0x00020000);
    };
    const int ldcb = static_cast<int>(p.ldc) * 2;  // < 2^23 (gemm_nt_supported)
    const int vo = (wr * 128 + fr_e) * ldcb + colx * 2;
    auto rowblk = [&](int ph, int ii) { return __builtin_amdgcn_readfirstlane((32 * ph + 16 * ii) * ldcb); };
    const __amdgpu_buffer_rsrc_t crs = tile_rsrc(p.c);
    i32x4 hv[4][2][2];  // EPI 2: every GELU derivative of the tile's lane issued before the first use (one round trip)
#ifndef GNT_DBG_HVLATE
    if (EPI == 2 || EPI == 4) {
      const __amdgpu_buffer_rsrc_t hrs = tile_rsrc(p.h);
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int q = 0; q < 2; ++q) hv[ph][ii][q] = __builtin_amdgcn_raw_buffer_load_b128(hrs, vo + 64 * q, rowblk(ph, ii), 0);
    }
#endif
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
#ifdef GNT_DBG_HVLATE
      if (EPI == 2 || EPI == 4) {
        const __amdgpu_buffer_rsrc_t hrs = tile_rsrc(p.h);
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int q = 0; q < 2; ++q) hv[ph][ii][q] = __builtin_amdgcn_raw_buffer_load_b128(hrs, vo + 64 * q, rowblk(ph, ii), 0);
      }
#endif
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        uint32_t lo[4], hi[4];  // bf16 pairs (columns r 0-1 / 2-3) of each block j, this lane's columns
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bf16 o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = static_cast<bf16>(acc[ph][ii][j][r] + bias[j][r]);  // EPI 2/3: bias 0
          __builtin_memcpy(&lo[j], o, 4);
          __builtin_memcpy(&hi[j], o + 2, 4);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const auto xl = __builtin_amdgcn_permlane16_swap(lo[2 * q], lo[2 * q + 1], false, false);
          const auto xh = __builtin_amdgcn_permlane16_swap(hi[2 * q], hi[2 * q + 1], false, false);
          const uint32_t w0 = xl[0], w1 = xh[0], w2 = xl[1], w3 = xh[1];
          const i32x4 w = {static_cast<int>(w0), static_cast<int>(w1), static_cast<int>(w2), static_cast<int>(w3)};
          bf16 v8[8];
          __builtin_memcpy(v8, &w, 16);
          i32x4 out = w;
          if (EPI == 3) {  // the BatchNorm statistics of the rounded output
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float f = static_cast<float>(v8[e]);
              cs[q][e] += f;
              cq2[q][e] = fmaf(f, f, cq2[q][e]);
            }
          } else if (EPI == 1) {
            // h = the bf16 pre-activation (as F.gelu(F.linear(...)) sees it): g = gelu(h) -> C2 and
            // its derivative gelu'(h) -> C (what the backward multiplies by; the pre-activation
            // itself is not needed again), both from one tanh / erf evaluation
            bf16 gg[8], dd[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = static_cast<float>(v8[e]);
              if constexpr (GF == 1) {
                constexpr float kK0 = 0.79788456080286536f, kK3 = 3.f * 0.044715f;
                const float t = gelu_tanh_t(x), hx = 0.5f * x;
                gg[e] = static_cast<bf16>(fmaf(hx, t, hx));
                dd[e] = static_cast<bf16>(fmaf(hx * fmaf(-t, t, 1.f), kK0 * fmaf(kK3 * x, x, 1.f), fmaf(0.5f, t, 0.5f)));
              } else {
                float cdf, ee;
                gelu_parts(x, cdf, ee);
                gg[e] = static_cast<bf16>(x * cdf);
                dd[e] = static_cast<bf16>(fmaf(x * 0.39894228040143268f, ee, cdf));
              }
            }
            i32x4 gv;
            __builtin_memcpy(&gv, gg, 16);
            __builtin_amdgcn_raw_buffer_store_b128(gv, tile_rsrc(p.c2), vo + 64 * q, rowblk(ph, ii), 0);
            store_guard();
            __builtin_memcpy(&out, dd, 16);
          } else if (EPI == 2) {
            // dh = bf16(dg) * gelu'(h), the derivative read as the forward epilogue (EPI 1) stored it
            bf16 dd[8], oo[8];
            __builtin_memcpy(dd, &hv[ph][ii][q], 16);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              oo[e] = static_cast<bf16>(static_cast<float>(v8[e]) * static_cast<float>(dd[e]));
              cs[q][e] += static_cast<float>(oo[e]);  // the bias gradient of the rounded dh
            }
            __builtin_memcpy(&out, oo, 16);
          } else if (EPI == 4) {
            // y = bf16(bf16(acc) + r): the residual summand of the input's gradient (a second
            // consumer's share), added to the rounded product in the exchanged 8-column layout
            bf16 rr[8], oo[8];
            __builtin_memcpy(rr, &hv[ph][ii][q], 16);
#pragma unroll
            for (int e = 0; e < 8; ++e) oo[e] = static_cast<bf16>(static_cast<float>(v8[e]) + static_cast<float>(rr[e]));
            __builtin_memcpy(&out, oo, 16);
          }
          __builtin_amdgcn_raw_buffer_store_b128(out, crs, vo + 64 * q, rowblk(ph, ii), 0);
          store_guard();
        }
      }
    }
    if (EPI == 2 || EPI == 3) {
      // the wave's 128 rows summed per column (butterflies over the 16 row lanes)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          cs[q][e] = row_sum16(cs[q][e]);
          if (EPI == 3) cq2[q][e] = row_sum16(cq2[q][e]);
        }
    }
    if (EPI == 2 && fr_e == 0) {  // fc1's bias-gradient partials: row 2 tm + wr of colpart
      float* dst = p.colpart + static_cast<int64_t>(2 * cur.tm + wr) * p.N + cur.n0() + colx;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        *reinterpret_cast<float4*>(dst + 32 * q) = float4{cs[q][0], cs[q][1], cs[q][2], cs[q][3]};
        *reinterpret_cast<float4*>(dst + 32 * q + 4) = float4{cs[q][4], cs[q][5], cs[q][6], cs[q][7]};
      }
    }
    if (EPI == 3 && fr_e == 0) {  // one atomic per column per wave row into the tile's statistics shard
      float* shard = p.stats + static_cast<int64_t>(cur.id % kShards) * 2 * p.N + cur.n0() + colx;
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          atomicAdd(shard + 32 * q + e, cs[q][e]);
          atomicAdd(shard + p.N + 32 * q + e, cq2[q][e]);
        }
    }
    }  // do_epi
    ++seg;
    after_epi = true;
    cur = nxt;
    if constexpr (CONV) crow = crow_n;
  }
  if (staggered && wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
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

// FLUXMPI_GEMM_NT_SPLIT: the fewest k-tiles of a workgroup's share of the split tail (0: no split,
// the default — measured slower end to end: ResNet-50 20.85 vs 20.32 ms/step, ViT-B/16 per-GEMM
// -7..+5 %, profiles/rd5d_*; 8 / 16: the tested settings). Shapes with an odd k-tile count or
// fewer than 16 k-tiles are never split.
int g_split_min = -1;  // < 0: not yet read from the environment

int split_norm(int x) { return x <= 0 ? 0 : (x < 2 ? 2 : x + (x & 1)); }

int split_min() {
  if (g_split_min < 0) {
    const char* e = std::getenv("FLUXMPI_GEMM_NT_SPLIT");
    g_split_min = split_norm(e != nullptr ? std::atoi(e) : 0);
  }
  return g_split_min;
}

// The split-tail workspace of the current device: fp32 partial slots and per-tile arrival
// counters (zeroed once; each split tile's last arriver resets its counter). One per device:
// gemm_nt launches are ordered on the compute stream (the DDP comm stream runs no GEMM), so no
// two launches use it at once. Grown outside stream capture only (warm-up calls size it).
struct SplitWs {
  float* ws = nullptr;
  size_t ws_bytes = 0;
  int* counters = nullptr;
  size_t n_counters = 0;
};

bool split_workspace(size_t ws_bytes, size_t n_counters, hipStream_t stream, float** ws, int** counters) {
  static SplitWs per_dev[64];
  int dev = 0;
  FLUXMPI_HIP_CHECK(hipGetDevice(&dev));
  SplitWs& w = per_dev[dev & 63];
  if (w.ws_bytes < ws_bytes || w.n_counters < n_counters) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    FLUXMPI_HIP_CHECK(hipStreamIsCapturing(stream, &cs));
    if (cs != hipStreamCaptureStatusNone) return false;  // no allocation inside a capture: run unsplit
    if (w.ws_bytes < ws_bytes) {
      if (w.ws != nullptr) FLUXMPI_HIP_CHECK(hipFree(w.ws));  // implicit device sync: no launch still reads it
      FLUXMPI_HIP_CHECK(hipMalloc(&w.ws, ws_bytes));
      w.ws_bytes = ws_bytes;
    }
    if (w.n_counters < n_counters) {
      if (w.counters != nullptr) FLUXMPI_HIP_CHECK(hipFree(w.counters));
      FLUXMPI_HIP_CHECK(hipMalloc(&w.counters, n_counters * sizeof(int)));
      FLUXMPI_HIP_CHECK(hipMemsetAsync(w.counters, 0, n_counters * sizeof(int), stream));
      w.n_counters = n_counters;
    }
  }
  *ws = w.ws, *counters = w.counters;
  return true;
}

// grid and split-tail setup: one persistent workgroup per CU (fewer when there are fewer tiles
// than CUs and no split); with a split tail every CU takes part and p.max_q / ws / counters are set
int setup_grid(NTArgs& p, hipStream_t stream) {
  const int64_t tiles = static_cast<int64_t>(p.tiles_m) * p.tiles_n;
  const int n = cus();
  p.split = 0, p.split_min = 2, p.max_q = 0, p.ws = nullptr, p.counters = nullptr;
  const int sm = split_min();
  if (sm > 0 && p.nk % 2 == 0 && p.nk >= 16 && tiles % n != 0) {
    const int G = n;
    int max_q = 0;
    for (int b = 0; b < G && b < 8; ++b) {  // every XCD's plan (positions 0..nw-1)
      for (int pos = 0;; ++pos) {
        const int bb = pos * 8 + b;
        if (bb >= G) break;
        const TailPlan t = tail_plan(static_cast<int>(tiles), G, p.nk, 1, sm, bb);
        if (t.e > t.s) {
          const int q = (t.e - 1) / p.nk - t.s / p.nk + 1;
          max_q = q > max_q ? q : max_q;
        }
      }
    }
    if (max_q > 0) {
      float* ws = nullptr;
      int* cnt = nullptr;
      if (split_workspace(static_cast<size_t>(G) * max_q * kSlotBytes, static_cast<size_t>(tiles), stream, &ws, &cnt)) {
        p.split = 1, p.split_min = sm, p.max_q = max_q, p.ws = ws, p.counters = cnt;
        return G;
      }
    }
  }
  return static_cast<int>(tiles < n ? tiles : n);
}

template <int EPI, int BIAS, bool CONV = false>
void launch(NTArgs& p, hipStream_t stream) {
  const int grid = setup_grid(p, stream);
  if constexpr (EPI == 1) {  // the GELU form is compiled in (its constants would stay live otherwise)
    if (p.gelu_tanh) gemm_nt_kernel<EPI, BIAS, CONV, 1><<<grid, kThreads, 0, stream>>>(p);
    else gemm_nt_kernel<EPI, BIAS, CONV, 0><<<grid, kThreads, 0, stream>>>(p);
  } else {
    gemm_nt_kernel<EPI, BIAS, CONV><<<grid, kThreads, 0, stream>>>(p);
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
  // the tile grid covers M, N and K exactly (no guards in the loaders or the epilogue)
  return M > 0 && N > 0 && K >= 2 * kBK && M % kT == 0 && N % kT == 0 && K % kBK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % 8 == 0 && lda >= K && ldb >= K && ldc >= N && lda < (int64_t(1) << 23) && ldb < (int64_t(1) << 23) &&
         ldc < (int64_t(1) << 22) &&  // the epilogue's 32-bit byte offsets within a tile
         M * lda * 2 < (int64_t(1) << 31) && N * ldb * 2 < (int64_t(1) << 31) &&  // 32-bit DMA offsets
         M / kT * (N / kT) * (K / kBK) < (int64_t(1) << 31);
}

bool gemm_nt_conv_supported(int64_t pixels, int64_t C, int64_t Cout) {
  // output pixels tile exactly, a k-tile inside one tap, 32-bit byte offsets into the image
  return C > 0 && C % kBK == 0 && pixels * C * 2 < (int64_t(1) << 31) &&
         gemm_nt_supported(pixels, Cout, 9 * C, 9 * C, 9 * C, Cout);
}

void gemm_nt_set_split(int min_ktiles) { g_split_min = split_norm(min_ktiles); }
int gemm_nt_get_split() { return split_min(); }

int gemm_nt_colpart_rows(int64_t M) { return static_cast<int>(2 * (M / kT)); }

void gemm_nt(const void* a, const void* b, void* c, void* c2, const void* bias, int bias_f32, const void* h,
             float* colpart, float* stats, int64_t lda, int64_t ldb, int64_t ldc, int64_t M, int64_t N, int64_t K,
             int epi, hipStream_t stream) {
  if (!gemm_nt_supported(M, N, K, lda, ldb, ldc))
    throw std::runtime_error("gemm_nt: unsupported shape (M, N multiples of 256, K of 64, leading dims of 8; M=" +
                             std::to_string(M) + " N=" + std::to_string(N) + " K=" + std::to_string(K) + ")");
  if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15u) != 0)
    throw std::runtime_error("gemm_nt: operands must be 16-byte aligned");
  if (epi == 1 && c2 == nullptr) throw std::runtime_error("gemm_nt: the GELU epilogue needs the second output");
  if (epi == 2 && (h == nullptr || colpart == nullptr))
    throw std::runtime_error("gemm_nt: the GELU-backward epilogue needs h and colpart");
  if (epi == 3 && (stats == nullptr || bias != nullptr))
    throw std::runtime_error("gemm_nt: the statistics epilogue needs the shard workspace (and takes no bias)");
  if (bias != nullptr && (reinterpret_cast<uintptr_t>(bias) & (bias_f32 ? 15u : 7u)) != 0)
    throw std::runtime_error("gemm_nt: bias must be 16-byte (fp32) / 8-byte (bf16) aligned");
  NTArgs p{};
  p.a = static_cast<const bf16*>(a), p.b = static_cast<const bf16*>(b), p.c = static_cast<bf16*>(c);
  p.c2 = static_cast<bf16*>(c2), p.bias = bias, p.h = static_cast<const bf16*>(h), p.colpart = colpart;
  p.stats = stats, p.lda = lda, p.ldb = ldb, p.ldc = ldc, p.N = N;
  p.nk = static_cast<int>(K / kBK), p.tiles_m = static_cast<int>(M / kT), p.tiles_n = static_cast<int>(N / kT);
  p.bias_f32 = bias_f32, p.gelu_tanh = gelu_form();
  const int bk = bias == nullptr ? 0 : bias_f32 ? 1 : 2;
  if (epi == 3) {
    launch<3, 0>(p, stream);
  } else if (epi == 2) {
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

void gemm_nt_conv(const void* x, const void* w, void* y, float* stats, int64_t nimg, int H, int W, int C,
                  int64_t Cout, int epi, hipStream_t stream, const void* residual) {
  const int64_t pixels = nimg * H * W;
  if (!gemm_nt_conv_supported(pixels, C, Cout))
    throw std::runtime_error("gemm_nt_conv: unsupported shape (pixels, Cout multiples of 256, C of 64; pixels=" +
                             std::to_string(pixels) + " C=" + std::to_string(C) + " Cout=" + std::to_string(Cout) + ")");
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) & 15u) != 0)
    throw std::runtime_error("gemm_nt_conv: operands must be 16-byte aligned");
  if (epi != 0 && epi != 3 && epi != 4)
    throw std::runtime_error("gemm_nt_conv: epilogue 0 (plain), 3 (statistics) or 4 (+ residual)");
  if (epi == 3 && stats == nullptr) throw std::runtime_error("gemm_nt_conv: the statistics epilogue needs the shards");
  if (epi == 4 && (residual == nullptr || (reinterpret_cast<uintptr_t>(residual) & 15u) != 0))
    throw std::runtime_error("gemm_nt_conv: the residual epilogue needs a 16-byte aligned residual");
  NTArgs p{};
  p.a = static_cast<const bf16*>(x), p.b = static_cast<const bf16*>(w), p.c = static_cast<bf16*>(y);
  p.stats = stats, p.lda = 9 * C, p.ldb = 9 * C, p.ldc = Cout, p.N = Cout;
  p.h = static_cast<const bf16*>(residual);  // EPI 4: the residual, laid out as y
  p.nk = 9 * C / kBK, p.tiles_m = static_cast<int>(pixels / kT), p.tiles_n = static_cast<int>(Cout / kT);
  p.gelu_tanh = 0;
  p.conv_h = H, p.conv_w = W, p.conv_c = C, p.conv_cpt = C / kBK;
  p.conv_inv_cpt = 1.f / static_cast<float>(C / kBK);
  p.a_bytes = static_cast<uint32_t>(pixels * C * 2);
  if (epi == 3) launch<3, 0, true>(p, stream);
  else if (epi == 4) launch<4, 0, true>(p, stream);
  else launch<0, 0, true>(p, stream);
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
