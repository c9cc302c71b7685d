// ResNet stem on MFMA: 7x7 / stride-2 / pad-3 convolution of a 224x224 NHWC image batch
// (input channels zero-padded 3 -> 4) with its BatchNorm statistics, and the WHOLE stem
// backward (max-pool gradient gather + BatchNorm backward + filter gradient) in one pass — gfx950.
//
// Before (r2m trace, bs 256): pad 42 us + MIOpen/CK conv 322 us + stats pass 103 us forward;
// pool gather 196 us + BN reduce 163 us + BN dx 225 us + MIOpen wrw 242 us backward.
//
// K layout. Output pixel (oy, ox) reads x[2oy + ky - 3][2ox + kx - 3]. Write ky - 3 = 2(ay - 2) + by,
// kx - 3 = 2(ax - 2) + bx (ay, ax in 0..3, by, bx in 0..1): the 8 bf16 at (ay, by, ax) for
// bx = 0..1, c = 0..3 are ONE 16-B chunk of the NHWC4 image (two adjacent pixels, 4 channels)
// at row 2oy + 2ay + by - 4, column 2(ox + ax) - 4. K = 32 chunks x 8 = 256 (the 7x7x3 = 147
// real taps plus zero filter entries: ky or kx = -1, and channel 3). Chunk order
// kc = (by * 4 + ax) * 4 + ay, so the four 8-element groups of one 32-deep MFMA step differ in ay
// only (two image rows apart); element e = bx * 4 + c. The packed filter W'[64][256] is built
// from the 7x7 filter on the host (fluxmpi_amd/ops/stem.py), rows in the channel order below.
//
// Forward (stem_fwd_kernel): a workgroup = 8 waves = 8 output rows of one image. It stages the
// packed filter (32 KiB) and the input "halo" (22 image rows x 120 chunks, zero chunks outside
// the image) in LDS with LDS-DMA, once; then each wave computes its 112 x 64 output row as
// 7 pixel tiles x 4 channel tiles of v_mfma_f32_16x16x32_bf16 (A = filter rows, B = pixels:
// both operands k-contiguous, plain ds_read_b128; a fragment's pixels are 16 consecutive
// chunks of one halo row, conflict-free). The im2col of the stem never exists: each image
// chunk is fetched from L2 about 1.4x (halo overlap) instead of 16x. Filter row R holds output
// channel 16 ((R >> 2) & 3) + 4 (R >> 4) + (R & 3), so a lane's 16 accumulators of one pixel
// are 16 CONSECUTIVE channels: two 16-B stores. The epilogue also reduces the per-channel
// sum / sum of squares of the (bf16-rounded) output into the BatchNorm workspace shards.
//
// Backward (stem_bwd_kernel): the gradient of the conv output is the BatchNorm backward of the
// max-pool gradient, dC = a*dz + b*x + d (per-channel a, b, d from sums over the whole batch),
// dz = the pool-gradient gather. So dW' = a*G1 + b*G2 + d*G3 with G1 = dz^T A, G2 = x^T A,
// G3 = column sums of A (A = the stem im2col): one pass over x, dz's inputs and the image
// computes G1, G2, G3 and the BN sums together; a combine kernel applies the coefficients.
// Persistent workgroups walk pairs of conv-output rows (224 pixels = 7 MFMA k-steps):
//   element phase: 512 lanes gather dz (<= 4 pooled windows, first-max index compare), round it
//     to bf16, accumulate sum(dz), sum(dz * xhat), write dz and x to two [224 px][64 ch] LDS
//     tiles (32-B groups XOR-swizzled by pixel bits); the image halo (10 rows) arrives by
//     LDS-DMA meanwhile;
//   MFMA phase: waves 0-3 accumulate G1, waves 4-7 G2, each a 64 x 64 slice of the 64 x 256
//     output; A = (dz or x)^T by ds_read_b64_tr_b16 (pixels along the lane's 8 k), B = the im2col
//     operand straight from the halo by transposed reads too (a lane's 8-B piece is one pixel's
//     4 channels; halo pitch 118 chunks keeps a 32-lane read on 64 distinct banks); G3 by
//     v_dot2c_f32_bf16 against ones on the B fragments.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {

void bn_finalize_bwd(float* ws, int64_t C, float* dw, float* db, hipStream_t s);  // batchnorm.hip

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4v;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void gl_void;

constexpr int kIH = 224, kIW = 224, kOH = 112, kOW = 112, kCo = 64, kKk = 256;
constexpr int kPH = 56, kPW = 56;  // 3x3 / 2 / pad-1 max-pool output
constexpr int kShards = 64;        // == batchnorm.hip

__device__ __attribute__((aligned(16))) uint4 g_stem_zero[4];

// s_waitcnt vmcnt(0) with expcnt / lgkmcnt left alone
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8)); }

// lane l's 16 B land at lds_base + 16 l (lds_base wave-uniform)
__device__ __forceinline__ void dma16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(lds_base), 16, 0, 0);
}

// ------------------------------------------------------------------------------ forward
constexpr int kFT = 512;                                   // 8 waves
constexpr int kFRows = 8;                                  // output rows per row group (one per wave)
constexpr int kFHaloRows = 2 * kFRows + 6;                 // image rows 2 oy0 - 4 .. 2 oy0 + 17
constexpr int kFPitch = 120;                               // chunks per halo row (2 pitch = 0 mod 16)
constexpr int kFHaloChunks = kFHaloRows * kFPitch;         // 2640
constexpr int kFHaloPerWave = (kFHaloChunks + kFT - 1) / kFT;  // 6 DMA instructions per wave per halo
constexpr int kFHaloBytes = kFHaloPerWave * kFT * 16;     // 49152 (slack chunks past 2640 unused)
constexpr int kWChunks = kCo * kKk / 8;                    // 2048
constexpr int kFSmem = kWChunks * 16 + 2 * kFHaloBytes;    // 131072 B: filter + two halo buffers

struct StemFwdArgs {
  const bf16* x;   // [N][224][224][4]
  const bf16* wp;  // [64][256] packed filter
  bf16* y;         // [N][112][112][64]
  float* stats;    // [kShards][2][64]
  int groups;      // N * 14 row groups
  int per_block;   // row groups per workgroup
};

// Persistent: one workgroup per CU stages the filter once, then walks its row groups with the
// NEXT group's halo in flight (LDS-DMA into the other buffer) while it computes the current one.
__global__ __launch_bounds__(kFT, 2) void stem_fwd_kernel(StemFwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sw = smem;  // filter: LDS chunk R * 32 + s = chunk s ^ (R & 15) of row R
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g0 = blockIdx.x * p.per_block;
  const int g1 = g0 + p.per_block < p.groups ? g0 + p.per_block : p.groups;
  // halo of row group gi into buffer buf: chunk hr * 120 + j = image row 2 oy0 - 4 + hr, pixels 2j - 4, 2j - 3
  auto issue_halo = [&](int gi, int buf) {
    const int img = gi / (kOH / kFRows);
    const int oy0 = (gi - img * (kOH / kFRows)) * kFRows;
    const bf16* ximg = p.x + static_cast<int64_t>(img) * kIH * kIW * 4;
    char* sh = smem + kWChunks * 16 + buf * kFHaloBytes;
#pragma unroll
    for (int i = 0; i < kFHaloPerWave; ++i) {
      const int t = i * (kFT / 64) + wave;
      const int L = t * 64 + lane;
      const int hr = L / kFPitch, j = L - hr * kFPitch;
      const int iy = 2 * oy0 - 4 + hr, px = 2 * j - 4;
      const void* src = g_stem_zero;
      if (L < kFHaloChunks && iy >= 0 && iy < kIH && px >= 0 && px < kIW) src = ximg + (iy * kIW + px) * 4;
      dma16(src, sh + t * 1024);
    }
  };
#pragma unroll
  for (int i = 0; i < kWChunks / 64 / 8; ++i) {
    const int base = (wave * (kWChunks / 64 / 8) + i) * 64;
    const int L = base + lane, R = L >> 5, s = L & 31;
    dma16(p.wp + R * kKk + (s ^ (R & 15)) * 8, sw + base * 16);
  }
  if (g0 < g1) issue_halo(g0, 0);

  const int g = lane >> 4, li = lane & 15;
  // A fragment (filter rows 16t + li, chunk kc = 4 kh + g): slot kc ^ li
  const char* arow = sw + li * (kKk * 2);
  float cs[16], cq[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) cs[e] = cq[e] = 0.f;
  for (int gi = g0; gi < g1; ++gi) {
    const int buf = (gi - g0) & 1;
    if (gi + 1 < g1) {
      issue_halo(gi + 1, buf ^ 1);  // that buffer's last readers finished before the previous barrier
      __builtin_amdgcn_s_waitcnt((kFHaloPerWave & 15) | ((kFHaloPerWave >> 4) << 14) | (7 << 4) | (15 << 8));
    } else {
      wait_vm0();
    }
    __builtin_amdgcn_s_barrier();  // every wave's pieces of this group's halo (and the filter) landed
    const int img = gi / (kOH / kFRows);
    const int oy = (gi - img * (kOH / kFRows)) * kFRows + wave;
    // B fragment (pixels 16 pt + li, chunk (ay = g, by, ax)): halo row 2 wave + 2g + by, chunk ox + ax
    const char* brow = smem + kWChunks * 16 + buf * kFHaloBytes + ((2 * wave + 2 * g) * kFPitch + li) * 16;
    f32x4 acc[7][4];
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int kh = 0; kh < 8; ++kh) {
      const int by = kh >> 2, ax = kh & 3;
      const int slot = (4 * kh + g) ^ li;
      bf16x8 a[4], b[7];
#pragma unroll
      for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const bf16x8*>(arow + t * 16 * (kKk * 2) + slot * 16);
#pragma unroll
      for (int pt = 0; pt < 7; ++pt)
        b[pt] = *reinterpret_cast<const bf16x8*>(brow + (by * kFPitch + 16 * pt + ax) * 16);
#pragma unroll
      for (int pt = 0; pt < 7; ++pt)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[pt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t], b[pt], acc[pt][t], 0, 0, 0);
    }
    // lane (g, li) holds channels 16g .. 16g + 15 of pixel 16 pt + li: two 16-B stores per tile
    bf16* yrow = p.y + (static_cast<int64_t>(img) * kOH + oy) * kOW * kCo;
#pragma unroll
    for (int pt = 0; pt < 7; ++pt) {
      bf16 v[16];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[4 * t + r] = static_cast<bf16>(acc[pt][t][r]);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float f = static_cast<float>(v[e]);
        cs[e] += f;
        cq[e] = fmaf(f, f, cq[e]);
      }
      uint4 w[2];
      __builtin_memcpy(w, v, 32);
      uint4* dst = reinterpret_cast<uint4*>(yrow + (16 * pt + li) * kCo + 16 * g);
      dst[0] = w[0];
      dst[1] = w[1];
    }
    __builtin_amdgcn_s_barrier();  // this buffer is refilled two groups on
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {  // 16-lane row sums by DPP (common.h)
    cs[e] = row_sum16(cs[e]);
    cq[e] = row_sum16(cq[e]);
  }
  wait_vm0();
  __syncthreads();  // every wave is done with the filter / halo: reuse the LDS
  float* red = reinterpret_cast<float*>(smem);  // [8 waves][2][64]
  if (li == 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      red[(wave * 2 + 0) * kCo + 16 * g + e] = cs[e];
      red[(wave * 2 + 1) * kCo + 16 * g + e] = cq[e];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * kCo) {
    const int which = threadIdx.x >> 6, c = threadIdx.x & 63;
    float s = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < kFT / 64; ++w2) s += red[(w2 * 2 + which) * kCo + c];
    atomicAdd(p.stats + static_cast<size_t>(blockIdx.x % kShards) * 2 * kCo + which * kCo + c, s);
  }
}

// ------------------------------------------------------------------------------ backward
constexpr int kBT = 512;
constexpr int kBPix = 2 * kOW;                             // 224 conv-output pixels per iteration
constexpr int kBHaloRows = 10;                             // image rows 2 h0 - 4 .. 2 h0 + 5
constexpr int kBPitch = 118;                               // 2 * 1888 B = 64 mod 128
constexpr int kBHaloChunks = kBHaloRows * kBPitch;         // 1180
constexpr int kBHaloPer = (kBHaloChunks + kBT - 1) / kBT;  // 3 DMA instructions per wave
constexpr int kBHaloBytes = kBHaloPer * kBT * 16;          // 24576 (slack past 1180 chunks unused)
constexpr int kPoolDpBytes = 2 * kPW * kCo * 2;            // pooled rows h0/2, h0/2 + 1: gradient 14336 B
constexpr int kPoolIxBytes = 2 * kPW * kCo;                // ... and window indices 7168 B
constexpr int kPoolChunks = (kPoolDpBytes + kPoolIxBytes) / 16;  // 1344
constexpr int kPoolPer = (kPoolChunks + kBT - 1) / kBT;    // 3
constexpr int kPoolBytes = kPoolPer * kBT * 16;            // 24576
constexpr int kStageBytes = kBHaloBytes + kPoolBytes;      // one iteration's DMA'd inputs
constexpr int kTileBytes = kBPix * kCo * 2;                // 28672
constexpr int kBSmemMain = 2 * kTileBytes + 2 * kStageBytes;  // 155648 B: two input stages
constexpr int kBSmem = kBSmemMain + 3 * kCo * 4;           // + mean / inv / -mean * inv
constexpr int kBDma = kBHaloPer + kPoolPer;                // DMA instructions per wave per stage
constexpr int kPart = 2 * kKk * kCo + kKk;                 // G1 [256][64], G2 [256][64], G3 [256]

struct StemBwdArgs {
  const bf16* x;        // padded image [N][224][224][4]
  const bf16* c;        // conv output = BatchNorm input [N][112][112][64]
  const bf16* dp;       // max-pool output gradient [N][56][56][64]
  const uint8_t* idx;   // window index of the max (0xFF: blocked by the ReLU) [N][56][56][64]
  const float* mean;    // BatchNorm batch mean / inverse std [64]
  const float* inv;
  float* part;          // [gridDim.x][kPart]
  float* stats;         // BN backward sums: [kShards][2][64] (sum dz, sum dz * xhat)
  int iters_per_block;  // row pairs per workgroup
  int total_iters;      // N * 56
};

// __restrict__: gives the transposed reads alias scopes; without them the waitcnt pass assumes they
// may read the LDS-DMA just issued into the other stage and drains vmcnt(0) before them
__device__ __forceinline__ bf16x8 tr_frag(const char* __restrict__ lo, const char* __restrict__ hi) {
  const short4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(lo));
  const short4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(hi));
  bf16x8 out;
  __builtin_memcpy(&out, &a, 8);
  __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &b, 8);
  return out;
}

// byte offset of (pixel P, 16-B chunk q) in a [224][64] bf16 tile: the 32-B group is XORed with
// bits 1 and 3 of P, so a transposed read's 32 lanes (pixels 8g + q, g in 0..1, 8-B pieces of a
// 16-channel group) land on 32 distinct 8-B bank slots; the swizzle is invariant under P += 32
// and P += 4 (the k-steps and the second half of a fragment)
__device__ __forceinline__ int tile_off(int P, int q) {
  return P * 128 + ((q ^ ((((P >> 1) & 1) | (((P >> 3) & 1) << 1)) << 1)) << 4);
}

// Element-phase item of pass r for a wave: 28 groups of 8 pixels (conv-output row of the pair,
// column parity, 8 consecutive pooled columns) over the 32 (pass, wave) slots, so row and
// parity — hence the set of pooled windows to visit — are wave-uniform.
struct Item {
  bool on;   // wave-uniform
  int row;   // 0 / 1: conv row h0 + row (wave-uniform)
  int par;   // column parity (wave-uniform)
  int m;     // pooled column ox >> 1
  int pix;   // pixel within the pair: row * 112 + ox
};
__device__ __forceinline__ Item item_of(int r, int wave, int slot) {
  const int G = r * (kBT / 64) + wave;
  Item it;
  it.on = G < 28;
  const int rem = G % 14;
  it.row = G / 14;
  it.par = rem / 7;
  it.m = 8 * (rem % 7) + slot;
  it.pix = it.row * kOW + 2 * it.m + it.par;
  return it;
}

// Pipelined: while the MFMA phase of row pair `it` runs, the DMA of row pair it + 1's image
// halo and pooled-gradient rows (into the other stage) and this lane's conv-output loads for
// it + 1 (registers) are in flight. One workgroup per CU (LDS: two stages + the dz / x tiles).
// MODE (round-3 bottleneck experiments, rebuilt by hand): 0 = normal, 1 = no MFMA phase,
// 2 = no element-phase gather (dz = 0), 3 = no next-iteration loads (stale stages)
template <int MODE>
__global__ __launch_bounds__(kBT, 2) void stem_bwd_kernel(StemBwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* tdz = smem;
  char* tx = smem + kTileBytes;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, pp = li & 3;
  const int cg = lane & 7, slot = lane >> 3;  // element phase: channel group, pixel slot
  float* smi = reinterpret_cast<float*>(smem + kBSmemMain);  // [64] mean, [64] inv std, [64] -mean * inv
  if (threadIdx.x < kCo) {
    const float m = p.mean[threadIdx.x], v = p.inv[threadIdx.x];
    smi[threadIdx.x] = m;
    smi[kCo + threadIdx.x] = v;
    smi[2 * kCo + threadIdx.x] = -m * v;
  }
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  // MFMA phase: waves 0-3 -> G1 (dz), 4-7 -> G2 (x); n tiles 4 wn .. 4 wn + 3
  const bool gx = wave >= 4;
  const int wn = wave & 3;
  f32x4 acc[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float g3[4] = {0.f, 0.f, 0.f, 0.f};
  // fragment addresses at k-step 0 (lo rows P0 = 8g + q4; hi rows + 4): A = tile + ks * 4096;
  // B (n tile): + ks * 512, + 1984 once the pixel is in the pair's second conv row
  const int P0 = 8 * g + q4;
  int a_lo[4];  // channel group t: chunk 2t + (pp >> 1) of the swizzled row (the XOR does not distribute over + 32t)
#pragma unroll
  for (int t = 0; t < 4; ++t)
    a_lo[t] = static_cast<int>((gx ? tx : tdz) - smem) + tile_off(P0, 2 * t + (pp >> 1)) + (pp & 1) * 8;
  int b_lo[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int kc = 2 * (4 * wn + n) + (pp >> 1);
    const int ay = kc & 3, ax = (kc >> 2) & 3, by = kc >> 4;
    b_lo[n] = (2 * ay + by) * (kBPitch * 16) + ax * 16 + (pp & 1) * 8 + P0 * 16;
  }
  const bf16x2 ones = {static_cast<bf16>(1.f), static_cast<bf16>(1.f)};

  // DMA pieces of this lane, fixed over the iterations. Halo chunk L = hr * 118 + j (image row
  // 2 h0 - 4 + hr, pixels 2j - 4, 2j - 3): element offset from the row-pair base, its row hr, and
  // whether the columns are inside the image. Pool stage chunk L: gradient rows (bf16) then index
  // rows (u8) of pooled rows h0/2, h0/2 + 1.
  int h_off[kBHaloPer], h_row[kBHaloPer];
#pragma unroll
  for (int i = 0; i < kBHaloPer; ++i) {
    const int L = (i * (kBT / 64) + wave) * 64 + lane;
    const int hr = L / kBPitch, j = L - hr * kBPitch;
    const bool ok = L < kBHaloChunks && j >= 2 && j <= kIW / 2 + 1;
    h_off[i] = hr * kIW * 4 + (2 * j - 4) * 4;
    h_row[i] = ok ? hr : -1000;
  }
  int q_off[kPoolPer], q_row[kPoolPer];  // q_row: pooled row offset (0 / 1), + 2 for index rows; -1000: none
#pragma unroll
  for (int i = 0; i < kPoolPer; ++i) {
    const int L = (i * (kBT / 64) + wave) * 64 + lane;
    if (L < kPoolDpBytes / 16) {
      q_row[i] = L / (kPW * kCo / 8);
      q_off[i] = L * 16;
    } else if (L < kPoolChunks) {
      const int Li = L - kPoolDpBytes / 16;
      q_row[i] = 2 + Li / (kPW * kCo / 16);
      q_off[i] = Li * 16;
    } else {
      q_row[i] = -1000;
      q_off[i] = 0;
    }
  }
  auto issue = [&](int it, int st) {
    const int img = it / kPH;
    const int h0 = (it - img * kPH) * 2;
    char* sh = smem + 2 * kTileBytes + st * kStageBytes;
    const bf16* hbase = p.x + (static_cast<int64_t>(img) * kIH + 2 * h0 - 4) * kIW * 4;
#pragma unroll
    for (int i = 0; i < kBHaloPer; ++i) {
      const bool ok = static_cast<unsigned>(2 * h0 - 4 + h_row[i]) < static_cast<unsigned>(kIH);
      const void* src = ok ? static_cast<const void*>(hbase + h_off[i]) : static_cast<const void*>(g_stem_zero);
      dma16(src, sh + (i * (kBT / 64) + wave) * 1024);
    }
    const int prow = h0 >> 1;
    const int64_t pimg = (static_cast<int64_t>(img) * kPH + prow) * kPW * kCo;
    const char* dpb = reinterpret_cast<const char*>(p.dp + pimg);
    const char* ixb = reinterpret_cast<const char*>(p.idx + pimg);
#pragma unroll
    for (int i = 0; i < kPoolPer; ++i) {
      const int r = q_row[i] & 1;
      const bool ok = q_row[i] >= 0 && prow + r < kPH;
      const char* base = q_row[i] >= 2 ? ixb : dpb;
      const void* src = ok ? static_cast<const void*>(base + q_off[i]) : static_cast<const void*>(g_stem_zero);
      dma16(src, sh + kBHaloBytes + (i * (kBT / 64) + wave) * 1024);
    }
  };
  // conv-output loads of this lane's items of row pair it
  auto load_x = [&](int it, uint4 (&xr)[4]) {
    const int img = it / kPH;
    const int h0 = (it - img * kPH) * 2;
    const bf16* cb = p.c + (static_cast<int64_t>(img) * kOH + h0) * kOW * kCo + cg * 8;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // unconditional load (an idle item re-reads pixel 0): a branch around it made the compiler
      // wait for every load (and every older LDS-DMA) right after issuing it
      const Item im = item_of(r, wave, slot);
      xr[r] = *reinterpret_cast<const uint4*>(cb + (im.on ? im.pix : 0) * kCo);
    }
  };

  const int it0 = blockIdx.x * p.iters_per_block;
  const int it1 = it0 + p.iters_per_block < p.total_iters ? it0 + p.iters_per_block : p.total_iters;
  uint4 xr[4];
  if (it0 < it1) {
    issue(it0, 0);
    load_x(it0, xr);
  }
  for (int it = it0; it < it1; ++it) {
    const int st = (it - it0) & 1;
    const int h0 = (it - (it / kPH) * kPH) * 2;
    wait_vm0();
    __syncthreads();  // stage st landed for every wave; the tiles' last readers (MFMA it - 1) are done
    const int sbase = 2 * kTileBytes + st * kStageBytes;
    const char* spd = smem + sbase + kBHaloBytes;  // pooled gradient [2][56][64] bf16
    const char* spi = spd + kPoolDpBytes;          // window index [2][56][64] u8
    const bool second_prow = (h0 >> 1) + 1 < kPH;
    // ---- element phase: dz (pool gradient gather from LDS) and x into the tiles, BN sums
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const Item im = item_of(r, wave, slot);
      if (im.on) {
        // windows covering (h0 + row, ox): pooled row 0 of the stage (+ row 1 for the odd conv
        // row), column m (+ m + 1 for an odd column); the window index of the pixel in each
        const int kya = im.row ? 2 : 1, kxa = im.par ? 2 : 1;
        const bool two_w = im.par && im.m + 1 < kPW;
        const bool two_h = im.row && second_prow;
        const int e00 = im.m * kCo + cg * 8;
        float dz[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        auto visit = [&](int e0, int kk) {
          const uint4 dv = *reinterpret_cast<const uint4*>(spd + e0 * 2);
          const uint2 iv2 = *reinterpret_cast<const uint2*>(spi + e0);
          bf16 d8[8];
          uint8_t a8[8];
          __builtin_memcpy(d8, &dv, 16);
          __builtin_memcpy(a8, &iv2, 8);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (static_cast<int>(a8[e]) == kk) dz[e] += static_cast<float>(d8[e]);
        };
        if (MODE != 2) visit(e00, kya * 3 + kxa);
        if (MODE != 2 && im.par) {
          if (two_w) visit(e00 + kCo, kya * 3);
        }
        if (MODE != 2 && two_h) {
          visit(e00 + kPW * kCo, kxa);
          if (im.par && two_w) visit(e00 + kPW * kCo + kCo, 0);
        }
        bf16 x8[8], z8[8];
        __builtin_memcpy(x8, &xr[r], 16);
        float iv[8], nm[8];  // xhat = x * inv + (-mean * inv)
        __builtin_memcpy(iv, smi + kCo + cg * 8, 32);
        __builtin_memcpy(nm, smi + 2 * kCo + cg * 8, 32);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          z8[e] = static_cast<bf16>(dz[e]);
          // BN sums from the fp32 gather (the tiles get the bf16 dz); the rounding of one pool
          // gradient per element is below the sums' own fp32 noise
          s1[e] += dz[e];
          s2[e] = fmaf(dz[e], fmaf(static_cast<float>(x8[e]), iv[e], nm[e]), s2[e]);
        }
        uint4 zv;
        __builtin_memcpy(&zv, z8, 16);
        const int o = tile_off(im.pix, cg);
        *reinterpret_cast<uint4*>(tdz + o) = zv;
        *reinterpret_cast<uint4*>(tx + o) = xr[r];
      }
    }
    // next row pair's inputs: its stage was last read before this iteration's barrier
    if (MODE != 3 && it + 1 < it1) {
      issue(it + 1, st ^ 1);
      load_x(it + 1, xr);
    }
    // tiles written: LDS writes drained (lgkmcnt) and a raw barrier — __syncthreads()' fence would
    // also drain the next row pair's loads just issued (vmcnt) and serialize them with the MFMAs
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    // ---- MFMA phase: 7 k-steps of 32 pixels
    const char* sb = smem + sbase;
#pragma unroll
    for (int ks = 0; ks < (MODE == 1 ? 0 : kBPix / 32); ++ks) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) fa[t] = tr_frag(smem + a_lo[t] + ks * 4096, smem + a_lo[t] + ks * 4096 + 512);
      // pixel P0 + 32 ks in the second conv row of the pair: always from k-step 4, from 3 for g >= 2
      const int rowoff = ks >= 4 ? 1984 : (ks == 3 && g >= 2 ? 1984 : 0);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const char* lo = sb + b_lo[n] + ks * 512 + rowoff;
        fb[n] = tr_frag(lo, lo + 64);
      }
      if (gx == static_cast<bool>(ks & 1)) {  // column sums of the im2col operand, split over the two groups
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          bf16x2 h2[4];
          __builtin_memcpy(h2, &fb[n], 16);
#pragma unroll
          for (int j = 0; j < 4; ++j) g3[n] = __builtin_amdgcn_fdot2_f32_bf16(h2[j], ones, g3[n], false);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t], fb[n], acc[t][n], 0, 0, 0);
    }
  }
  wait_vm0();
  __syncthreads();  // LDS reused below

  // ---- partials: G[k][c] (k = 16 nt + li, c = 16 t + 4 g + r), G3[k]
  float* part = p.part + static_cast<size_t>(blockIdx.x) * kPart;
  float* gp = part + (gx ? kKk * kCo : 0);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int k = 16 * (4 * wn + n) + li;
      *reinterpret_cast<f32x4*>(gp + k * kCo + 16 * t + 4 * g) = acc[t][n];
    }
  // G3: both wave groups hold partial column sums of their 4 n tiles (the other half of the k-steps)
#pragma unroll
  for (int n = 0; n < 4; ++n) g3[n] = butterfly_from<16>(g3[n]);
  float* red3 = reinterpret_cast<float*>(smem) + 2 * (kBT / 64) * kCo;  // [256]
  if (gx && g == 0) {
#pragma unroll
    for (int n = 0; n < 4; ++n) red3[16 * (4 * wn + n) + li] = g3[n];
  }
  // ---- BatchNorm backward sums: lanes with equal lane & 7 share channels
#pragma unroll
  for (int e = 0; e < 8; ++e) {  // LDS-free cross-lane butterflies (common.h)
    s1[e] = butterfly_from<8>(s1[e]);
    s2[e] = butterfly_from<8>(s2[e]);
  }
  float* red = reinterpret_cast<float*>(smem);  // [8 waves][2][64]
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(wave * 2 + 0) * kCo + lane * 8 + e] = s1[e];
      red[(wave * 2 + 1) * kCo + lane * 8 + e] = s2[e];
    }
  }
  __syncthreads();
  if (!gx && g == 0) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int k = 16 * (4 * wn + n) + li;
      part[2 * kKk * kCo + k] = g3[n] + red3[k];
    }
  }
  if (threadIdx.x < 2 * kCo) {
    const int which = threadIdx.x >> 6, c = threadIdx.x & 63;
    float s = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < kBT / 64; ++w2) s += red[(w2 * 2 + which) * kCo + c];
    atomicAdd(p.stats + static_cast<size_t>(blockIdx.x % kShards) * 2 * kCo + which * kCo + c, s);
  }
}

// dW'[c][k] = a_c G1[k][c] + b_c G2[k][c] + d_c G3[k] summed over the partials: one workgroup per k,
// 4 groups of 64 lanes (channels) split the partials, LDS sum. a, b, d as in bn_bwd_dx_kernel.
constexpr int kCT = 256;
__global__ __launch_bounds__(kCT) void stem_wgrad_combine_kernel(const float* __restrict__ part, int blocks,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ inv,
                                                                 const float* __restrict__ sdzx,
                                                                 const float* __restrict__ sdz, float inv_n,
                                                                 float* __restrict__ out) {
  __shared__ float red[3][kCT];
  const int k = blockIdx.x, c = threadIdx.x & 63, grp = threadIdx.x >> 6;
  float a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 4
  for (int b = grp; b < blocks; b += kCT / 64) {
    const float* pb = part + static_cast<size_t>(b) * kPart;
    a1 += pb[k * kCo + c];
    a2 += pb[kKk * kCo + k * kCo + c];
    a3 += pb[2 * kKk * kCo + k];
  }
  red[0][threadIdx.x] = a1;
  red[1][threadIdx.x] = a2;
  red[2][threadIdx.x] = a3;
  __syncthreads();
  if (grp != 0) return;
  const float g1 = red[0][c] + red[0][c + 64] + red[0][c + 128] + red[0][c + 192];
  const float g2 = red[1][c] + red[1][c + 64] + red[1][c + 128] + red[1][c + 192];
  const float g3 = red[2][c] + red[2][c + 64] + red[2][c + 128] + red[2][c + 192];
  const float iv = inv[c], m = mean[c];
  const float sc = (w ? w[c] : 1.f) * iv;
  const float k2 = sdz[c] * inv_n, k3 = sdzx[c] * inv_n;
  const float cb = -sc * iv * k3, cd = sc * (m * iv * k3 - k2);
  out[c * kKk + k] = fmaf(sc, g1, fmaf(cb, g2, cd * g3));
}

void check_ptr(const void* ptr, const char* what) {
  if (ptr == nullptr || reinterpret_cast<uintptr_t>(ptr) % 16 != 0)
    throw std::runtime_error(std::string("stem: ") + what + " must be a non-null 16-byte aligned pointer");
}

}  // namespace

namespace {
void set_lds_attrs() {
  static bool done = false;
  if (done) return;
  FLUXMPI_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_fwd_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kFSmem));
  for (const void* k : {reinterpret_cast<const void*>(&stem_bwd_kernel<0>), reinterpret_cast<const void*>(&stem_bwd_kernel<1>),
                        reinterpret_cast<const void*>(&stem_bwd_kernel<2>), reinterpret_cast<const void*>(&stem_bwd_kernel<3>)})
    FLUXMPI_HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kBSmem));
  done = true;
}
}  // namespace

int stem_bwd_blocks(int64_t n) {
  static int b = [] {
    set_lds_attrs();
    const int r = resident_blocks(reinterpret_cast<const void*>(&stem_bwd_kernel<0>), kBT, kBSmem);
    return r > 0 ? r : 512;
  }();
  const int64_t iters = n * kPH;
  return static_cast<int>(iters < b ? iters : b);
}

int64_t stem_part_floats() { return kPart; }

void stem_fwd(const void* x, const void* wp, void* y, float* stats, int64_t n, hipStream_t s) {
  check_ptr(x, "x");
  check_ptr(wp, "packed filter");
  check_ptr(y, "y");
  check_ptr(stats, "stats");
  if (n < 1 || n * kOH * kOW * kCo >= (int64_t(1) << 40)) throw std::runtime_error("stem_fwd: bad batch");
  set_lds_attrs();
  const int groups = static_cast<int>(n * (kOH / kFRows));
  static int resident = [] { return resident_blocks(reinterpret_cast<const void*>(&stem_fwd_kernel), kFT, kFSmem); }();
  const int blocks = groups < resident ? groups : resident;
  const int per = (groups + blocks - 1) / blocks;
  StemFwdArgs a{static_cast<const bf16*>(x), static_cast<const bf16*>(wp), static_cast<bf16*>(y), stats, groups, per};
  stem_fwd_kernel<<<static_cast<unsigned>((groups + per - 1) / per), kFT, kFSmem, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void stem_bwd(const void* x, const void* c, const void* dp, const uint8_t* idx, const float* w, const float* mean,
              const float* inv, float* part, int blocks, float* stats, float* dw_bn, float* db_bn, float* dwp,
              int64_t n, hipStream_t s) {
  check_ptr(x, "x");
  check_ptr(c, "conv output");
  check_ptr(dp, "pooled gradient");
  check_ptr(idx, "pool index");
  check_ptr(part, "partials");
  if (n < 1 || blocks < 1 || blocks > stem_bwd_blocks(n)) throw std::runtime_error("stem_bwd: bad batch / grid");
  set_lds_attrs();
  // FLUXMPI_STEM_BWD_DIAG=1/2/3: the MODE builds (time split of the phases; results are wrong)
  static const int mode = [] {
    const char* e = std::getenv("FLUXMPI_STEM_BWD_DIAG");
    const int v = e != nullptr ? std::atoi(e) : 0;
    return v >= 0 && v <= 3 ? v : 0;
  }();
  const int total = static_cast<int>(n * kPH);
  StemBwdArgs a{static_cast<const bf16*>(x), static_cast<const bf16*>(c), static_cast<const bf16*>(dp), idx, mean, inv,
                part, stats, (total + blocks - 1) / blocks, total};
  auto kern = mode == 1 ? stem_bwd_kernel<1> : mode == 2 ? stem_bwd_kernel<2> : mode == 3 ? stem_bwd_kernel<3> : stem_bwd_kernel<0>;
  kern<<<static_cast<unsigned>(blocks), kBT, kBSmem, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  bn_finalize_bwd(stats, kCo, dw_bn, db_bn, s);
  stem_wgrad_combine_kernel<<<kKk, kCT, 0, s>>>(part, blocks, w, mean, inv, dw_bn, db_bn,
                                               1.f / static_cast<float>(n * kOH * kOW), dwp);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
