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
  int iters_per_block;  // row pairs (pair kernel) / rows (wave-specialised kernel) per workgroup
  int total_iters;      // N * 56 / N * 112
  int nimg;             // N
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

// ------------------------------------------------------- backward, wave-specialised (one row per phase)
// OPT-IN (FLUXMPI_STEM_BWD=ws), measured slower than the pair kernel: see stem_bwd_ws() below.
// The same sums with the two phases on DIFFERENT waves of one 16-wave workgroup per CU, so they run
// concurrently (the pair kernel above runs them one after the other behind barriers; phase split
// in profiles/rd6h_stem_bwd_split.jsonl: MFMA ~111 us, element work ~213 of 324). Phase q:
//   waves 8-15 (element role): pool-gradient gather of conv row q from pool stage q & 1 (+ the
//     conv-output registers loaded during phase q - 1), BN sums, dz / x tiles into tile buffer
//     q & 1; then row q + 1's conv-output loads;
//   waves 0-7 (MFMA role): LDS-DMA of row q + 1's pooled gradient into pool stage (q + 1) & 1,
//     then row q - 1's 4 k-steps from tile buffer (q - 1) & 1 and halo buffer (q - 1) & 1; before
//     the next phase's first barrier they wait for their DMA and issue row q + 1's image halo into
//     halo buffer (q + 1) & 1 (its last reader was row q - 1's MFMA work, finished by then).
// Only the MFMA waves issue LDS-DMA: their fragment reads carry alias scopes (tr_frag), and the
// element waves' gather never has a DMA of its own in flight (the waitcnt pass would drain it before
// every LDS read). Two barriers per phase, executed by all 16 waves: B1 (the stages a phase reads
// are complete) and B2 (this phase's tiles written, its MFMA reads done). Rows are 112 pixels padded
// to 128 (4 k-steps): the padded rows of the tiles are zero (written once), their halo reads land
// in zero slack, G3 skips them. 16 waves per CU: each role's registers fit in 128.
constexpr int kWT = 1024;
constexpr int kWPix = 128;
constexpr int kWTile = kWPix * kCo * 2;                     // 16384: one operand tile of one row
constexpr int kWHaloRows = 8;                               // image rows 2 oy - 4 .. 2 oy + 3
constexpr int kWHaloChunks = kWHaloRows * kBPitch;          // 944
constexpr int kWHaloPer = 2;                                // DMA instructions per MFMA wave (1024 slots)
constexpr int kWHalo = kWHaloPer * 512 * 16;                // 16384 (chunks 944.. zero slack)
constexpr int kWPoolPer = 3;                                // 1536 slots >= kPoolChunks
constexpr int kWPool = kWPoolPer * 512 * 16;                // 24576
constexpr int kWTilesOff = 0;                               // [2 buffers][dz, x][kWTile]
constexpr int kWHaloOff = 4 * kWTile;                       // [2 buffers][kWHalo]
constexpr int kWPoolOff = kWHaloOff + 2 * kWHalo;           // [2 buffers][kWPool]
constexpr int kWSmiOff = kWPoolOff + 2 * kWPool;
constexpr int kWRedOff = kWSmiOff + 3 * kCo * 4;            // element role's BN sums [8][2][64]
constexpr int kWSmem = kWRedOff + 8 * 2 * kCo * 4;          // 152320
static_assert(kWHaloChunks <= kWHaloPer * 512 && kPoolChunks <= kWPoolPer * 512, "staging slots");
static_assert((7 * kBPitch + (kWPix - 1) + 3) * 16 + 16 <= kWHalo, "halo slack covers the padded pixels");
static_assert(kWSmem <= 160 * 1024, "LDS");

__global__ __launch_bounds__(kWT) void stem_bwd_ws_kernel(StemBwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  float* smi = reinterpret_cast<float*>(smem + kWSmiOff);
  float* sred = reinterpret_cast<float*>(smem + kWRedOff);  // [8][2][64]
  if (threadIdx.x < kCo) {
    const float m = p.mean[threadIdx.x], v = p.inv[threadIdx.x];
    smi[threadIdx.x] = m;
    smi[kCo + threadIdx.x] = v;
    smi[2 * kCo + threadIdx.x] = -m * v;
  }
  if (threadIdx.x < 512) {  // padded pixels 112..127 of the 4 tiles, once
    const int t = threadIdx.x >> 7, P = 112 + ((threadIdx.x >> 3) & 15), q = threadIdx.x & 7;
    *reinterpret_cast<uint4*>(smem + kWTilesOff + t * kWTile + tile_off(P, q)) = uint4{0, 0, 0, 0};
  } else if (threadIdx.x < 512 + 8 * 2 * kCo / 4) {
    reinterpret_cast<float4*>(sred)[threadIdx.x - 512] = float4{0.f, 0.f, 0.f, 0.f};
  }
  const int it0 = blockIdx.x * p.iters_per_block;
  const int it1 = it0 + p.iters_per_block < p.total_iters ? it0 + p.iters_per_block : p.total_iters;
  const int n = it1 > it0 ? it1 - it0 : 0;

  if (wave >= 8) {
    // ================================================================ element role
    const int ew = wave - 8;
    const int cg = lane & 7, slot = lane >> 3;
    auto item = [&](int r, bool& on, int& par, int& m) {
      const int G = r * 8 + ew;
      on = G < 14;
      par = G / 7;
      m = 8 * (G - 7 * par) + slot;
    };
    // unconditional loads from a valid address (a branch around a load waits for it at the join)
    auto load_x = [&](int it, uint4 (&xr)[2]) {
      const int img = it / kOH, oy = it - img * kOH;
      const bf16* cb = p.c + (static_cast<int64_t>(img) * kOH + oy) * kOW * kCo + cg * 8;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        bool on;
        int par, m;
        item(r, on, par, m);
        xr[r] = *reinterpret_cast<const uint4*>(cb + (on ? 2 * m + par : 0) * kCo);
      }
    };
    uint4 xr[2];
    if (n > 0) load_x(it0, xr);
    __syncthreads();  // A: smi, zero rows, sred; row 0's stages (issued by the MFMA role)
    for (int ph = 0; ph <= n; ++ph) {
      __builtin_amdgcn_s_barrier();  // B1
      if (ph < n) {
        const int oy = (it0 + ph) % kOH;
        const bool odd = oy & 1;
        const bool second_prow = (oy >> 1) + 1 < kPH;
        const int kya = odd ? 2 : 1;
        const char* spd = smem + kWPoolOff + (ph & 1) * kWPool;  // pooled gradient [2][56][64] bf16
        const char* spi = spd + kPoolDpBytes;                      // window index [2][56][64] u8
        char* tdz = smem + kWTilesOff + (ph & 1) * 2 * kWTile;
        char* tx = tdz + kWTile;
        float s1[8], sx[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) s1[e] = sx[e] = 0.f;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          bool on;
          int par, m;
          item(r, on, par, m);
          if (on) {
            const int kxa = par ? 2 : 1;
            const bool two_w = par && m + 1 < kPW;
            const bool two_h = odd && second_prow;
            const int e00 = m * kCo + cg * 8;
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
            visit(e00, kya * 3 + kxa);
            if (two_w) visit(e00 + kCo, kya * 3);
            if (two_h) {
              visit(e00 + kPW * kCo, kxa);
              if (two_w) visit(e00 + kPW * kCo + kCo, 0);
            }
            bf16 x8[8], z8[8];
            __builtin_memcpy(x8, &xr[r], 16);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              z8[e] = static_cast<bf16>(dz[e]);
              s1[e] += dz[e];
              sx[e] = fmaf(dz[e], static_cast<float>(x8[e]), sx[e]);
            }
            uint4 zv;
            __builtin_memcpy(&zv, z8, 16);
            const int o = tile_off(2 * m + par, cg);
            *reinterpret_cast<uint4*>(tdz + o) = zv;
            *reinterpret_cast<uint4*>(tx + o) = xr[r];
          }
        }
        if (ph + 1 < n) load_x(it0 + ph + 1, xr);
        // BN sums per (element wave, channel), flushed once per row: sum(dz) and
        // sum(dz * xhat) = inv * sum(dz * x) + (-mean * inv) * sum(dz) over the row's items
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[e] = butterfly_from<8>(s1[e]);
          sx[e] = butterfly_from<8>(sx[e]);
        }
        if (lane < 8) {
          float iv[8], nm[8];
          __builtin_memcpy(iv, smi + kCo + lane * 8, 32);
          __builtin_memcpy(nm, smi + 2 * kCo + lane * 8, 32);
          float* r0 = sred + (ew * 2) * kCo + lane * 8;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            r0[e] += s1[e];
            r0[kCo + e] += fmaf(iv[e], sx[e], nm[e] * s1[e]);
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): tile writes done; conv-output loads in flight
      __builtin_amdgcn_s_barrier();         // B2
    }
    wait_vm0();
    __syncthreads();  // E
    __syncthreads();  // F
    if (threadIdx.x - 512 < 2 * kCo) {
      const int t = threadIdx.x - 512, which = t >> 6, c = t & 63;
      float s = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 8; ++w2) s += sred[(w2 * 2 + which) * kCo + c];
      atomicAdd(p.stats + static_cast<size_t>(blockIdx.x % kShards) * 2 * kCo + which * kCo + c, s);
    }
  } else {
    // ================================================================ MFMA role (+ the stage DMA)
    // DMA pieces of this lane: slot L = (i * 8 + wave) * 64 + lane of a stage
    // Stage DMA through buffer resources: wave-uniform bases in SGPRs, one 32-bit lane offset per
    // piece, and out-of-range offsets (padding pixels, rows outside the image, unused slots, the
    // pooled row past the last image) read as zeros — few VGPRs in this role's loop (128 budget).
    auto issue_pool = [&](int it, int buf) {
      const int img = it / kOH, oy = it - img * kOH;
      const int64_t pimg = (static_cast<int64_t>(img) * kPH + (oy >> 1)) * kPW * kCo;
      const int64_t rest = static_cast<int64_t>(p.nimg) * kPH * kPW * kCo - pimg;  // elements from the row on
      const __amdgpu_buffer_rsrc_t rdp = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<bf16*>(p.dp) + pimg, 0, static_cast<int>(rest * 2 < 0x7fffffff ? rest * 2 : 0x7fffffff), 0x00020000);
      const __amdgpu_buffer_rsrc_t rix = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint8_t*>(p.idx) + pimg, 0, static_cast<int>(rest < 0x7fffffff ? rest : 0x7fffffff), 0x00020000);
      char* dst = smem + kWPoolOff + buf * kWPool;
#pragma unroll
      for (int i = 0; i < kWPoolPer; ++i) {
        const int L0 = (i * 8 + wave) * 64;  // wave-uniform: the dp / idx / unused boundaries are multiples of 64
        const bool is_dp = L0 < kPoolDpBytes / 16;
        const uint32_t off = L0 < kPoolChunks ? static_cast<uint32_t>((is_dp ? L0 : L0 - kPoolDpBytes / 16) + lane) * 16
                                              : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(is_dp ? rdp : rix, (lds_char*)(dst + (i * 8 + wave) * 1024), 16,
                                                 static_cast<int>(off), 0, 0, 0);
      }
    };
    uint32_t lofs[kWHaloPer];  // this lane's halo chunk: byte offset from its image row, or out of range
#pragma unroll
    for (int i = 0; i < kWHaloPer; ++i) {
      const int L = (i * 8 + wave) * 64 + lane;
      const int hr = L / kBPitch, j = L - hr * kBPitch;
      const bool ok = L < kWHaloChunks && j >= 2 && j <= kIW / 2 + 1;
      lofs[i] = ok ? static_cast<uint32_t>(hr * kIW * 8 + (2 * j - 4) * 8) : 0x80000000u;
    }
    auto issue_halo = [&](int it, int buf) {
      const int img = it / kOH, oy = it - img * kOH;
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<bf16*>(p.x) + static_cast<int64_t>(img) * kIH * kIW * 4, 0, kIH * kIW * 8, 0x00020000);
      const int rowterm = (2 * oy - 4) * kIW * 8;  // may be negative: rows above the image wrap out of range
      char* dst = smem + kWHaloOff + buf * kWHalo;
#pragma unroll
      for (int i = 0; i < kWHaloPer; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_char*)(dst + (i * 8 + wave) * 1024), 16,
                                                 static_cast<int>(lofs[i] + static_cast<uint32_t>(rowterm)), 0, 0, 0);
    };
    const int g = lane >> 4, li = lane & 15, q4 = li >> 2, pp = li & 3;
    const bool gx = wave >= 4;
    const int wn = wave & 3;
    f32x4 acc[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) acc[t][nn] = f32x4{0.f, 0.f, 0.f, 0.f};
    float g3[4] = {0.f, 0.f, 0.f, 0.f};
    const int P0 = 8 * g + q4;
    int a_lo[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      a_lo[t] = kWTilesOff + (gx ? kWTile : 0) + tile_off(P0, 2 * t + (pp >> 1)) + (pp & 1) * 8;
    int b_lo[4];
#pragma unroll
    for (int nn = 0; nn < 4; ++nn) {
      const int kc = 2 * (4 * wn + nn) + (pp >> 1);
      const int ay = kc & 3, ax = (kc >> 2) & 3, by = kc >> 4;
      b_lo[nn] = kWHaloOff + (2 * ay + by) * (kBPitch * 16) + ax * 16 + (pp & 1) * 8 + P0 * 16;
    }
    if (n > 0) issue_pool(it0, 0);
    wait_vm0();
    __syncthreads();  // A
    for (int ph = 0; ph <= n; ++ph) {
      __builtin_amdgcn_s_barrier();  // B1: pool stage ph & 1 (row ph) and halo buffer (ph - 1) & 1 complete
      // row ph + 1's pool stage (its buffer's last reader: row ph - 1's gather) and row ph's halo
      // (its buffer's last reader: row ph - 2's MFMA work), both waited for before B2
      if (ph + 1 < n) issue_pool(it0 + ph + 1, (ph + 1) & 1);
      if (ph < n) issue_halo(it0 + ph, ph & 1);
      if (ph >= 1) {
        const int buf = (ph - 1) & 1;
        const int ta = buf * 2 * kWTile, hb = buf * kWHalo;
#pragma unroll
        for (int ks = 0; ks < kWPix / 32; ++ks) {
          bf16x8 fa[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const char* lo = smem + a_lo[t] + ta + ks * 4096;
            fa[t] = tr_frag(lo, lo + 512);
          }
          // column sums over the real pixels (k-step 3: lane groups 0-1), the k-steps split between the
          // two wave groups; branch-free (a divergent branch here cost registers: spills)
          const bool colsum = gx == static_cast<bool>(ks & 1) && (ks < 3 || g < 2);
          const bf16 one = static_cast<bf16>(colsum ? 1.f : 0.f);
          const bf16x2 w1 = {one, one};
#pragma unroll
          for (int nn = 0; nn < 4; ++nn) {
            const char* lo = smem + b_lo[nn] + hb + ks * 512;
            const bf16x8 fb = tr_frag(lo, lo + 64);
#pragma unroll
            for (int t = 0; t < 4; ++t)
              acc[t][nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t], fb, acc[t][nn], 0, 0, 0);
            {
              bf16x2 h2[4];
              __builtin_memcpy(h2, &fb, 16);
#pragma unroll
              for (int j = 0; j < 4; ++j) g3[nn] = __builtin_amdgcn_fdot2_f32_bf16(h2[j], w1, g3[nn], false);
            }
            __builtin_amdgcn_sched_barrier(0);  // one B fragment live at a time (128-VGPR budget)
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): this wave's DMA landed, fragment reads done
      __builtin_amdgcn_s_barrier();         // B2
    }
    __syncthreads();  // E
    float* part = p.part + static_cast<size_t>(blockIdx.x) * kPart;
    float* gp = part + (gx ? kKk * kCo : 0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) {
        const int k = 16 * (4 * wn + nn) + li;
        *reinterpret_cast<f32x4*>(gp + k * kCo + 16 * t + 4 * g) = acc[t][nn];
      }
#pragma unroll
    for (int nn = 0; nn < 4; ++nn) g3[nn] = butterfly_from<16>(g3[nn]);
    float* red3 = reinterpret_cast<float*>(smem);  // [256] (the tiles are free after E)
    if (gx && g == 0) {
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) red3[16 * (4 * wn + nn) + li] = g3[nn];
    }
    __syncthreads();  // F
    if (!gx && g == 0) {
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) {
        const int k = 16 * (4 * wn + nn) + li;
        part[2 * kKk * kCo + k] = g3[nn] + red3[k];
      }
    }
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
  FLUXMPI_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_bwd_ws_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kWSmem));
  done = true;
}
}  // namespace

// FLUXMPI_STEM_BWD=ws: the wave-specialised kernel instead of the row-pair one. Measured SLOWER
// (profiles/rd6k_stem_ws_ab.jsonl: 404-414 vs 311-320 us per call, ResNet-50 -0.4 %): the element
// role's VALU-heavy gather shares each SIMD's issue with the MFMA role's dense k-steps (an MFMA
// holds the vector issue for half its cycles), so it runs ~2x slower than with the SIMDs to
// itself, and it was already the longer of the two phases.
static bool stem_bwd_ws() {
  static const bool on = [] {
    const char* e = std::getenv("FLUXMPI_STEM_BWD");
    return e != nullptr && std::string(e) == "ws";
  }();
  return on;
}

int stem_bwd_blocks(int64_t n) {
  static int b = [] {
    set_lds_attrs();
    const int r = stem_bwd_ws() ? resident_blocks(reinterpret_cast<const void*>(&stem_bwd_ws_kernel), kWT, kWSmem)
                                : resident_blocks(reinterpret_cast<const void*>(&stem_bwd_kernel<0>), kBT, kBSmem);
    return r > 0 ? r : 256;
  }();
  const int64_t iters = n * (stem_bwd_ws() ? kOH : kPH);
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
  const bool ws = stem_bwd_ws() && mode == 0;
  const int total = static_cast<int>(n * (ws ? kOH : kPH));
  StemBwdArgs a{static_cast<const bf16*>(x), static_cast<const bf16*>(c), static_cast<const bf16*>(dp), idx, mean, inv,
                part, stats, (total + blocks - 1) / blocks, total, static_cast<int>(n)};
  if (ws) {
    stem_bwd_ws_kernel<<<static_cast<unsigned>(blocks), kWT, kWSmem, s>>>(a);
  } else {
    auto kern = mode == 1 ? stem_bwd_kernel<1> : mode == 2 ? stem_bwd_kernel<2> : mode == 3 ? stem_bwd_kernel<3> : stem_bwd_kernel<0>;
    kern<<<static_cast<unsigned>(blocks), kBT, kBSmem, s>>>(a);
  }
  FLUXMPI_HIP_CHECK(hipGetLastError());
  bn_finalize_bwd(stats, kCo, dw_bn, db_bn, s);
  stem_wgrad_combine_kernel<<<kKk, kCT, 0, s>>>(part, blocks, w, mean, inv, dw_bn, db_bn,
                                               1.f / static_cast<float>(n * kOH * kOW), dwp);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
