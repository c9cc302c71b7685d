// MFMA bf16 GEMM for 1x1 convolutions (NHWC) with BatchNorm fusions — gfx950.
//
// C[M,N] = A[M,K] · B[N,K]^T, fp32 accumulation on v_mfma_f32_16x16x32_bf16.
// Each operand is stored either K-major ([rows][K], K contiguous) or
// row-major along M/N ([K][rows], rows contiguous); the three 1x1-conv passes
// map onto it as
//
//   forward  Y[m,co]  = X[m,:] · W[co,:]^T        A = X  (K-major)  B = W (K-major)
//   dgrad    dX[m,ci] = dY[m,:] · W[:,ci]         A = dY (K-major)  B = W (N-major)
//   wgrad    dW[co,ci]= dY[:,co]^T · X[:,ci]      A = dY (M-major)  B = X (N-major), split-K
//
// Staging is global -> registers -> LDS in the operand's natural orientation
// (16 B per lane, coalesced). K-major tiles are read as MFMA fragments with
// ds_read_b128; M/N-major tiles with two ds_read_b64_tr_b16 (gfx950 transposed
// LDS read), so no operand is ever transposed in memory.
//
// Fusions that remove whole activation passes of ResNet-50:
//  * prologue: an optional per-channel affine + ReLU (the previous BatchNorm,
//    y = relu(x*scale + shift), bit-identical to the fused-BN kernels) applied
//    to the A operand (forward, per k) or the B operand (wgrad, per n) while
//    staging, so the normalised activation is never written to HBM;
//  * epilogue: bf16 store + per-column sum / sum-of-squares of the stored bf16
//    values into a sharded fp32 accumulator (the next BatchNorm's statistics,
//    so its stats pass disappears); or fp32 atomic accumulation (split-K).
//
// Tiles: 256 threads = 4 waves (2 x 2), BM x BN x 32 with BM, BN in {64, 128};
// LDS double buffer, next tile's global loads issued before the MFMAs of the
// current one. Blocks are mapped XCD-aware (consecutive tiles of one XCD share
// the A panel in its L2).
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int BK = 32;
constexpr int kShards = 64;  // must match batchnorm.hip

struct GemmArgs {
  const bf16* a;
  const bf16* b;
  void* c;
  int64_t lda, ldb, ldc;  // row strides of the stored matrices (elements)
  int64_t M, N, K;
  int64_t k_per_split;  // K range per blockIdx.z
  const float* a_scale;  // prologue affine on A (per k) — forward
  const float* a_shift;
  const float* b_scale;  // prologue affine on B (per n) — wgrad
  const float* b_shift;
  float* stats;  // [kShards][2][N] sharded per-column sum / sumsq (epilogue mode 1)
  const bf16* res;  // optional residual added in the bf16 epilogue (modes 0/1), row stride ldr
  int64_t ldr;
  // mode 1 with bnb_x: instead of sum/sumsq of the output, accumulate the BatchNorm-backward
  // reductions of a BN whose output gradient IS this GEMM's output: sum(dy_eff) and
  // sum(dy_eff * xhat), xhat = (x - mean) * invstd, dy_eff = dy masked by the BN's ReLU
  // (bnb_rm 0: none, 2: recomputed as fma(x, w*invstd, b - mean*w*invstd) > 0, 3: bit mask)
  const bf16* bnb_x;  // BN input, [M][N] dense
  const float* bnb_w;
  const float* bnb_b;
  const float* bnb_mean;
  const float* bnb_inv;
  const uint8_t* bnb_mask;
  int bnb_rm;
  int mode;      // 0: store bf16; 1: store bf16 + stats; 2: fp32 atomic add into c
  int tiles_m, tiles_n;
  // implicit 3x3 / stride 1 / pad 1 convolution (CONV kernels): A row m is output pixel m of an
  // NHWC image batch [M / (H*W)][H][W][C]; K = 9*C ordered (tap r*3+s, channel); K-tile t reads
  // the C-slice of tap t*BK/C from pixel m + (r-1)*W + (s-1) (zero outside the image)
  int conv_h, conv_w, conv_c;
};

template <int ROWS, bool KMAJOR>
struct Tile {
  // K-major image: [ROWS][BK + 8] (80 B rows: conflict-free 16-row b128 reads)
  // rows-major image: [BK][ROWS + 16] (row stride == 8 dwords mod 64 for tr reads)
  static constexpr int kStride = KMAJOR ? (BK + 8) : (ROWS + 16);
  static constexpr int kElems = KMAJOR ? ROWS * kStride : BK * kStride;
  static constexpr int kChunks = ROWS * BK / 8;  // 16 B chunks per tile
};

__device__ __forceinline__ void affine_relu8(uint4& v, const float* __restrict__ sc, const float* __restrict__ sh,
                                             int64_t c0) {
  bf16 e[8];
  __builtin_memcpy(e, &v, 16);
  const float4 s0 = *reinterpret_cast<const float4*>(sc + c0);
  const float4 s1 = *reinterpret_cast<const float4*>(sc + c0 + 4);
  const float4 h0 = *reinterpret_cast<const float4*>(sh + c0);
  const float4 h1 = *reinterpret_cast<const float4*>(sh + c0 + 4);
  const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float o = fmaf(static_cast<float>(e[j]), s[j], h[j]);
    e[j] = static_cast<bf16>(o > 0.f ? o : 0.f);
  }
  __builtin_memcpy(&v, e, 16);
}

// Load this thread's share of one operand tile into registers.
// KMAJOR: tile rows r0..r0+ROWS of [rows][K] storage, k range k0..k0+BK.
// !KMAJOR: k rows k0..k0+BK of [K][rows] storage, columns r0..r0+ROWS.
template <int ROWS, bool KMAJOR, int CPT>
__device__ __forceinline__ void stage_load(uint4 (&reg)[CPT],
                                           const bf16* __restrict__ g, int64_t ld, int64_t rows, int64_t r0,
                                           int64_t k0, const float* __restrict__ sc, const float* __restrict__ sh,
                                           int64_t kend) {
  static_assert(CPT == ROWS * BK / 8 / kThreads, "chunks per thread");
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    uint4 v = make_uint4(0, 0, 0, 0);  // zero fill: out-of-range rows / k contribute nothing
    if (KMAJOR) {
      const int r = idx / (BK / 8), kc = idx % (BK / 8);
      const int64_t row = r0 + r;
      if (row < rows && k0 + kc * 8 < kend) {  // K % 8 == 0 for K-major operands (host-checked)
        v = *reinterpret_cast<const uint4*>(g + row * ld + k0 + kc * 8);
        if (sc != nullptr) affine_relu8(v, sc, sh, k0 + kc * 8);
      }
    } else {
      const int kr = idx / (ROWS / 8), rc = idx % (ROWS / 8);
      const int64_t col = r0 + rc * 8;
      if (col < rows && k0 + kr < kend) {
        v = *reinterpret_cast<const uint4*>(g + (k0 + kr) * ld + col);
        if (sc != nullptr) affine_relu8(v, sc, sh, col);  // per-row-channel affine (wgrad B = X)
      }
    }
    reg[i] = v;
  }
}

// Implicit-convolution A tile (K-major, BK channels of one tap per K-tile): chunk i of this
// thread is row r_i of the tile, whose output pixel lies at image position (ph[i], pw[i]).
template <int ROWS, int CPT>
__device__ __forceinline__ void stage_load_conv(uint4 (&reg)[CPT], const bf16* __restrict__ x, int64_t rows,
                                                int64_t r0, int64_t k0, const int (&ph)[CPT], const int (&pw)[CPT],
                                                int H, int W, int C, const float* __restrict__ sc,
                                                const float* __restrict__ sh) {
  const int tap = static_cast<int>(k0 / C);
  const int c0 = static_cast<int>(k0 - static_cast<int64_t>(tap) * C);
  const int dr = tap / 3 - 1, ds = tap % 3 - 1;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    const int r = idx / (BK / 8), kc = idx % (BK / 8);
    const int64_t row = r0 + r;
    uint4 v = make_uint4(0, 0, 0, 0);  // zero padding of the (activated) input
    if (row < rows && static_cast<unsigned>(ph[i] + dr) < static_cast<unsigned>(H) &&
        static_cast<unsigned>(pw[i] + ds) < static_cast<unsigned>(W)) {
      const int64_t pix = row + dr * W + ds;
      v = *reinterpret_cast<const uint4*>(x + pix * C + c0 + kc * 8);
      if (sc != nullptr) affine_relu8(v, sc, sh, c0 + kc * 8);
    }
    reg[i] = v;
  }
}

template <int ROWS, bool KMAJOR, int CPT>
__device__ __forceinline__ void stage_store(bf16* __restrict__ lds, const uint4 (&reg)[CPT]) {
  constexpr int S = Tile<ROWS, KMAJOR>::kStride;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (KMAJOR) {
      const int r = idx / (BK / 8), kc = idx % (BK / 8);
      *reinterpret_cast<uint4*>(lds + r * S + kc * 8) = reg[i];
    } else {
      const int kr = idx / (ROWS / 8), rc = idx % (ROWS / 8);
      *reinterpret_cast<uint4*>(lds + kr * S + rc * 8) = reg[i];
    }
  }
}

// Fragment of a 16-row slice starting at tile row `r0` for the 16x16x32 MFMA:
// lane l gets rows (r0 + (l&15)), k = 8*(l>>4) .. +7.
template <int ROWS, bool KMAJOR>
__device__ __forceinline__ bf16x8 read_frag(const bf16* __restrict__ lds, int r0) {
  const int l = threadIdx.x & 63;
  constexpr int S = Tile<ROWS, KMAJOR>::kStride;
  if (KMAJOR) {
    return *reinterpret_cast<const bf16x8*>(lds + (r0 + (l & 15)) * S + 8 * (l >> 4));
  } else {
    // ds_read_b64_tr_b16: in each 16-lane group g, lane 4q+p addresses row (k) q of a
    // 4-row block, columns 4p..4p+3; lane i receives column i of the 4 rows.
    const int g = l >> 4, li = l & 15, q = li >> 2, p = li & 3;
    const bf16* base0 = lds + (8 * g + q) * S + r0 + 4 * p;
    const bf16* base1 = base0 + 4 * S;
    typedef short short4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) short4v lds_short4v;
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(base0));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(base1));
    bf16x8 out;
    __builtin_memcpy(&out, &lo, 8);
    __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
    return out;
  }
}

// NBUF = 2: double-buffered LDS, the next K-tile's loads overlap this tile's MFMAs
// (compute-bound shapes). NBUF = 1: half the LDS, so twice the workgroups per CU —
// for short K (memory-bound 1x1 convs) other workgroups' loads hide the latency.
// EX: epilogue extras (residual add, BN-backward statistics) compiled in; the plain variant
// keeps the lean epilogue (its register footprint sets the occupancy of the main loop)
template <int BM, int BN, bool AK, bool BKM, int NBUF, bool EX, bool CONV = false>
__global__ __launch_bounds__(kThreads) void gemm_kernel(GemmArgs p) {
  using TA = Tile<BM, AK>;
  using TB = Tile<BN, BKM>;
  constexpr int WM = BM / 2, WN = BN / 2;  // per-wave tile
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int kSmem = NBUF * (TA::kElems + TB::kElems);
  __shared__ __attribute__((aligned(16))) bf16 smem[kSmem];
  // buffer b of A at smem + b*kElemsA, of B at smem + NBUF*kElemsA + b*kElemsB
  auto la = [&](int b) { return smem + b * TA::kElems; };
  auto lb = [&](int b) { return smem + NBUF * TA::kElems + b * TB::kElems; };

  // XCD-aware tile order: blocks b and b+8 share an XCD; give each XCD a contiguous
  // range of tiles (n fastest) so neighbouring tiles share A rows in that L2.
  const int nt = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nt / 8, r = nt % 8, xcd = bid % 8, pos = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int tm = bid / p.tiles_n, tn = bid % p.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * BM, n0 = static_cast<int64_t>(tn) * BN;
  const int64_t kbeg = static_cast<int64_t>(blockIdx.z) * p.k_per_split;
  int64_t kend = kbeg + p.k_per_split;
  if (kend > p.K) kend = p.K;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int CA = TA::kChunks / kThreads;
  uint4 ra[CA], rb[TB::kChunks / kThreads];
  // CONV: image position of the output pixel of each A row this thread stages (fixed over K)
  int ph[CA], pw[CA];
  if (CONV) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int64_t row = m0 + (threadIdx.x + i * kThreads) / (BK / 8);
      const int hw = static_cast<int>(row % (static_cast<int64_t>(p.conv_h) * p.conv_w));
      ph[i] = hw / p.conv_w;
      pw[i] = hw - ph[i] * p.conv_w;
    }
  }
  auto load_a = [&](int64_t k0) {
    if (CONV) stage_load_conv<BM>(ra, p.a, p.M, m0, k0, ph, pw, p.conv_h, p.conv_w, p.conv_c, p.a_scale, p.a_shift);
    else stage_load<BM, AK>(ra, p.a, p.lda, p.M, m0, k0, p.a_scale, p.a_shift, kend);
  };
  const int64_t nk = (kend - kbeg + BK - 1) / BK;  // last K-tile may be partial (zero-filled)
  if (nk > 0) {
    load_a(kbeg);
    stage_load<BN, BKM>(rb, p.b, p.ldb, p.N, n0, kbeg, p.b_scale, p.b_shift, kend);
    stage_store<BM, AK>(la(0), ra);
    stage_store<BN, BKM>(lb(0), rb);
  }
  __syncthreads();
  for (int64_t t = 0; t < nk; ++t) {
    const int cur = NBUF == 2 ? (t & 1) : 0;
    const bool more = t + 1 < nk;
    if (NBUF == 1 && t > 0) {  // single buffer: refill after every wave finished reading it
      __syncthreads();
      stage_store<BM, AK>(la(0), ra);
      stage_store<BN, BKM>(lb(0), rb);
      __syncthreads();
    }
    if (more) {  // issue next tile's global loads before this tile's MFMAs
      const int64_t k1 = kbeg + (t + 1) * BK;
      load_a(k1);
      stage_load<BN, BKM>(rb, p.b, p.ldb, p.N, n0, k1, p.b_scale, p.b_shift, kend);
    }
    bf16x8 fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = read_frag<BM, AK>(la(cur), wm * WM + i * 16);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = read_frag<BN, BKM>(lb(cur), wn * WN + j * 16);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (NBUF == 2) {
      if (more) {
        stage_store<BM, AK>(la(cur ^ 1), ra);
        stage_store<BN, BKM>(lb(cur ^ 1), rb);
      }
      __syncthreads();
    }
  }
  if (NBUF == 1) __syncthreads();

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][r]: row m0 + wm*WM + i*16 + 4*(lane>>4) + r, col n0 + wn*WN + j*16 + (lane&15)
  const int col_in = lane & 15, rq = 4 * (lane >> 4);
  if (p.mode == 2 || p.mode == 3) {
    // 2: fp32 atomic accumulate into C; 3: plain fp32 store of this split's partial into
    // slice blockIdx.z of a [splits][M][ldc] workspace (summed by splitk_reduce_kernel)
    float* c = static_cast<float*>(p.c) + (p.mode == 3 ? static_cast<int64_t>(blockIdx.z) * p.M * p.ldc : 0);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t n = n0 + wn * WN + j * 16 + col_in;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t m = m0 + wm * WM + i * 16 + rq + r;
          if (m < p.M && n < p.N) {
            if (p.mode == 2) atomicAdd(c + m * p.ldc + n, acc[i][j][r]);
            else c[m * p.ldc + n] = acc[i][j][r];
          }
        }
      }
    return;
  }
  // bf16 output: stage the tile through LDS (the operand buffers are free after the
  // loop's final barrier) so every lane stores 16 contiguous bytes; the BatchNorm
  // statistics are taken from the same staged bf16 values.
  constexpr int CS = BN + 8;  // padded row (bf16 elements)
  // the C tile is staged in NP passes of BM/NP rows when it exceeds the operand LDS
  constexpr int NP = (BM * CS <= kSmem) ? 1 : 2;
  static_assert(NP == 1 || (BM / 2) * CS <= kSmem, "C half tile must fit the operand LDS");
  static_assert(NP == 1 || WM == BM / 2, "pass split follows the wave rows");
  constexpr int PR = BM / NP;            // rows per pass
  constexpr int CPR = BN / 8;            // 16 B chunks per row
  constexpr int RPI = kThreads / CPR;    // rows per store sweep
  bf16* cl = smem;
  const int cc = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
  const int64_t n = n0 + cc * 8;
  const bool ncol_ok = n + 8 <= p.N;
  bf16* c = static_cast<bf16*>(p.c);
  float cs[8], cq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] = 0.f;
    cq[e] = 0.f;
  }
  const bool bnb = EX && p.mode == 1 && p.bnb_x != nullptr;
  // BN-backward epilogue: per-column (mean, invstd, forward scale, forward shift) in LDS
  // (registers would lower the occupancy of the whole kernel)
  __shared__ float bcoef[EX ? 4 : 1][EX ? BN : 1];
  if (EX && bnb) {
    for (int col = threadIdx.x; col < BN; col += kThreads) {
      const int64_t c = n0 + col < p.N ? n0 + col : p.N - 1;
      const float mu = p.bnb_mean[c], iv = p.bnb_inv[c];
      const float sc = (p.bnb_w ? p.bnb_w[c] : 1.f) * iv;  // == forward scale
      bcoef[0][col] = mu;
      bcoef[1][col] = iv;
      bcoef[2][col] = sc;
      bcoef[3][col] = fmaf(-mu, sc, p.bnb_b ? p.bnb_b[c] : 0.f);  // == forward shift
    }
  }
  // rows this thread stores per pass; the residual / BN-input rows they need are fetched
  // PB rows at a time (one latency per batch instead of one per row)
  constexpr int NIT = (PR + RPI - 1) / RPI;
  constexpr int PB = EX ? (NIT < 3 ? NIT : 3) : 1;
  const bool want_res = EX && p.res != nullptr, want_x = bnb, want_mask = bnb && p.bnb_rm == 3;
#pragma unroll
  for (int h = 0; h < NP; ++h) {
    if (h > 0) __syncthreads();  // previous pass fully read
    if (NP == 1 || wm == h) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cl[(wm * WM - h * PR + i * 16 + rq + r) * CS + wn * WN + j * 16 + col_in] =
                static_cast<bf16>(acc[i][j][r]);
    }
    __syncthreads();
#pragma unroll
    for (int it0 = 0; it0 < NIT; it0 += PB) {
      uint4 rv[PB], xv[PB];
      unsigned mbv[PB];
#pragma unroll
      for (int b = 0; b < PB; ++b) {
        const int r = r0 + (it0 + b) * RPI;
        const int64_t m = m0 + h * PR + r;
        const bool ok = it0 + b < NIT && r < PR && m < p.M && ncol_ok;
        rv[b] = xv[b] = make_uint4(0, 0, 0, 0);
        mbv[b] = 0u;
        if (want_res && ok) rv[b] = *reinterpret_cast<const uint4*>(p.res + m * p.ldr + n);
        if (want_x && ok) xv[b] = *reinterpret_cast<const uint4*>(p.bnb_x + m * p.N + n);
        if (want_mask && ok) mbv[b] = p.bnb_mask[(m * p.N + n) >> 3];
      }
#pragma unroll
      for (int b = 0; b < PB; ++b) {
        const int it = it0 + b;
        const int r = r0 + it * RPI;
        const int64_t m = m0 + h * PR + r;
        if (it >= NIT || r >= PR || m >= p.M) continue;
        uint4 v = *reinterpret_cast<const uint4*>(cl + r * CS + cc * 8);
        if (want_res) {  // fused residual add: C = bf16(bf16(A*B) + R)
          bf16 e8[8], r8[8];
          __builtin_memcpy(e8, &v, 16);
          if (ncol_ok) {
            __builtin_memcpy(r8, &rv[b], 16);
          } else {
            for (int e = 0; e < 8; ++e) r8[e] = n + e < p.N ? p.res[m * p.ldr + n + e] : static_cast<bf16>(0.f);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e)
            e8[e] = static_cast<bf16>(static_cast<float>(e8[e]) + static_cast<float>(r8[e]));
          __builtin_memcpy(&v, e8, 16);
        }
        if (ncol_ok) {
          *reinterpret_cast<uint4*>(c + m * p.ldc + n) = v;
        } else {
          const bf16* e8 = reinterpret_cast<const bf16*>(&v);
          for (int e = 0; e < 8 && n + e < p.N; ++e) c[m * p.ldc + n + e] = e8[e];
        }
        if (bnb) {
          bf16 e8[8], x8[8];
          __builtin_memcpy(e8, &v, 16);
          const int64_t xo = m * p.N + n;  // x is dense [M][N]
          unsigned mb = 0xFFu;
          if (ncol_ok) {
            __builtin_memcpy(x8, &xv[b], 16);
            if (want_mask) mb = mbv[b];
          } else {
            for (int e = 0; e < 8; ++e) x8[e] = n + e < p.N ? p.bnb_x[xo + e] : static_cast<bf16>(0.f);
            if (want_mask) mb = p.bnb_mask[xo >> 3];
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int col = cc * 8 + e;
            const float xf = static_cast<float>(x8[e]);
            bool keep = n + e < p.N;
            if (p.bnb_rm == 2) keep = keep && fmaf(xf, bcoef[2][col], bcoef[3][col]) > 0.f;
            if (p.bnb_rm == 3) keep = keep && ((mb >> e) & 1u);
            const float dd = keep ? static_cast<float>(e8[e]) : 0.f;
            cs[e] += dd;
            cq[e] = fmaf(dd, (xf - bcoef[0][col]) * bcoef[1][col], cq[e]);
          }
        } else if (p.mode == 1) {
          bf16 e8[8];
          __builtin_memcpy(e8, &v, 16);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = static_cast<float>(e8[e]);
            cs[e] += f;
            cq[e] = fmaf(f, f, cq[e]);
          }
        }
      }
    }
  }
  if (p.mode == 1) {
    // lanes of a wave with equal cc differ in the bits above log2(CPR): butterfly them,
    // then combine the 4 waves through LDS and add one atomic per column per block.
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // LDS-free cross-lane butterflies (common.h)
      cs[e] = butterfly_from<CPR>(cs[e]);
      cq[e] = butterfly_from<CPR>(cq[e]);
    }
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [4 waves][2][BN]
    static_assert(4 * 2 * BN * 4 <= kSmem * 2, "stats scratch");
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2 + 0) * BN + cc * 8 + e] = cs[e];
        red[(wave * 2 + 1) * BN + cc * 8 + e] = cq[e];
      }
    }
    __syncthreads();
    float* shard = p.stats + static_cast<size_t>(blockIdx.x % kShards) * 2 * p.N;
    for (int col = threadIdx.x; col < BN; col += kThreads) {
      const float s = red[0 * BN + col] + red[2 * BN + col] + red[4 * BN + col] + red[6 * BN + col];
      const float q = red[1 * BN + col] + red[3 * BN + col] + red[5 * BN + col] + red[7 * BN + col];
      if (n0 + col < p.N) {
        atomicAdd(shard + n0 + col, s);
        atomicAdd(shard + p.N + n0 + col, q);
      }
    }
  }
}

// Split-K reduction as a G-ary tree over the [splits][n] fp32 partials: level l sums
// groups of G logical slices (slice i lives at ws + i*step*n) in parallel over
// (element chunk, group) and writes each group's sum over its first slice (in place:
// every lane reads and writes only its own elements); the last level (<= G slices)
// writes the output dtype. Parallel over splits, so thousands of tiny partial slices
// (small dW, huge K) reduce in a few microseconds.
constexpr int kReduceGroup = 16;

// The reduced row's destination: columns [k seg, (k + 1) seg) go to p[k] (k < 3) — one launch
// writes e.g. a LayerNorm's dw and db straight into their two DDP bucket slices. seg % 4 == 0,
// so a float4 group never straddles two segments.
template <typename TO>
struct OutSeg {
  TO* p[3];
  int64_t seg;
  __device__ __forceinline__ TO* at(int64_t e) const {
    const int64_t k = e / seg;
    return p[k] + (e - k * seg);
  }
};

template <typename TO, bool FINAL>
__global__ __launch_bounds__(kThreads) void splitk_reduce_kernel(float* __restrict__ ws, int cs, int64_t step,
                                                                 int64_t n, OutSeg<TO> out) {
  const int g = blockIdx.y;
  const int i0 = g * kReduceGroup;
  int cnt = cs - i0;
  if (cnt > kReduceGroup) cnt = kReduceGroup;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads * 4;
  for (int64_t e = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * 4; e < n; e += stride) {
    float* base = ws + static_cast<int64_t>(i0) * step * n;
    if ((n & 3) == 0) {  // 16 B aligned slices: 4 independent loads per step
      float4 acc = *reinterpret_cast<const float4*>(base + e);
      int i = 1;
      for (; i + 3 < cnt; i += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(base + (i + u) * step * n + e);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
        }
      }
      for (; i < cnt; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(base + i * step * n + e);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      if (FINAL) {
        TO* o = out.at(e);
        o[0] = static_cast<TO>(acc.x);
        o[1] = static_cast<TO>(acc.y);
        o[2] = static_cast<TO>(acc.z);
        o[3] = static_cast<TO>(acc.w);
      } else {
        *reinterpret_cast<float4*>(base + e) = acc;
      }
    } else {
      for (int64_t k = e; k < e + 4 && k < n; ++k) {
        float a = 0.f;
        for (int i = 0; i < cnt; ++i) a += base[i * step * n + k];
        if (FINAL) *out.at(k) = static_cast<TO>(a);
        else base[k] = a;
      }
    }
  }
}

// One-launch column reduction of S (16 < S <= kColMaxS) partial rows (n % 4 == 0): a workgroup owns
// kColV float4 columns (128 contiguous bytes of a row) x kColPh row phases; each lane sums rows
// ph, ph + kColPh, ... (4 loads in flight), the phases meet in an LDS tree (fixed order:
// deterministic). The G-ary tree below needs 2-3 launches for the few hundred to few thousand
// partial rows of the colsum / LayerNorm / GELU-bias producers and the long-K weight gradients,
// each mostly launch + memory latency (~5 us).
constexpr int kColV = 8, kColPh = 32, kColMaxS = 2048;

template <typename TO>
__global__ __launch_bounds__(kColV * kColPh) void colreduce_kernel(const float* __restrict__ ws, int S, int64_t n,
                                                                   OutSeg<TO> out) {
  const int q = threadIdx.x % kColV, ph = threadIdx.x / kColV;
  const int64_t c4 = static_cast<int64_t>(blockIdx.x) * kColV + q;
  const int64_t n4 = n / 4;
  const int64_t cc = c4 < n4 ? c4 : n4 - 1;  // clamped: loads unconditional, the store is masked
  const float4* w4 = reinterpret_cast<const float4*>(ws);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int s = ph;
  for (; s + 3 * kColPh < S; s += 4 * kColPh) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = w4[static_cast<int64_t>(s + u * kColPh) * n4 + cc];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
    }
  }
  for (; s < S; s += kColPh) {
    const float4 v = w4[static_cast<int64_t>(s) * n4 + cc];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  __shared__ float4 red[kColPh][kColV];
  red[ph][q] = acc;
  __syncthreads();
#pragma unroll
  for (int w = kColPh / 2; w > 0; w >>= 1) {
    if (ph < w) {
      const float4 o = red[ph + w][q];
      float4& m = red[ph][q];
      m.x += o.x; m.y += o.y; m.z += o.z; m.w += o.w;
    }
    __syncthreads();
  }
  if (ph == 0 && c4 < n4) {
    const float4 r = red[0][q];
    TO* o = out.at(c4 * 4);
    o[0] = static_cast<TO>(r.x);
    o[1] = static_cast<TO>(r.y);
    o[2] = static_cast<TO>(r.z);
    o[3] = static_cast<TO>(r.w);
  }
}

// n == 1 (a scalar's partials, e.g. the DEQ adjoint's |u_new - u|^2): one workgroup, fixed order
template <typename TO>
__global__ __launch_bounds__(kThreads) void sumall_kernel(const float* __restrict__ ws, int S, TO* __restrict__ out) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < S; i += kThreads) acc += ws[i];
  __shared__ float red[kThreads / 64];
  const float w = wave_sum_dpp(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) t += red[i];
    out[0] = static_cast<TO>(t);
  }
}

template <int BM, int BN, bool AK, bool BKM, int NBUF, bool EX = false, bool CONV = false>
void launch(const GemmArgs& a0, int splits, hipStream_t s) {
  GemmArgs a = a0;
  a.tiles_m = static_cast<int>((a.M + BM - 1) / BM);
  a.tiles_n = static_cast<int>((a.N + BN - 1) / BN);
  dim3 grid(a.tiles_m * a.tiles_n, 1, splits);
  gemm_kernel<BM, BN, AK, BKM, NBUF, EX, CONV><<<grid, kThreads, 0, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

void gemm_bf16(const GemmProblem& g, hipStream_t stream) {
  // engine 0 (auto): the LDS-DMA pipelined kernel for every problem it covers
  // (not for a prologue affine: its per-fragment transform costs the LDS-DMA kernel 1.3-2.3x —
  // measured — while register staging applies it on the way to LDS; engine 2 forces it)
  const bool glds_only = g.res_mask != nullptr || g.res_sub_h > 0 || g.a_sub_h > 0 || g.conv_s == 2 || g.conv_s >= 16;
  if (glds_only && !gemm_glds_supported(g))
    throw std::runtime_error("gemm_bf16: a masked / subsampled residual or a subsampled A needs the LDS-DMA kernel");
  if (g.engine >= 2 || glds_only || (g.engine == 0 && g.a_scale == nullptr && gemm_glds_supported(g))) {
    gemm_glds(g, stream);
    return;
  }
  if ((g.a_kmajor || g.b_kmajor) && g.K % 8 != 0) throw std::runtime_error("gemm_bf16: K-major operands need K % 8 == 0");
  if ((g.a_kmajor ? g.lda : g.lda) % 8 != 0 || g.ldb % 8 != 0)
    throw std::runtime_error("gemm_bf16: leading dimensions must be multiples of 8");
  if (g.mode == 1 && g.stats == nullptr) throw std::runtime_error("gemm_bf16: stats buffer required");
  if ((g.a_scale != nullptr) && !g.a_kmajor) throw std::runtime_error("gemm_bf16: A affine needs K-major A");
  if ((g.b_scale != nullptr) && g.b_kmajor) throw std::runtime_error("gemm_bf16: B affine needs N-major B");
  GemmArgs a{};
  a.a = static_cast<const bf16*>(g.a);
  a.b = static_cast<const bf16*>(g.b);
  a.c = g.c;
  a.lda = g.lda; a.ldb = g.ldb; a.ldc = g.ldc;
  a.M = g.M; a.N = g.N; a.K = g.K;
  int splits = g.splits < 1 ? 1 : g.splits;
  int64_t kps = ((g.K + BK - 1) / BK + splits - 1) / splits * BK;
  splits = static_cast<int>((g.K + kps - 1) / kps);
  a.k_per_split = kps;
  a.a_scale = g.a_scale; a.a_shift = g.a_shift;
  a.b_scale = g.b_scale; a.b_shift = g.b_shift;
  a.stats = g.stats;
  a.mode = g.mode;
  a.res = static_cast<const bf16*>(g.res);
  a.ldr = g.ldr;
  a.bnb_x = static_cast<const bf16*>(g.bnb_x);
  a.bnb_w = g.bnb_w;
  a.bnb_b = g.bnb_b;
  a.bnb_mean = g.bnb_mean;
  a.bnb_inv = g.bnb_inv;
  a.bnb_mask = g.bnb_mask;
  a.bnb_rm = g.bnb_rm;
  if (a.bnb_x != nullptr) {
    if (g.mode != 1 || g.ldc != g.N || g.N % 8 != 0 || g.bnb_mean == nullptr || g.bnb_inv == nullptr ||
        (g.bnb_rm == 3 && g.bnb_mask == nullptr) || (g.bnb_rm != 0 && g.bnb_rm != 2 && g.bnb_rm != 3))
      throw std::runtime_error("gemm_bf16: BN-backward epilogue needs mode 1, dense C (ldc == N, N % 8 == 0), "
                               "mean/invstd and a valid ReLU mode");
  }
  if (a.res != nullptr && (g.mode > 1 || g.ldr % 8 != 0))
    throw std::runtime_error("gemm_bf16: residual epilogue needs mode 0/1 and ldr % 8 == 0");
  if (splits > 1 && g.mode != 2 && g.mode != 3)
    throw std::runtime_error("gemm_bf16: split-K needs mode 2 (fp32 atomics) or 3 (fp32 partials)");
  const bool bm128 = g.M >= 128 && g.tile_m != 64;
  const bool bn128 = g.N >= 128 && g.tile_n != 64;
  if (g.conv_h > 0) {
    // implicit 3x3/s1/p1 convolution: A = NHWC image (K = 9*C), B = K-major [N][9*C] filter
    if (!g.a_kmajor || !g.b_kmajor || g.conv_c % BK != 0 || g.K != 9LL * g.conv_c || g.conv_w <= 0 ||
        g.M % (static_cast<int64_t>(g.conv_h) * g.conv_w) != 0 || splits != 1 || g.mode > 1 ||
        a.res != nullptr || a.bnb_x != nullptr)
      throw std::runtime_error("gemm_bf16: implicit conv needs K-major A/B, C % 32 == 0, K == 9*C, M a multiple of "
                               "H*W, no split and mode 0/1 without residual / BN-backward epilogue");
    a.conv_h = g.conv_h;
    a.conv_w = g.conv_w;
    a.conv_c = g.conv_c;
    if (bm128 && bn128) launch<128, 128, true, true, 2, false, true>(a, 1, stream);
    else if (bm128) launch<128, 64, true, true, 2, false, true>(a, 1, stream);
    else if (bn128) launch<64, 128, true, true, 2, false, true>(a, 1, stream);
    else launch<64, 64, true, true, 2, false, true>(a, 1, stream);
    return;
  }
#define DISPATCH2(AK, BKM, NB)                                          \
  if (bm128 && bn128) launch<128, 128, AK, BKM, NB>(a, splits, stream);  \
  else if (bm128) launch<128, 64, AK, BKM, NB>(a, splits, stream);       \
  else if (bn128) launch<64, 128, AK, BKM, NB>(a, splits, stream);       \
  else launch<64, 64, AK, BKM, NB>(a, splits, stream);
#define DISPATCH(AK, BKM) \
  if (single) { DISPATCH2(AK, BKM, 1) } else { DISPATCH2(AK, BKM, 2) }
  // double buffering measured faster for every ResNet-50 1x1 shape (fwd/dgrad/wgrad);
  // the single-buffered variant is kept selectable for experiments
  const bool single = g.nbuf == 1;
  if (a.res != nullptr || a.bnb_x != nullptr) {
    // epilogue extras: compiled for the dgrad layout (K-major dY, N-major W) only
    // (always double-buffered: the single-buffered variant is not compiled with extras)
    if (!(g.a_kmajor && !g.b_kmajor) || splits != 1)
      throw std::runtime_error("gemm_bf16: residual / BN-backward epilogues need the dgrad layout and no split");
    if (bm128 && bn128) launch<128, 128, true, false, 2, true>(a, 1, stream);
    else if (bm128) launch<128, 64, true, false, 2, true>(a, 1, stream);
    else if (bn128) launch<64, 128, true, false, 2, true>(a, 1, stream);
    else launch<64, 64, true, false, 2, true>(a, 1, stream);
    return;
  }
  if (g.a_kmajor && g.b_kmajor) { DISPATCH(true, true) }
  else if (g.a_kmajor && !g.b_kmajor) { DISPATCH(true, false) }
  else if (!g.a_kmajor && !g.b_kmajor) { DISPATCH(false, false) }
  else { DISPATCH(false, true) }
#undef DISPATCH2
#undef DISPATCH
}

// the one-launch column reduce wherever it applies (the multi-launch tree otherwise)
static bool colreduce_on() { return true; }

namespace {
template <typename TO>
OutSeg<TO> out_seg(void* o0, void* o1, void* o2, int64_t seg) {
  return OutSeg<TO>{{static_cast<TO*>(o0), static_cast<TO*>(o1), static_cast<TO*>(o2)}, seg};
}
}  // namespace

void gemm_splitk_reduce_seg(const float* ws_c, int splits, int64_t n, int64_t seg, void* out0, void* out1, void* out2,
                            int out_dtype, hipStream_t stream) {
  if (out_dtype != static_cast<int>(kF32) && out_dtype != static_cast<int>(kBF16))
    throw std::runtime_error("gemm_splitk_reduce: out dtype must be fp32 or bf16");
  if (seg <= 0 || seg % 4 != 0 || (n + seg - 1) / seg > 3 || (n > seg && out1 == nullptr) ||
      (n > 2 * seg && out2 == nullptr))
    throw std::runtime_error("gemm_splitk_reduce_seg: segments must be multiples of 4, at most 3, all present");
  const bool f32 = out_dtype == static_cast<int>(kF32);
  float* ws = const_cast<float*>(ws_c);  // intermediate tree levels are written in place
  int64_t bx = (n / 4 + kThreads - 1) / kThreads;
  int cs = splits < 1 ? 1 : splits;
  if (cs > kReduceGroup && n == 1 && colreduce_on()) {
    if (f32) sumall_kernel<float><<<1, kThreads, 0, stream>>>(ws, cs, static_cast<float*>(out0));
    else sumall_kernel<bf16><<<1, kThreads, 0, stream>>>(ws, cs, static_cast<bf16*>(out0));
    FLUXMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  if (cs > kReduceGroup && cs <= kColMaxS && n % 4 == 0 && n > 0 && colreduce_on()) {
    const unsigned gx = static_cast<unsigned>((n / 4 + kColV - 1) / kColV);
    if (f32) colreduce_kernel<float><<<gx, kColV * kColPh, 0, stream>>>(ws, cs, n, out_seg<float>(out0, out1, out2, seg));
    else colreduce_kernel<bf16><<<gx, kColV * kColPh, 0, stream>>>(ws, cs, n, out_seg<bf16>(out0, out1, out2, seg));
    FLUXMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  int64_t step = 1;
  while (cs > kReduceGroup) {
    const int groups = (cs + kReduceGroup - 1) / kReduceGroup;
    int64_t gx = bx;
    // ~2048 workgroups per level in total
    const int64_t cap = (2048 + groups - 1) / groups;
    if (gx > cap) gx = cap;
    if (gx < 1) gx = 1;
    splitk_reduce_kernel<float, false><<<dim3((unsigned)gx, (unsigned)groups), kThreads, 0, stream>>>(
        ws, cs, step, n, OutSeg<float>{{nullptr, nullptr, nullptr}, n});
    FLUXMPI_HIP_CHECK(hipGetLastError());
    cs = groups;
    step *= kReduceGroup;
  }
  int64_t gx = bx > 4096 ? 4096 : (bx < 1 ? 1 : bx);
  if (f32)
    splitk_reduce_kernel<float, true><<<(unsigned)gx, kThreads, 0, stream>>>(ws, cs, step, n,
                                                                             out_seg<float>(out0, out1, out2, seg));
  else
    splitk_reduce_kernel<bf16, true><<<(unsigned)gx, kThreads, 0, stream>>>(ws, cs, step, n,
                                                                            out_seg<bf16>(out0, out1, out2, seg));
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void gemm_splitk_reduce(const float* ws_c, int splits, int64_t n, void* out, int out_dtype, hipStream_t stream) {
  // one segment covering the row (n % 4 != 0 rows only take the tree path, which masks per element)
  const int64_t seg = n > 0 ? ((n + 3) / 4) * 4 : 4;
  gemm_splitk_reduce_seg(ws_c, splits, n, seg, out, nullptr, nullptr, out_dtype, stream);
}

}  // namespace fluxmpi
