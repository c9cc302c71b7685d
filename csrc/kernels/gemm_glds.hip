// Pipelined MFMA bf16 GEMM (C = A * B^T, both operands K-major) with direct global->LDS
// staging — gfx950.
//
// The register-staged kernel in gemm.hip keeps one K-tile in flight: the next tile's global
// loads are issued before the current tile's MFMAs and must land before the LDS store that
// follows them, so at a 32-deep K-tile (256 MFMA cycles per wave) an L2 round trip is exposed
// on every step. Here the operand tiles go straight from global memory into LDS with
// `global_load_lds_dwordx4` (no staging registers, no ds_write pass) through a ring of
// kStages LDS stages, kStages-1 tiles in flight: a wave waits with a counted
// `s_waitcnt vmcnt(N)` for the OLDEST tile only, then a raw `s_barrier` (never
// __syncthreads(), whose fence would drain the younger DMAs) publishes it to all waves.
//
// LDS image of a stage: [rows][32] bf16 (64 B rows, no padding: an LDS-DMA writes
// lane-linear 1 KiB pieces = 16 rows). The 16-B chunk q of row r sits in slot
// q ^ f(r), f = [0, 3, 2, 1][(r >> 2) & 3] — the swizzle is applied on the per-lane GLOBAL
// source address — so each of ds_read_b128's four 16-lane bank groups ({0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31}, and the same +32: MI355X_MICROARCH.md §LDS) covers the 64 banks once.
// (Round 3: the earlier f = (r >> 2) & 3 put lanes 0-3 and 20-23 on the same banks, a 2-way
// conflict on every fragment read — 8 LDS cycles per ds_read_b128 instead of 4.)
//
// A is either a plain K-major matrix or (CONV) the implicit im2col of a 3x3 / stride 1 /
// pad 1 convolution over an NHWC image batch; out-of-image taps read a line of zeros.
// Epilogue: bf16 C staged through LDS (16-B stores), optional residual add, optional
// per-column sum / sum of squares into the sharded BatchNorm workspace (mode 1).
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kThreads = 256;
constexpr int kShards = 64;  // must match batchnorm.hip

__device__ __attribute__((aligned(16))) uint4 g_zero_line[4];  // source of zero-filled chunks
// stand-in for an absent 1-bit mask (all bits set)
__device__ __attribute__((aligned(16))) uint4 g_ff_line[1] = {{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}};
// Out-of-image / out-of-range chunks of an operand that gets the BatchNorm+ReLU prologue: a
// bf16 NaN payload (0x7FC1) the fragment transform maps to 0 (the padding of the ACTIVATED
// tensor), which relu(0 * scale + shift) would not be.
constexpr unsigned short kPadBits = 0x7FC1;
__device__ __attribute__((aligned(16))) uint4 g_pad_line[4] = {
    {0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u}, {0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u},
    {0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u}, {0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u, 0x7FC17FC1u}};
constexpr int kMaxAffC = 512;  // channels of a prologue affine (scale/shift staged in LDS)

struct GldsArgs {
  const bf16* a;
  const bf16* b;
  bf16* c;
  const bf16* res;
  float* stats;
  int64_t lda, ldb, ldc, ldr;
  int64_t M, N, K;
  int mode;  // 0: C; 1: C + column statistics (or BN-backward reductions, bnb_x != nullptr)
  int tiles_m, tiles_n;
  int conv_h, conv_w, conv_c;
  const bf16* bnb_x;  // BN-backward epilogue: the BatchNorm input [M][N] dense
  const float* bnb_w;
  const float* bnb_b;
  const float* bnb_mean;
  const float* bnb_inv;
  const uint8_t* bnb_mask;
  int bnb_rm;
  const uint8_t* res_mask;  // RES: 1-bit mask of the residual ([M][N] bits, n fastest), or nullptr
  int res_sub_h, res_sub_w;  // RES: > 0 — compact stride-2 residual of an [M/(H*W)][H][W] row grid
  const float* a_scale;  // AFF: A element (m, k) -> relu(A * a_scale[c] + a_shift[c]), c = channel of k
  const float* a_shift;
  int aff_c;             // channels of the affine (C for the implicit conv, K for a 1x1)
  int a_sub_h, a_sub_w;  // > 0: A row (n, ho, wo) is image row (n, 2ho, 2wo) of [.][a_sub_h][a_sub_w] (see api.h)
  int conv_s;            // CONV: 1, or 2 (stride-2 3x3 over the [.][conv_h][conv_w] input; rows = output pixels),
                         // or 16 + (py * 2 + px): one parity class of a stride-2 3x3 INPUT gradient (rows =
                         // the dY pixels [.][conv_h][conv_w] = the class's dX pixels (2a + py, 2b + px))
};

// dX row of class row m = (img, a, b) of the [.][Ho][Wo] dY grid: pixel (img, 2a + py, 2b + px)
// of the [.][2 Ho][2 Wo] input (32-bit math: M < 2^31 host-checked)
__device__ __forceinline__ int64_t dx_row(int64_t m, int Ho, int Wo, int cls) {
  const unsigned mm = static_cast<unsigned>(m), hw = static_cast<unsigned>(Ho) * Wo;
  const unsigned img = mm / hw, r = mm - img * hw, a = r / Wo, b = r - a * Wo;
  return (static_cast<int64_t>(img) * (2 * Ho) + 2 * a + (cls >> 1)) * (2 * Wo) + 2 * b + (cls & 1);
}

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int LPT, int MAXAHEAD>
__device__ __forceinline__ void wait_tiles_ahead(int ahead) {
  if (MAXAHEAD >= 2 && ahead >= 2) wait_vmcnt<(MAXAHEAD >= 2 ? 2 : 0) * LPT>();
  else if (ahead == 1) wait_vmcnt<LPT>();
  else wait_vmcnt<0>();
}

// chunk-slot swizzle of a [rows][BK] bf16 stage tile (BK/8 16-B chunks per row): every 16-lane
// bank group of a ds_read_b128 fragment read (16 rows x one chunk) covers the 64 banks once
// (checked against the instruction's lane grouping by scripts/lds_banks.py)
template <int BK>
__device__ __forceinline__ int swz(int row) {
  return BK == 32 ? ((-(row >> 2)) & 3) : ((row >> 1) & 7);
}

// Issue this wave's LDS-DMA pieces of one operand tile (ROWS x BK) for K offset k0.
// A 1 KiB piece holds RPP = 512/BK rows; piece j of wave w covers tile rows
// (w * PPW + j) * RPP ..; lane l fills row +(l / CPR), slot (l % CPR) with global chunk
// slot ^ swz(row).
// srow (plain operand, optional): the source row of piece j's rows, if not grow itself.
// CONV: ph / pw / pbase = input row, column and pixel index of the tap-centre of piece j's row.
// When C is a multiple of BK a K tile lies inside one tap (one division per tile); otherwise
// (C % 8 == 0, e.g. the 48-channel DEQ cell) a tile straddles taps and every 16-B chunk finds its
// own tap (a chunk never straddles: C % 8 == 0), with K = 9C's partial last tile reading zeros.
template <int ROWS, int BK, bool CONV, bool PAD = false>
__device__ __forceinline__ void issue_tile(bf16* lds_tile, const bf16* __restrict__ g, int64_t ld,
                                           int64_t rows, int64_t r0, int64_t k0, int64_t kend,
                                           const int* ph, const int* pw, int H, int W, int C,
                                           const int64_t* srow = nullptr, const int* pbase = nullptr,
                                           int tapcls = -1) {
  constexpr int CPR = BK / 8, RPP = 64 / CPR;
  constexpr int PPW = ROWS * BK / 2048;  // 1 KiB pieces per wave
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int dr = 0, ds = 0, c0 = 0;
  const bool tile_tap = !CONV || C % BK == 0;  // kernel-uniform
  int64_t bk = k0;  // tap class (plain B operand): the column of the flipped [ci][3][3][co] filter
  if (CONV && tile_tap) {
    const int tap = static_cast<int>(k0 / C);
    c0 = static_cast<int>(k0 - static_cast<int64_t>(tap) * C);
    if (tapcls >= 0) {
      // stride-2 input-gradient parity class (py, px) = (tapcls >> 1, tapcls & 1): its taps in
      // (row tap, column tap) order, row taps kh = 1 (py = 0) or kh = 0, 2 (py = 1) reading dY
      // rows a + 1 and a (dr = +1, 0); columns likewise
      const int px = tapcls & 1, nc = px ? 2 : 1;
      const int tr = tap / nc, tc = tap - tr * nc;
      dr = (tapcls >> 1) && tr == 0 ? 1 : 0;
      ds = px && tc == 0 ? 1 : 0;
    } else {
      dr = tap / 3 - 1;
      ds = tap % 3 - 1;
    }
  } else if (!CONV && tapcls >= 0) {
    const int px = tapcls & 1, nc = px ? 2 : 1;
    const int tap = static_cast<int>(k0 / C), tr = tap / nc, tc = tap - tr * nc;
    const int kh = (tapcls >> 1) ? (tr == 0 ? 0 : 2) : 1, kw = px ? (tc == 0 ? 0 : 2) : 1;
    bk = static_cast<int64_t>(8 - (kh * 3 + kw)) * C + (k0 - static_cast<int64_t>(tap) * C);
  }
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int piece = wave * PPW + j;
    const int row = piece * RPP + lane / CPR;
    const int q = (lane % CPR) ^ swz<BK>(row);
    const int64_t grow = r0 + row;
    const void* src = PAD ? static_cast<const void*>(g_pad_line) : static_cast<const void*>(g_zero_line);
    if (CONV) {
      int cdr = dr, cds = ds, cc = c0 + q * 8;
      bool kin = true;
      if (!tile_tap) {  // K = 9C < 2^31 (host-checked M < 2^31, C <= 8192)
        const unsigned kq = static_cast<unsigned>(k0) + static_cast<unsigned>(q * 8);
        const unsigned tap = kq / static_cast<unsigned>(C);
        cc = static_cast<int>(kq - tap * static_cast<unsigned>(C));
        cdr = static_cast<int>(tap / 3u) - 1;
        cds = static_cast<int>(tap % 3u) - 1;
        kin = static_cast<int64_t>(kq) < kend;
      }
      if (kin && grow < rows && static_cast<unsigned>(ph[j] + cdr) < static_cast<unsigned>(H) &&
          static_cast<unsigned>(pw[j] + cds) < static_cast<unsigned>(W))
        src = g + (static_cast<int64_t>(pbase[j]) + cdr * W + cds) * C + cc;
    } else {
      if (grow < rows && k0 + q * 8 < kend) src = g + (srow != nullptr ? srow[j] : grow) * ld + bk + q * 8;
    }
    typedef __attribute__((address_space(3))) char lds_char;
    typedef __attribute__((address_space(1))) void gl_void;
    __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(reinterpret_cast<char*>(lds_tile) + piece * 1024), 16,
                                     0, 0);
  }
}

// MFMA fragment (16 rows from r0, k = 32 * kh + 8 * (lane >> 4) .. +7) of a swizzled stage tile
template <int BK>
__device__ __forceinline__ bf16x8 read_frag(const bf16* __restrict__ tile, int r0, int kh) {
  const int l = threadIdx.x & 63;
  const int row = r0 + (l & 15);
  const int q = ((l >> 4) + 4 * kh) ^ swz<BK>(row);
  return *reinterpret_cast<const bf16x8*>(tile + row * BK + q * 8);
}

// relu(x * s + t) of the 8 channels of a fragment, bit-identical to the fused BN kernels'
// fmaf; padding chunks (kPadBits) become 0
__device__ __forceinline__ bf16x8 affine_frag(bf16x8 f, const float* __restrict__ st) {
  const float4 q0 = *reinterpret_cast<const float4*>(st);       // s0 t0 s1 t1
  const float4 q1 = *reinterpret_cast<const float4*>(st + 4);   // s2 t2 s3 t3
  const float4 q2 = *reinterpret_cast<const float4*>(st + 8);
  const float4 q3 = *reinterpret_cast<const float4*>(st + 12);
  const float s[8] = {q0.x, q0.z, q1.x, q1.z, q2.x, q2.z, q3.x, q3.z};
  const float t[8] = {q0.y, q0.w, q1.y, q1.w, q2.y, q2.w, q3.y, q3.w};
  unsigned short u[8];
  __builtin_memcpy(u, &f, 16);
  bf16 e[8];
  __builtin_memcpy(e, &f, 16);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float o = fmaf(static_cast<float>(e[j]), s[j], t[j]);
    e[j] = u[j] == kPadBits ? static_cast<bf16>(0.f) : static_cast<bf16>(o > 0.f ? o : 0.f);
  }
  bf16x8 out;
  __builtin_memcpy(&out, e, 16);
  return out;
}

// BNB: the BN-backward epilogue is compiled in (its registers would otherwise cost the lean
// variants occupancy: the allocation covers the epilogue's peak too)
template <int BM, int BN, int kBK, int kStages, bool CONV, bool RES, bool AFF = false, bool BNB = false>
__global__ __launch_bounds__(kThreads, 2) void gemm_glds_kernel(GldsArgs p) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int A_ELEMS = BM * kBK, B_ELEMS = BN * kBK;
  constexpr int kRing = kStages * (A_ELEMS + B_ELEMS);
  constexpr int CS = BN + 8;  // epilogue C staging row (bf16)
  constexpr int kRingOrC = kRing > BM * CS ? kRing : BM * CS;
  // AFF: interleaved (scale, shift) fp32 pairs of the A channels after the ring
  constexpr int kSmem = kRingOrC + (AFF ? kMaxAffC * 4 : 0);
  constexpr int LPT = (BM + BN) * kBK / 2048;  // LDS-DMA instructions per wave per K-tile
  // ONE __shared__ array for the ring, the epilogue staging and the statistics scratch
  __shared__ __attribute__((aligned(16))) bf16 smem[kSmem];
  auto sa = [&](int s) { return smem + s * A_ELEMS; };
  auto sb = [&](int s) { return smem + kStages * A_ELEMS + s * B_ELEMS; };

  // XCD-aware tile order (bijective): blocks sharing an XCD get a contiguous tile range
  const int nt = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nt / 8, r = nt % 8, xcd = bid % 8, pos = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int tm = bid / p.tiles_n, tn = bid % p.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * BM, n0 = static_cast<int64_t>(tn) * BN;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int tapcls = CONV && p.conv_s >= 16 ? p.conv_s - 16 : -1;  // stride-2 input-gradient parity class

  // CONV: image position of each A row this lane stages (fixed over K)
  constexpr int PPWA = BM * kBK / 2048, RPPA = 512 / kBK;
  int ph[PPWA], pw[PPWA], pbase[CONV ? PPWA : 1];
  if (CONV) {
#pragma unroll
    for (int j = 0; j < PPWA; ++j) {
      const int64_t row = m0 + (wave * PPWA + j) * RPPA + lane / (kBK / 8);
      if (p.conv_s == 2) {  // output pixel (img, oh, ow) -> input tap-centre (2oh, 2ow); M < 2^31 host-checked
        const int ho = (p.conv_h + 1) >> 1, wo = (p.conv_w + 1) >> 1;
        const int r = static_cast<int>(row), img = r / (ho * wo), rr = r - img * (ho * wo), oh = rr / wo;
        ph[j] = 2 * oh;
        pw[j] = 2 * (rr - oh * wo);
        pbase[j] = (img * p.conv_h + ph[j]) * p.conv_w + pw[j];
      } else {
        const int hw = static_cast<int>(row % (static_cast<int64_t>(p.conv_h) * p.conv_w));
        ph[j] = hw / p.conv_w;
        pw[j] = hw - ph[j] * p.conv_w;
        pbase[j] = static_cast<int>(row);
      }
    }
  }
  // plain A: the image row each staged A row reads (a_sub: the stride-2 subsample's source pixel)
  int64_t arow[CONV ? 1 : PPWA];
  if (!CONV) {
#pragma unroll
    for (int j = 0; j < PPWA; ++j) {
      const int64_t row = m0 + (wave * PPWA + j) * RPPA + lane / (kBK / 8);
      arow[j] = row;
      if (p.a_sub_h > 0) {  // 32-bit math (host-checked M < 2^31)
        const unsigned ho = (p.a_sub_h + 1) >> 1, wo = (p.a_sub_w + 1) >> 1;
        const unsigned mm = static_cast<unsigned>(row), hw = ho * wo;
        const unsigned img = mm / hw, r = mm - img * hw, y = r / wo, x = r - y * wo;
        arow[j] = (static_cast<int64_t>(img) * p.a_sub_h + 2 * y) * p.a_sub_w + 2 * x;
      }
    }
  }
  auto issue = [&](int s, int64_t k0) {
    issue_tile<BM, kBK, CONV, AFF>(sa(s), p.a, p.lda, p.M, m0, k0, p.K, ph, pw, p.conv_h, p.conv_w, p.conv_c,
                                   CONV ? nullptr : arow, CONV ? pbase : nullptr, tapcls);
    issue_tile<BN, kBK, false>(sb(s), p.b, p.ldb, p.N, n0, k0, p.K, nullptr, nullptr, 0, 0, p.conv_c, nullptr,
                               nullptr, tapcls);
  };
  float* st_lds = reinterpret_cast<float*>(smem + kRingOrC);
  if (AFF) {  // stage the affine pairs once (read back with ds_read_b128 per fragment)
    for (int c = threadIdx.x; c < p.aff_c; c += kThreads) {
      st_lds[2 * c] = p.a_scale[c];
      st_lds[2 * c + 1] = p.a_shift[c];
    }
    __syncthreads();
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---------------------------------------------------------------- epilogue geometry
  // each thread owns one 16-B column chunk (cc) of rows r0, r0 + RPI, ...; its residual /
  // BN-input / mask loads go out in batches of UB rows
  constexpr int CPR = BN / 8;          // 16-B chunks per row
  constexpr int RPI = kThreads / CPR;  // rows per sweep
  constexpr int UB = BNB ? 1 : 4;      // rows per batch (BNB: 2 — its x / mask loads would otherwise push the variant to 185 VGPRs, two workgroups per CU instead of three)
  constexpr int NB = (BM + UB * RPI - 1) / (UB * RPI);
  const int cc = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
  const int64_t n = n0 + cc * 8;
  const bool ncol_ok = n < p.N;  // N % 8 == 0 (host-checked): a chunk is all in or all out
  const int rows_valid = p.M - m0 < BM ? static_cast<int>(p.M - m0) : BM;
  const bool bnb = BNB && p.bnb_x != nullptr;
  // Epilogue operand loads are UNCONDITIONAL (rows / columns outside the problem read row m0 /
  // column 0, which exist, and are skipped when used): a load under a branch makes the compiler
  // wait for it at the join, one exposed memory latency per row. Masks: a 0xFF byte stands in
  // when there is none, and the even-position test of a compact stride-2 residual zeroes its mask.
  struct EpiIn {
    uint4 rv[RES ? UB : 1], xv[BNB ? UB : 1];
    unsigned rmk[RES ? UB : 1], mk[BNB ? UB : 1];
  };
  auto epi_load = [&](int b, EpiIn& e) {
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int r = r0 + (b * UB + u) * RPI;
      const bool ok = r < BM && r < rows_valid && ncol_ok;
      const int64_t m = m0 + (ok ? r : 0);
      const int64_t nn = ncol_ok ? n : 0;
      if (RES) {
        int64_t roff;
        unsigned keep = 0xFFu;
        if (p.res_sub_h > 0) {  // 32-bit row math (host-checked M < 2^31)
          const unsigned mm = static_cast<unsigned>(m), W = p.res_sub_w;
          const unsigned HW = static_cast<unsigned>(p.res_sub_h) * W;
          const unsigned img = mm / HW, hw = mm - img * HW, h = hw / W, w = hw - h * W;
          const unsigned ho = (p.res_sub_h + 1) >> 1, wo = (W + 1) >> 1;
          roff = static_cast<int64_t>((img * ho + (h >> 1)) * wo + (w >> 1)) * p.ldr + nn;
          keep = ((h | w) & 1u) == 0 ? 0xFFu : 0u;
        } else {
          roff = m * p.ldr + nn;
        }
        e.rv[u] = *reinterpret_cast<const uint4*>(p.res + roff);
        const uint8_t* mp = p.res_mask != nullptr ? p.res_mask + ((m * p.N + nn) >> 3)
                                                  : reinterpret_cast<const uint8_t*>(g_ff_line);
        e.rmk[u] = *mp & keep;
      }
      if (BNB) {
        const bf16* xp = bnb ? p.bnb_x + m * p.N + nn : reinterpret_cast<const bf16*>(g_zero_line);
        e.xv[u] = *reinterpret_cast<const uint4*>(xp);
        const uint8_t* mp = (bnb && p.bnb_rm == 3) ? p.bnb_mask + ((m * p.N + nn) >> 3)
                                                   : reinterpret_cast<const uint8_t*>(g_ff_line);
        e.mk[u] = *mp;
      }
    }
  };
  auto mma_tile = [&](int t) {
    const bf16* ta = sa(t % kStages);
    const bf16* tb = sb(t % kStages);
    // AFF: channel of this lane's fragment chunk = (k0 - tap * C) + 8 * ((lane >> 4) + 4 * kh)
    const int c_base = AFF ? static_cast<int>(CONV ? (static_cast<int64_t>(t) * kBK) % p.conv_c
                                                   : static_cast<int64_t>(t) * kBK) + 8 * (lane >> 4) : 0;
#pragma unroll
    for (int kh = 0; kh < kBK / 32; ++kh) {
      bf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = read_frag<kBK>(ta, wm * WM + i * 16, kh);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = read_frag<kBK>(tb, wn * WN + j * 16, kh);
      if (AFF) {
        const int c = c_base + 32 * kh;
        const float* st = st_lds + 2 * (c < p.aff_c ? c : 0);  // K tail: padding chunks anyway
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = affine_frag(fa[i], st);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          // B as the MFMA's first operand: D = C^T, so a lane's 4 accumulators are 4 consecutive
          // COLUMNS of one row (one 8-B LDS write in the epilogue instead of four 2-B ones)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = static_cast<int>((p.K + kBK - 1) / kBK);
#pragma unroll
  for (int s = 0; s < kStages - 1; ++s)
    if (s < nk) issue(s, static_cast<int64_t>(s) * kBK);
  for (int t = 0; t < nk - 1; ++t) {
    const int ahead = nk - 1 - t < kStages - 2 ? nk - 1 - t : kStages - 2;
    wait_tiles_ahead<LPT, kStages - 2>(ahead);  // this wave's pieces of tile t have landed
    __builtin_amdgcn_s_barrier();   // ... and every wave's; every wave is done with tile t-1
    if (t + kStages - 1 < nk) issue((t + kStages - 1) % kStages, static_cast<int64_t>(t + kStages - 1) * kBK);
    mma_tile(t);
  }
  // last tile: nothing is left to stage, so the first epilogue batch's loads go out before its
  // MFMAs and land under them
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  EpiIn ecur;
  if (RES || BNB) epi_load(0, ecur);
  if (nk > 0) mma_tile(nk - 1);
  // ring fully consumed; lgkmcnt only (a __syncthreads() would also wait for the epilogue loads)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][r]: row m0 + wm*WM + i*16 + (lane&15), col n0 + wn*WN + j*16 + 4*(lane>>4) + r
  // (row pitch CS = BN + 8 bf16: the 32 lanes of a half-wave's 8-B writes cover 64 distinct banks)
  const int row_in = lane & 15, cq4 = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bf16 e4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) e4[r] = static_cast<bf16>(acc[i][j][r]);
      uint2 pk;
      __builtin_memcpy(&pk, e4, 8);
      *reinterpret_cast<uint2*>(smem + (wm * WM + i * 16 + row_in) * CS + wn * WN + j * 16 + cq4) = pk;
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  // BN-backward epilogue (mode 1 + bnb_x): C is the output gradient of a BatchNorm whose input is
  // bnb_x; accumulate sum(dy_eff) and sum(dy_eff * xhat) per column instead of sum / sumsq of C.
  // dy_eff = C masked by the BN's ReLU: rm 2 recomputes it bit-identically to the forward
  // (fma(x, w*invstd, b - mean*w*invstd) > 0), rm 3 reads the 1-bit mask.
  float bmu[BNB ? 8 : 1], biv[BNB ? 8 : 1], bsc[BNB ? 8 : 1], bsh[BNB ? 8 : 1];
  if (BNB && bnb) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t c = ncol_ok ? n + e : 0;
      bmu[e] = p.bnb_mean[c];
      biv[e] = p.bnb_inv[c];
      bsc[e] = (p.bnb_w ? p.bnb_w[c] : 1.f) * biv[e];
      bsh[e] = fmaf(-bmu[e], bsc[e], p.bnb_b ? p.bnb_b[c] : 0.f);
    }
  }
  float cs[8], cq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = cq[e] = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    EpiIn enext;  // the next batch's loads fly while this one is processed
    if ((RES || BNB) && b + 1 < NB) epi_load(b + 1, enext);
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int r = r0 + (b * UB + u) * RPI;
      if (r >= BM || r >= rows_valid || !ncol_ok) continue;
      const int64_t m = m0 + r;
      uint4 v = *reinterpret_cast<const uint4*>(smem + r * CS + cc * 8);
      bf16 e8[8];
      __builtin_memcpy(e8, &v, 16);
      if (RES) {
        bf16 r8[8];
        __builtin_memcpy(r8, &ecur.rv[u], 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float rf = (ecur.rmk[u] >> e) & 1u ? static_cast<float>(r8[e]) : 0.f;
          e8[e] = static_cast<bf16>(static_cast<float>(e8[e]) + rf);
        }
        __builtin_memcpy(&v, e8, 16);
      }
      *reinterpret_cast<uint4*>(p.c + (tapcls >= 0 ? dx_row(m, p.conv_h, p.conv_w, tapcls) : m) * p.ldc + n) = v;
      if (BNB && bnb) {
        bf16 x8[8];
        __builtin_memcpy(x8, &ecur.xv[u], 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xf = static_cast<float>(x8[e]);
          bool keep = (ecur.mk[u] >> e) & 1u;  // rm 3: the saved bit; 0xFF otherwise
          if (p.bnb_rm == 2) keep = fmaf(xf, bsc[e], bsh[e]) > 0.f;
          const float dd = keep ? static_cast<float>(e8[e]) : 0.f;
          cs[e] += dd;
          cq[e] = fmaf(dd, (xf - bmu[e]) * biv[e], cq[e]);
        }
      } else if (p.mode == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = static_cast<float>(e8[e]);
          cs[e] += f;
          cq[e] = fmaf(f, f, cq[e]);
        }
      }
    }
    if ((RES || BNB) && b + 1 < NB) ecur = enext;
  }
  if (p.mode == 1) {
    // lanes of a wave with equal cc differ in the bits above log2(CPR): butterfly them, then
    // combine the 4 waves through LDS and add one atomic per column per block
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

template <int BM, int BN, int BK, int ST, bool CONV, bool RES, bool AFF = false, bool BNB = false>
void launch_glds(GldsArgs a, hipStream_t s) {
  a.tiles_m = static_cast<int>((a.M + BM - 1) / BM);
  a.tiles_n = static_cast<int>((a.N + BN - 1) / BN);
  gemm_glds_kernel<BM, BN, BK, ST, CONV, RES, AFF, BNB><<<a.tiles_m * a.tiles_n, kThreads, 0, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}


// ---------------------------------------------------------------------------------------------
// Weight gradient: C[m][n] (+)= sum_k A[k][m] * B[k][n] with BOTH operands stored k-major-rows
// ([K][M] / [K][N], the pixel index k slowest: dY [pix][Cout] and X [pix][Cin] of NHWC
// activations), split over K (one 1-D grid over split x tile) into fp32 partials. The tiles [32 k][ROWS] go
// global -> LDS by LDS-DMA through a 3-stage ring and are read as MFMA fragments with
// ds_read_b64_tr_b16 (the transposed LDS read). Swizzle of a 16-B slot in a k-row,
// swz_tr(k): the 64 lanes of one tr read touch 16 k-rows x 32 B, and every 32 lanes (8 rows)
// land on 8 distinct 32-B bank groups. CONVB: B is the implicit im2col of a 3x3 / s1 / p1
// convolution (n = tap * Cin + ci, out-of-image taps read zeros).
template <int ROWS>
__device__ __forceinline__ int swz_tr(int k) {
  return ROWS == 128 ? (((k & 3) << 1) | (((k >> 3) & 1) << 3)) : (((((k >> 1) & 1) | (((k >> 3) & 1) << 1))) << 1);
}

struct WgradArgs {
  const bf16* a;  // [K][lda] (M contiguous)
  const bf16* b;  // [K][ldb] (N contiguous), or the NHWC image (CONVB)
  float* c;       // [splits][M][N] fp32 partials
  int64_t lda, ldb;
  int64_t M, N, K;
  int64_t k_per_split;
  int tiles_m, tiles_n;
  int conv_h, conv_w, conv_c;
  int remap;  // 1: XCD-aware (split, tile) order over the whole grid (default); 0: dispatch order
};

// Per-lane LDS-DMA loader of a [BK k-rows][ROWS] tile sequence (k advancing by BK per step).
// A lane's tile row and column (hence its swizzled chunk) never change, so every division is
// done once: the loop only bumps a pointer (plain operand) or a pixel index with its image
// position (CONVB, where the tap shift and channel of the lane's column are fixed too).
// MODE 0: plain [K][ld] rows; 1 (CONVB): the implicit 3x3 im2col; 2 (SUB): row k = pixel
// (img, ho, wo) of the [.][Ho][Wo] grid of a stride-2 1x1 convolution's output reads image row
// (img, 2ho, 2wo) of the NHWC input [.][H][W][ld] (H, W as the conv_h / conv_w arguments);
// 3: the implicit im2col of a 3x3 / stride 2 / pad 1 convolution (tap (dr, ds) of output pixel
// (img, ho, wo) reads input pixel (img, 2ho + dr, 2wo + ds), zeros outside the image).
template <int ROWS, int BK, int MODE>
struct TrLoader {
  static constexpr bool CONVB = MODE == 1 || MODE == 3, SUB = MODE == 2 || MODE == 3, S2 = MODE == 3;
  static constexpr int SPR = ROWS / 8;      // 16-B slots per k-row
  static constexpr int RPP = 64 / SPR;      // k-rows per 1 KiB piece
  static constexpr int PPW = BK / RPP / 4;  // pieces per wave (BK k-rows, 4 waves)
  const bf16* ptr[PPW];  // plain: address of (k, col); CONVB: image + ci; SUB: image + col
  int k[PPW];            // pixel / row index of the current step
  int h[PPW], w[PPW];    // CONVB: image position of pixel k; SUB: (ho, wo) of output pixel k
  int img[PPW];          // SUB: image of output pixel k
  int off[PPW];          // CONVB: tap shift in pixels, dr * W + ds
  int dr[PPW], ds[PPW];
  bool colok[PPW];

  __device__ __forceinline__ void init(const bf16* __restrict__ g, int64_t ld, int64_t cols, int64_t c0, int64_t kbeg,
                                       int H, int W, int C) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int row = (wave * PPW + j) * RPP + lane / SPR;
      const int chunk = (lane % SPR) ^ swz_tr<ROWS>(row);
      const int64_t col = c0 + chunk * 8;
      colok[j] = col < cols;
      k[j] = static_cast<int>(kbeg) + row;
      if (CONVB) {
        const int tap = static_cast<int>(col) / C;
        const int ci = static_cast<int>(col) - tap * C;
        dr[j] = tap / 3 - 1;
        ds[j] = tap % 3 - 1;
        off[j] = dr[j] * W + ds[j];
        ptr[j] = g + ci;
      }
      if (CONVB && !S2) {
        const int hw = k[j] % (H * W);
        h[j] = hw / W;
        w[j] = hw - h[j] * W;
      } else if (SUB) {
        const int ho = (H + 1) >> 1, wo = (W + 1) >> 1;
        if (!S2) ptr[j] = g + col;
        img[j] = k[j] / (ho * wo);
        const int r = k[j] - img[j] * (ho * wo);
        h[j] = r / wo;
        w[j] = r - h[j] * wo;
      } else {
        ptr[j] = g + static_cast<int64_t>(k[j]) * ld + col;
      }
    }
  }

  // issue this wave's pieces of the current step into lds_tile, then advance one step
  __device__ __forceinline__ void issue_next(bf16* lds_tile, int kend, int64_t ld, int H, int W, int C, int dh_step,
                                             int dw_step, int dimg_step = 0) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const void* src = g_zero_line;
      if (colok[j] && k[j] < kend) {
        if (S2) {
          const int hi = 2 * h[j] + dr[j], wi = 2 * w[j] + ds[j];
          if (static_cast<unsigned>(hi) < static_cast<unsigned>(H) && static_cast<unsigned>(wi) < static_cast<unsigned>(W))
            src = ptr[j] + ((static_cast<int64_t>(img[j]) * H + hi) * W + wi) * C;
        } else if (CONVB) {
          if (static_cast<unsigned>(h[j] + dr[j]) < static_cast<unsigned>(H) &&
              static_cast<unsigned>(w[j] + ds[j]) < static_cast<unsigned>(W))
            src = ptr[j] + static_cast<int64_t>(k[j] + off[j]) * C;
        } else if (SUB) {
          src = ptr[j] + ((static_cast<int64_t>(img[j]) * H + 2 * h[j]) * W + 2 * w[j]) * ld;
        } else {
          src = ptr[j];
        }
      }
      typedef __attribute__((address_space(3))) char lds_char;
      typedef __attribute__((address_space(1))) void gl_void;
      __builtin_amdgcn_global_load_lds((gl_void*)(src),
                                       (lds_char*)(reinterpret_cast<char*>(lds_tile) + (wave * PPW + j) * 1024), 16, 0, 0);
      k[j] += BK;
      if (CONVB && !S2) {  // pixel k -> k + BK: (h, w) += (BK / W mod H, BK % W) with one carry each
        w[j] += dw_step;
        h[j] += dh_step;
        if (w[j] >= W) {
          w[j] -= W;
          ++h[j];
        }
        if (h[j] >= H) h[j] -= H;
      } else if (SUB) {  // output pixel k -> k + BK over the (Ho, Wo) grid, carries into img
        const int ho = (H + 1) >> 1, wo = (W + 1) >> 1;
        img[j] += dimg_step;
        w[j] += dw_step;
        h[j] += dh_step;
        if (w[j] >= wo) {
          w[j] -= wo;
          ++h[j];
        }
        if (h[j] >= ho) {
          h[j] -= ho;
          ++img[j];
        }
      } else {
        ptr[j] += BK * ld;
      }
    }
  }
};

// fragment of 16 columns from r0 of a swizzled [BK][ROWS] tile: lane l holds
// tile[k = 32 * kh + 8 * (l >> 4) + j][r0 + (l & 15)], j = 0..7 (two ds_read_b64_tr_b16)
template <int ROWS>
__device__ __forceinline__ bf16x8 read_frag_tr(const bf16* __restrict__ tile, int r0, int kh = 0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, li = l & 15, q = li >> 2, p = li & 3;
  const int col = r0 + 4 * p;
  const int k0 = 32 * kh + 8 * g + q, k1 = k0 + 4;
  const bf16* a0 = tile + k0 * ROWS + (((col >> 3) ^ swz_tr<ROWS>(k0)) << 3) + (col & 7);
  const bf16* a1 = tile + k1 * ROWS + (((col >> 3) ^ swz_tr<ROWS>(k1)) << 3) + (col & 7);
  typedef short short4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4v lds_short4v;
  short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(a0));
  short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(a1));
  bf16x8 out;
  __builtin_memcpy(&out, &lo, 8);
  __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
  return out;
}

template <int BM, int BN, int kBK, int kStages, int BMODE>
__global__ __launch_bounds__(kThreads, 2) void gemm_wgrad_kernel(WgradArgs p) {
  constexpr bool CONVB = BMODE == 1;  // (BMODE 2 / 3: stride-2 gathers over the output grid)
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int A_ELEMS = BM * kBK, B_ELEMS = BN * kBK;
  constexpr int LPT = (BM + BN) * kBK / 2048;
  __shared__ __attribute__((aligned(16))) bf16 smem[kStages * (A_ELEMS + B_ELEMS)];
  auto sa = [&](int s) { return smem + s * A_ELEMS; };
  auto sb = [&](int s) { return smem + kStages * A_ELEMS + s * B_ELEMS; };
  // 1-D grid over (split, tile), XCD-aware and bijective over the whole grid: each XCD gets a
  // contiguous range of (split-major) ids, so the tiles of one K-split — which read the same
  // A / B rows — run on one XCD and share its L2 (blockIdx round-robins the XCDs otherwise)
  const int nt = p.tiles_m * p.tiles_n;
  const int total = static_cast<int>(gridDim.x);
  int lid = blockIdx.x;
  if (p.remap && total >= 8) {
    const int q = total / 8, r = total % 8, xcd = lid % 8, pos = lid / 8;
    lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int split = lid / nt, bid = lid - split * nt;
  const int tm = bid / p.tiles_n, tn = bid % p.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * BM, n0 = static_cast<int64_t>(tn) * BN;
  const int64_t kbeg = static_cast<int64_t>(split) * p.k_per_split;
  const int64_t kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  TrLoader<BM, kBK, 0> la;
  TrLoader<BN, kBK, BMODE> lb;
  const int H = p.conv_h, W = p.conv_w, C = p.conv_c;
  // per-step advance of a lane's pixel: CONVB over (H, W); SUB over the (Ho, Wo) output grid
  const int sho = (H + 1) >> 1, swo = (W + 1) >> 1;
  const int dw_step = CONVB ? kBK % W : (BMODE >= 2 ? (kBK % (sho * swo)) % swo : 0);
  const int dh_step = CONVB ? (kBK / W) % H : (BMODE >= 2 ? (kBK % (sho * swo)) / swo : 0);
  const int dimg_step = BMODE >= 2 ? kBK / (sho * swo) : 0;
  la.init(p.a, p.lda, p.M, m0, kbeg, 0, 1, 1);
  lb.init(p.b, p.ldb, p.N, n0, kbeg, H, W, C);
  const int kend32 = static_cast<int>(kend);
  auto issue = [&](int s) {
    la.issue_next(sa(s), kend32, p.lda, 0, 1, 1, 0, 0);
    lb.issue_next(sb(s), kend32, p.ldb, H, W, C, dh_step, dw_step, dimg_step);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = kend > kbeg ? static_cast<int>((kend - kbeg + kBK - 1) / kBK) : 0;
#pragma unroll
  for (int s = 0; s < kStages - 1; ++s)
    if (s < nk) issue(s);
  for (int t = 0; t < nk; ++t) {
    const int ahead = nk - 1 - t < kStages - 2 ? nk - 1 - t : kStages - 2;
    wait_tiles_ahead<LPT, kStages - 2>(ahead);
    __builtin_amdgcn_s_barrier();
    if (t + kStages - 1 < nk) issue((t + kStages - 1) % kStages);
    const bf16* ta = sa(t % kStages);
    const bf16* tb = sb(t % kStages);
#pragma unroll
    for (int kh = 0; kh < kBK / 32; ++kh) {
      bf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = read_frag_tr<BM>(ta, wm * WM + i * 16, kh);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = read_frag_tr<BN>(tb, wn * WN + j * 16, kh);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  // fp32 partial of this split: acc[i][j][r] is (row wm*WM + i*16 + 4*(lane>>4) + r, col wn*WN + j*16 + lane&15)
  float* c = p.c + static_cast<int64_t>(split) * p.M * p.N;
  const int col_in = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t n = n0 + wn * WN + j * 16 + col_in;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * WM + i * 16 + rq + r;
        if (m < p.M && n < p.N) c[m * p.N + n] = acc[i][j][r];
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Filter transposition for the input-gradient GEMMs: out[ci][t][co] = in[co][T-1-t][ci] for
// every tensor of a list (T = taps: 1 for a 1x1 filter, 9 for a 3x3 one, whose taps are then
// also flipped). One launch for up to kMaxXT filters; 64x64 (co x ci) tiles through LDS so
// both the reads and the writes are 128-B coalesced rows.
constexpr int kMaxXT = 40;
struct XposeArgs {
  uintptr_t src[kMaxXT];
  uintptr_t dst[kMaxXT];
  int co[kMaxXT], ci[kMaxXT], taps[kMaxXT];
  int32_t start[kMaxXT + 1];  // prefix of tiles per tensor
  int n;
};

__global__ __launch_bounds__(kThreads) void xpose_taps_kernel(XposeArgs a) {
  __shared__ bf16 tile[64][66];
  const int b = blockIdx.x;
  const int t = find_tensor(a.start, a.n, b);
  const int co = a.co[t], ci = a.ci[t], T = a.taps[t];
  const int tci = (ci + 63) / 64, tco = (co + 63) / 64;
  int rem = b - a.start[t];
  const int tap = rem / (tco * tci);
  rem -= tap * tco * tci;
  const int bco = rem / tci, bci = rem % tci;
  const bf16* __restrict__ src = reinterpret_cast<const bf16*>(a.src[t]);
  bf16* __restrict__ dst = reinterpret_cast<bf16*>(a.dst[t]);
  const int r = threadIdx.x / 4, c0 = (threadIdx.x % 4) * 16;
  // full 16-element runs in range with 16-B aligned rows (ci, co % 8 == 0): two 16-B loads /
  // stores per lane instead of 16 predicated 2-byte ones (the scalar form ran ~47 us per
  // ResNet-50 step's batch of 3x3 filters)
  {  // read rows co = bco*64 + r, 16 ci each, of source tap T-1-tap
    const int oc = bco * 64 + r;
    const int ic0 = bci * 64 + c0;
    const bf16* sp = src + (static_cast<int64_t>(oc) * T + (T - 1 - tap)) * ci + ic0;
    if (oc < co && ic0 + 16 <= ci && ci % 8 == 0) {
      bf16 v0[8], v1[8];
      load8(sp, v0);
      load8(sp + 8, v1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        tile[r][c0 + j] = v0[j];
        tile[r][c0 + 8 + j] = v1[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        tile[r][c0 + j] = (oc < co && ic0 + j < ci) ? sp[j] : static_cast<bf16>(0.f);
    }
  }
  __syncthreads();
  {  // write rows ci = bci*64 + r, 16 co each, of destination tap `tap`
    const int ic = bci * 64 + r;
    const int oc0 = bco * 64 + c0;
    if (ic < ci) {
      bf16* dp = dst + (static_cast<int64_t>(ic) * T + tap) * co + oc0;
      if (oc0 + 16 <= co && co % 8 == 0) {
        bf16 v0[8], v1[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v0[j] = tile[c0 + j][r];
          v1[j] = tile[c0 + 8 + j][r];
        }
        store8(dp, v0);
        store8(dp + 8, v1);
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (oc0 + j < co) dp[j] = tile[c0 + j][r];
      }
    }
  }
}
}  // namespace


int64_t s2_class_taps(int cls) { return static_cast<int64_t>(((cls >> 1) ? 2 : 1) * ((cls & 1) ? 2 : 1)); }

bool gemm_glds_supported(const GemmProblem& g) {
  const int64_t aff_c = g.conv_h > 0 ? g.conv_c : g.K;
  return g.a_kmajor && g.b_kmajor && g.mode <= 1 && (g.splits <= 1) &&
         (g.a_scale == nullptr || (aff_c <= kMaxAffC && g.res == nullptr && g.bnb_x == nullptr)) &&
         g.b_scale == nullptr && g.K % 8 == 0 && g.N % 8 == 0 && g.lda % 8 == 0 && g.ldb % 8 == 0 &&
         g.ldc % 8 == 0 && (g.res == nullptr || g.ldr % 8 == 0) &&
         (g.bnb_x == nullptr || (g.mode == 1 && g.ldc == g.N && g.bnb_mean != nullptr && g.bnb_inv != nullptr &&
                                 (g.bnb_rm == 0 || g.bnb_rm == 2 || (g.bnb_rm == 3 && g.bnb_mask != nullptr)))) &&
         // implicit 3x3 conv: C % 32 == 0 (a K tile inside one tap), or C % 8 == 0 with per-chunk taps
         // (no A affine then: its per-tile channel base assumes one tap per tile)
         (g.conv_h == 0 || ((g.conv_c % 32 == 0 || (g.conv_c % 8 == 0 && g.a_scale == nullptr && g.conv_c <= 8192)) &&
                            g.K == (g.conv_s >= 16 ? s2_class_taps(g.conv_s - 16) : 9LL) * g.conv_c &&
                            g.M < (1LL << 31))) &&
         // stride-2 input-gradient class: plain epilogue, C % 32 == 0 (a K tile inside one tap), K-major
         // flipped-transposed filter [N][9][conv_c] as B
         (g.conv_s < 16 || (g.conv_s < 20 && g.conv_h > 0 && g.conv_c % 32 == 0 && g.mode == 0 && g.res == nullptr &&
                            g.a_scale == nullptr && g.bnb_x == nullptr && g.ldb >= 9LL * g.conv_c &&
                            g.M % (static_cast<int64_t>(g.conv_h) * g.conv_w) == 0)) &&
         (g.conv_s != 2 || (g.conv_h > 0 && g.M % (static_cast<int64_t>((g.conv_h + 1) / 2) * ((g.conv_w + 1) / 2)) == 0)) &&
         (g.a_sub_h == 0 || (g.conv_h == 0 && g.a_kmajor && g.a_sub_w > 0 && g.M < (1LL << 31) &&
                             g.M % (static_cast<int64_t>((g.a_sub_h + 1) / 2) * ((g.a_sub_w + 1) / 2)) == 0)) &&
         (g.res_sub_h == 0 || (g.res != nullptr && g.res_mask == nullptr && g.res_sub_w > 0 && g.M < (1LL << 31) &&
                               g.M % (static_cast<int64_t>(g.res_sub_h) * g.res_sub_w) == 0));
}

void gemm_glds(const GemmProblem& g, hipStream_t stream) {
  if (!gemm_glds_supported(g)) throw std::runtime_error("gemm_glds: unsupported problem");
  GldsArgs a{};
  a.a = static_cast<const bf16*>(g.a);
  a.b = static_cast<const bf16*>(g.b);
  a.c = static_cast<bf16*>(g.c);
  a.res = static_cast<const bf16*>(g.res);
  a.stats = g.stats;
  a.lda = g.lda; a.ldb = g.ldb; a.ldc = g.ldc; a.ldr = g.ldr;
  a.M = g.M; a.N = g.N; a.K = g.K;
  a.mode = g.mode;
  a.conv_h = g.conv_h; a.conv_w = g.conv_w; a.conv_c = g.conv_c;
  a.bnb_x = static_cast<const bf16*>(g.bnb_x);
  a.bnb_w = g.bnb_w; a.bnb_b = g.bnb_b; a.bnb_mean = g.bnb_mean; a.bnb_inv = g.bnb_inv;
  a.bnb_mask = g.bnb_mask; a.bnb_rm = g.bnb_rm;
  a.a_scale = g.a_scale; a.a_shift = g.a_shift;
  a.res_mask = g.res_mask;
  a.res_sub_h = g.res_sub_h; a.res_sub_w = g.res_sub_w;
  a.a_sub_h = g.a_sub_h; a.a_sub_w = g.a_sub_w;
  a.conv_s = g.conv_s == 2 || (g.conv_s >= 16 && g.conv_s < 20) ? g.conv_s : 1;
  a.aff_c = static_cast<int>(g.conv_h > 0 ? g.conv_c : g.K);
  const bool aff = g.a_scale != nullptr;
  const bool bnb = g.bnb_x != nullptr;
  const bool conv = g.conv_h > 0, res = g.res != nullptr;
  // variant: 1 BK32/3 stages; 2 BK32/4; 3 BK64/2; 4 BK64/3; 5 BK32/2 (engine 3..6 / 9 force one).
  // Auto (measured on MI355X, ResNet-50 1x1 and 3x3 shapes): a 64-deep K-step in a 2-stage ring
  // (64 KiB at 128x128: 2 workgroups/CU) wins for the 3x3 convolutions and once K >= 1024;
  // shorter K (memory-bound 1x1 convolutions) prefers the 32-deep 3-stage ring (48 KiB:
  // 3 workgroups/CU).
  int var = g.engine >= 3 && g.engine <= 6 ? g.engine - 2 : (g.engine == 9 ? 5 : 0);
  // engine 7 / 8: 256x128 tiles (waves of 128x64: 25% less LDS fragment traffic per MFMA than
  // 64x64 waves), 32-deep 3-stage / 64-deep 2-stage ring; plain / residual / implicit-conv only
  const bool big = (g.engine == 7 || g.engine == 8) && !aff && !bnb && g.M > 128 && g.N > 64;
  if (big) {
    const bool k64 = g.engine == 8 && (!conv || g.conv_c % 64 == 0);
#define GB(BK, ST)                                                                                      \
  {                                                                                                    \
    if (conv) { if (res) launch_glds<256, 128, BK, ST, true, true>(a, stream); else launch_glds<256, 128, BK, ST, true, false>(a, stream); } \
    else { if (res) launch_glds<256, 128, BK, ST, false, true>(a, stream); else launch_glds<256, 128, BK, ST, false, false>(a, stream); } \
  }
    if (k64) GB(64, 2) else GB(32, 3)
#undef GB
    return;
  }
  // narrow channel counts (C % 32 != 0: per-chunk taps, e.g. the 48-channel DEQ cell, K = 432)
  // stay on 32-deep K steps: 64-deep ones measured slower on the DEQ cell's 28x28x48 input
  // gradient (34.1 vs 31.3 us per call, round 3)
  const bool k64ok = !conv || g.conv_c % 64 == 0;
  // K <= 64 (two 32-deep steps: all in flight after one wait anyway): a 2-stage ring, whose
  // smaller LDS footprint (the C staging tile sets it) fits a 4th workgroup per CU — measured
  // 153 -> 116 us on ResNet-50's 56x56 64->256 forward (scripts/bench_gemm_bw.py)
  // The stride-2 row gather (a_sub) likewise: 108 / 73 us vs 119 / 83 us with 3 stages on the
  // 56x56 256->512 and 28x28 512->1024 downsample convolutions (scripts/bench_ds.py).
  if (var == 0) var = ((conv || g.K >= 1024) && k64ok) ? 3 : ((g.K <= 64 || g.a_sub_h > 0) ? 5 : 1);
  if ((var == 3 || var == 4) && !k64ok) var = 1;
  // 128x128 tiles whenever both dimensions allow (measured: 128x64 tiles lose more to the lower
  // operand reuse than they win back from finer wave quantization)
  const bool bm128 = g.M > 64 && g.tile_m != 64;
  const bool bn128 = g.N > 64 && g.tile_n != 64;
#define GV(BM, BN, BK, ST)                                                                                \
  {                                                                                                      \
    if (aff) { if (conv) launch_glds<BM, BN, BK, ST, true, false, true>(a, stream); else launch_glds<BM, BN, BK, ST, false, false, true>(a, stream); } \
    else if (bnb) { if (conv) launch_glds<BM, BN, BK, ST, true, false, false, true>(a, stream);                    \
                    else if (res) launch_glds<BM, BN, BK, ST, false, true, false, true>(a, stream);                \
                    else launch_glds<BM, BN, BK, ST, false, false, false, true>(a, stream); }                      \
    else if (conv) { if (res) launch_glds<BM, BN, BK, ST, true, true>(a, stream); else launch_glds<BM, BN, BK, ST, true, false>(a, stream); } \
    else { if (res) launch_glds<BM, BN, BK, ST, false, true>(a, stream); else launch_glds<BM, BN, BK, ST, false, false>(a, stream); }    \
  }
#define GL(BM, BN)                          \
  {                                         \
    if (var == 1) GV(BM, BN, 32, 3)         \
    else if (var == 3) GV(BM, BN, 64, 2)    \
    else if (var == 4) GV(BM, BN, 64, 3)    \
    else if (var == 5) GV(BM, BN, 32, 2)    \
    else GV(BM, BN, 32, 4)                  \
  }
  if (bm128 && bn128) GL(128, 128)
  else if (bm128) GL(128, 64)
  else if (bn128) GL(64, 128)
  else GL(64, 64)
#undef GV
#undef GL
}

void gemm_wgrad(const void* a, const void* b, float* ws, int64_t lda, int64_t ldb, int64_t M, int64_t N, int64_t K,
                int splits, int conv_h, int conv_w, int conv_c, hipStream_t stream, int variant, int b_sub) {
  if (lda % 8 != 0 || ldb % 8 != 0 || M % 8 != 0 || N % 8 != 0 || splits < 1)
    throw std::runtime_error("gemm_wgrad: M, N, lda, ldb must be multiples of 8");
  if (conv_c > 0 && (conv_c % 8 != 0 || N != 9LL * conv_c))
    throw std::runtime_error("gemm_wgrad: implicit 3x3 B needs C % 8 == 0 and N == 9*C");
  const int64_t grid_px = b_sub ? static_cast<int64_t>((conv_h + 1) / 2) * ((conv_w + 1) / 2)
                                : static_cast<int64_t>(conv_h) * conv_w;
  if (b_sub && (conv_h <= 0 || conv_w <= 0 || (conv_c == 0 && N > ldb)))
    throw std::runtime_error("gemm_wgrad: the stride-2 B gather needs the input H, W and N <= ldb");
  if (K >= (1LL << 31) || (conv_h > 0 && K % grid_px != 0))
    throw std::runtime_error("gemm_wgrad: K must fit 31 bits (and be whole images for the implicit conv)");
  WgradArgs w{};
  w.a = static_cast<const bf16*>(a);
  w.b = static_cast<const bf16*>(b);
  w.c = ws;
  w.lda = lda; w.ldb = ldb; w.M = M; w.N = N; w.K = K;
  // variant 0/1: 32-deep K-step, 3-stage ring; 2: 64-deep, 2 stages. Split boundaries are
  // multiples of 64 for both (the Python side computes the same split count).
  const int64_t nk = (K + 63) / 64;
  w.k_per_split = (nk + splits - 1) / splits * 64;
  const int sp = static_cast<int>((K + w.k_per_split - 1) / w.k_per_split);
  w.conv_h = conv_h; w.conv_w = conv_w; w.conv_c = conv_c;
  w.remap = (variant & 4) ? 0 : 1;  // bit 2 of variant: plain dispatch order (A/B experiments)
  variant &= 3;
  const bool m128 = M > 64, n128 = N > 64;
#define WG(BM, BN)                                                                                      \
  {                                                                                                     \
    w.tiles_m = static_cast<int>((M + BM - 1) / BM);                                                   \
    w.tiles_n = static_cast<int>((N + BN - 1) / BN);                                                   \
    dim3 grid(w.tiles_m * w.tiles_n * sp);                                                              \
    if (variant == 2) {                                                                                 \
      if (b_sub && conv_c > 0) gemm_wgrad_kernel<BM, BN, 64, 2, 3><<<grid, kThreads, 0, stream>>>(w);   \
      else if (b_sub) gemm_wgrad_kernel<BM, BN, 64, 2, 2><<<grid, kThreads, 0, stream>>>(w);            \
      else if (conv_h > 0) gemm_wgrad_kernel<BM, BN, 64, 2, 1><<<grid, kThreads, 0, stream>>>(w);       \
      else gemm_wgrad_kernel<BM, BN, 64, 2, 0><<<grid, kThreads, 0, stream>>>(w);                       \
    } else {                                                                                            \
      if (b_sub && conv_c > 0) gemm_wgrad_kernel<BM, BN, 32, 3, 3><<<grid, kThreads, 0, stream>>>(w);   \
      else if (b_sub) gemm_wgrad_kernel<BM, BN, 32, 3, 2><<<grid, kThreads, 0, stream>>>(w);            \
      else if (conv_h > 0) gemm_wgrad_kernel<BM, BN, 32, 3, 1><<<grid, kThreads, 0, stream>>>(w);       \
      else gemm_wgrad_kernel<BM, BN, 32, 3, 0><<<grid, kThreads, 0, stream>>>(w);                       \
    }                                                                                                   \
  }
  if (m128 && n128) WG(128, 128)
  else if (m128) WG(128, 64)
  else if (n128) WG(64, 128)
  else WG(64, 64)
#undef WG
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void transpose_filters(const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst,
                       const std::vector<int>& co, const std::vector<int>& ci, const std::vector<int>& taps,
                       hipStream_t stream) {
  const size_t n = src.size();
  if (dst.size() != n || co.size() != n || ci.size() != n || taps.size() != n)
    throw std::runtime_error("transpose_filters: length mismatch");
  for (size_t i0 = 0; i0 < n; i0 += kMaxXT) {
    XposeArgs a{};
    a.n = static_cast<int>(n - i0 < static_cast<size_t>(kMaxXT) ? n - i0 : kMaxXT);
    int32_t tiles = 0;
    for (int i = 0; i < a.n; ++i) {
      a.src[i] = src[i0 + i];
      a.dst[i] = dst[i0 + i];
      a.co[i] = co[i0 + i];
      a.ci[i] = ci[i0 + i];
      a.taps[i] = taps[i0 + i];
      a.start[i] = tiles;
      tiles += a.taps[i] * ((a.co[i] + 63) / 64) * ((a.ci[i] + 63) / 64);
    }
    a.start[a.n] = tiles;
    if (tiles == 0) continue;
    xpose_taps_kernel<<<tiles, kThreads, 0, stream>>>(a);
    FLUXMPI_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace fluxmpi
