// Softmax attention (forward + backward) for short sequences (ViT: T = 197, head dim 64) — gfx950.
//
// Why kernels of our own: PyTorch-ROCm's flash backward (AOTriton bwd_kernel_dk_dv +
// bwd_kernel_dq + bwd_preprocess) takes ~740 us per ViT-B/16 block at batch 256 on MI355X
// (s49 trace, profiles/r1_vit_b16_s49.md) — ~4x its forward, far from the ~75 MB x 5 of
// operand traffic — and its forward output / three gradients need layout copies to and from
// the packed QKV projection (another ~170 us per block).
//
// Here the whole key (or query) range of one (batch, head) is swept by one workgroup in
// 32-row chunks staged through LDS (the next chunk's global loads in flight during the
// current one), the output is written in the [B, T, H, 64] layout the projection GEMM reads,
// and each gradient straight into its slot of the packed [B, T, 3, H, 64] gradient:
//
//   attn_fwd     one workgroup = (b, h, 64 queries), 4 waves x 16 queries, transposed
//                orientation S^T[key, q] = K . Q^T: each lane owns ONE query column, so the
//                online-softmax rescale of its O^T accumulators is a per-lane scalar;
//                O^T += V^T . P^T (V^T from a transposed LDS image). Writes O and the row
//                log-sum-exp (base 2, of the scaled scores) to an fp32 side buffer.
//   attn_bwd_dq  same decomposition: D = rowsum(dO * O) (written for the next kernel),
//                dS^T = P^T * (dO V^T - D)^T, dQ^T += K^T . dS^T.
//   attn_bwd_dkv one workgroup = (b, h, 64 keys), 4 waves x 16 keys, dK^T / dV^T held in
//                accumulators while the workgroup sweeps all queries:
//                S = Q K^T, P = exp2(S c - lse2), dP = dO V^T, dS = P (dP - D),
//                dV^T += dO^T P, dK^T += Q^T dS  (dO^T, Q^T from transposed LDS images).
//
// Masking of rows >= T: staged rows past the end are zero, so a padded key contributes
// nothing to O, dQ (its K^T / V^T columns are zero) or anything stored; only the softmax
// denominator of the forward needs an explicit mask, in the last chunk. Padded queries get
// lse = +inf in the dK/dV sweep (P = 0).
//
// MFMA: v_mfma_f32_16x16x32_bf16 (A[row l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][col l&15],
// C[row 4(l>>4)+r][col l&15]). An accumulator pair (rows 0-15, 16-31 of a 32-row chunk) is
// reused as the next B operand with k-slot j of lane group g <-> row 4g+j (j<4) and
// 16+4g+j-4 (j>=4); the A operand reads the same rows from a transposed LDS image as two
// 8-byte pieces.  1-D grid with an XCD-aware order (the blocks of one (b, h) share an L2).
#include <cmath>
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

constexpr int DH = 64;      // head dim
constexpr int CH = 32;      // rows per staged chunk
constexpr int LN = DH + 8;  // padded row (elements) of a [CH][DH] LDS image (144 B)
constexpr int LT = CH + 4;  // padded row of a transposed [DH][CH] image (72 B)
constexpr float kInf = __builtin_huge_valf();
constexpr float kLog2e = 1.4426950408889634f;

struct AttnBwdArgs {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  const bf16* o;
  const bf16* dout;
  bf16* o_out;  // forward output (same strides as o)
  bf16* dq;
  bf16* dk;
  bf16* dv;
  float* stats;              // [B][H][T][2] = (lse2 from attn_fwd, D)
  int64_t sq_b, sq_t;        // q/k/v/dq/dk/dv strides (head stride DH)
  int64_t so_b, so_t, so_h;  // o strides
  int64_t sg_b, sg_t;        // dout strides (head stride DH)
  int B, T, H, nblk;
  float scale;
  // resident backward pair (optional): per (b, part, wave) row, the column sums of the gradient
  // rows the wave wrote ([rows][3][H][64] fp32, rows = B * nblk * waves): the packed QKV bias
  // gradient is then one small reduce instead of a column-sum pass over dQKV (ops/linear.py)
  float* colpart;
};

__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// 2^x as the bare v_exp_f32 (exp2f adds a denormal range check and rescale around it: five
// more VALU instructions per element; softmax weights below 2^-126 may flush to zero)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// A operand from a transposed [DH][CH] image: row m, k-slots {4g..4g+3, 16+4g..16+4g+3}
__device__ __forceinline__ bf16x8 ld_tr(const bf16* img, int m, int g) {
  const bf16* p = img + m * LT;
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(p + 4 * g);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + 16 + 4 * g);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// B operand from an accumulator pair (rows 0-15 in a, 16-31 in b)
__device__ __forceinline__ bf16x8 pack(f32x4 a, f32x4 b) {
  return bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}

// (b, h, row block) of this workgroup; consecutive ids of one XCD take consecutive blocks
__device__ __forceinline__ void block_coords(const AttnBwdArgs& a, int& b, int& h, int& blk) {
  const int total = a.B * a.H * a.nblk;
  int id = blockIdx.x;
  if ((total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
  blk = id % a.nblk;
  const int bh = id / a.nblk;
  h = bh % a.H;
  b = bh / a.H;
}

// Staging of rows [r0, r0+CH) of a [T][DH] operand (row stride st), split into a global fetch
// into registers (issued one chunk ahead, so its latency hides behind the current chunk's
// MFMAs) and an LDS write: row-major image (if img) and transposed image (if tr); rows >= T
// are zero. 256 threads, one 16-byte piece each: thread t takes row t & 31, columns
// 8 (t >> 5) .. +7, so a wave's transposed 2-byte writes for one column cover 16 consecutive
// dwords per 32-lane half and the two halves land 16 banks apart.
__device__ __forceinline__ bf16x8 fetch(const bf16* base, int64_t st, int r0, int T) {
  const int r = threadIdx.x & 31, d0 = (threadIdx.x >> 5) * 8;
  bf16x8 x = {};
  if (r0 + r < T) x = ld8(base + static_cast<int64_t>(r0 + r) * st + d0);
  return x;
}

__device__ __forceinline__ void put(bf16x8 x, bf16* img, bf16* tr) {
  const int r = threadIdx.x & 31, d0 = (threadIdx.x >> 5) * 8;
  if (img) *reinterpret_cast<bf16x8*>(img + r * LN + d0) = x;
  if (tr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) tr[(d0 + j) * LT + r] = x[j];
  }
}

__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sK[CH * LN];
  __shared__ __attribute__((aligned(16))) bf16 sVt[DH * LT];
  int b, h, blk;
  block_coords(a, b, h, blk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, g = lane >> 4;
  const int qi = blk * 64 + w * 16 + col;
  const bool qok = qi < a.T;
  const int64_t qoff = b * a.sq_b + static_cast<int64_t>(qi) * a.sq_t + h * DH;
  const bf16* kbase = a.k + b * a.sq_b + h * DH;
  const bf16* vbase = a.v + b * a.sq_b + h * DH;
  bf16x8 qf[2] = {};
  if (qok) {
    qf[0] = ld8(a.q + qoff + 8 * g);
    qf[1] = ld8(a.q + qoff + 32 + 8 * g);
  }
  const int nch = (a.T + CH - 1) / CH;
  const float c2 = a.scale * kLog2e;
  float m = -kInf, l = 0.f;  // running max (uniform over the 4 lane groups of a column), partial sum
  f32x4 acc[4] = {};
  bf16x8 kx = fetch(kbase, a.sq_t, 0, a.T), vx = fetch(vbase, a.sq_t, 0, a.T);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();
    put(kx, sK, nullptr);
    put(vx, nullptr, sVt);
    __syncthreads();
    if (c + 1 < nch) {
      kx = fetch(kbase, a.sq_t, (c + 1) * CH, a.T);
      vx = fetch(vbase, a.sq_t, (c + 1) * CH, a.T);
    }
    f32x4 x[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const bf16* kp = sK + (kt * 16 + col) * LN + 8 * g;
      f32x4 s = {};
      s = mfma(ld8(kp), qf[0], s);
      s = mfma(ld8(kp + 32), qf[1], s);
      x[kt] = s * c2;
    }
    if ((c + 1) * CH > a.T) {  // last, partial chunk: padded keys leave the denominator
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (c * CH + kt * 16 + 4 * g + r >= a.T) x[kt][r] = -kInf;
    }
    float mx = fmaxf(fmaxf(fmaxf(x[0][0], x[0][1]), fmaxf(x[0][2], x[0][3])),
                     fmaxf(fmaxf(x[1][0], x[1][1]), fmaxf(x[1][2], x[1][3])));
    mx = xor_max<32>(xor_max<16>(mx));  // permlane swaps (common.h)
    const float mn = fmaxf(m, mx);  // finite from the first chunk on (key 0 is real)
    const float f = fast_exp2(m - mn);
    m = mn;
    l *= f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] *= f;
    f32x4 p[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[kt][r] = fast_exp2(x[kt][r] - m);
        l += p[kt][r];
      }
    const bf16x8 bop = pack(p[0], p[1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(ld_tr(sVt, dt * 16 + col, g), bop, acc[dt]);
  }
  l = butterfly_from<16>(l);  // permlane swaps (common.h)
  if (qok) {
    const float inv = 1.f / l;
    bf16* op = a.o_out + b * a.so_b + static_cast<int64_t>(qi) * a.so_t + h * a.so_h;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 o = {(bf16)(acc[dt][0] * inv), (bf16)(acc[dt][1] * inv), (bf16)(acc[dt][2] * inv),
                        (bf16)(acc[dt][3] * inv)};
      *reinterpret_cast<bf16x4*>(op + dt * 16 + 4 * g) = o;
    }
    if (g == 0) a.stats[((static_cast<int64_t>(b) * a.H + h) * a.T + qi) * 2] = m + __log2f(l);
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sK[CH * LN];
  __shared__ __attribute__((aligned(16))) bf16 sV[CH * LN];
  __shared__ __attribute__((aligned(16))) bf16 sKt[DH * LT];
  int b, h, blk;
  block_coords(a, b, h, blk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, g = lane >> 4;
  const int qi = blk * 64 + w * 16 + col;
  const bool qok = qi < a.T;
  const int64_t qoff = b * a.sq_b + static_cast<int64_t>(qi) * a.sq_t + h * DH;
  const bf16* kbase = a.k + b * a.sq_b + h * DH;
  const bf16* vbase = a.v + b * a.sq_b + h * DH;
  bf16x8 qf[2] = {}, gf[2] = {};
  float dsum = 0.f;
  if (qok) {
    qf[0] = ld8(a.q + qoff + 8 * g);
    qf[1] = ld8(a.q + qoff + 32 + 8 * g);
    const bf16* gp = a.dout + b * a.sg_b + static_cast<int64_t>(qi) * a.sg_t + h * DH;
    gf[0] = ld8(gp + 8 * g);
    gf[1] = ld8(gp + 32 + 8 * g);
    const bf16* op = a.o + b * a.so_b + static_cast<int64_t>(qi) * a.so_t + h * a.so_h;
    const bf16x8 o0 = ld8(op + 8 * g), o1 = ld8(op + 32 + 8 * g);
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum += (float)gf[0][j] * (float)o0[j] + (float)gf[1][j] * (float)o1[j];
  }
  dsum = butterfly_from<16>(dsum);  // permlane swaps (common.h)

  const int nch = (a.T + CH - 1) / CH;
  const float c2 = a.scale * kLog2e;
  float* st = a.stats + ((static_cast<int64_t>(b) * a.H + h) * a.T + (qok ? qi : 0)) * 2;
  const float lse = qok ? st[0] : 0.f;
  if (qok && g == 0) st[1] = dsum;
  bf16x8 kx;

  // pass 2: dQ^T[d, q] = sum over keys of K^T[d, key] dS^T[key, q]
  f32x4 acc[4] = {};
  kx = fetch(kbase, a.sq_t, 0, a.T);
  bf16x8 vx = fetch(vbase, a.sq_t, 0, a.T);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();
    put(kx, sK, sKt);
    put(vx, sV, nullptr);
    __syncthreads();
    if (c + 1 < nch) {
      kx = fetch(kbase, a.sq_t, (c + 1) * CH, a.T);
      vx = fetch(vbase, a.sq_t, (c + 1) * CH, a.T);
    }
    f32x4 ds[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const bf16* kp = sK + (kt * 16 + col) * LN + 8 * g;
      const bf16* vp = sV + (kt * 16 + col) * LN + 8 * g;
      f32x4 s = {}, dp = {};
      s = mfma(ld8(kp), qf[0], s);
      s = mfma(ld8(kp + 32), qf[1], s);
      dp = mfma(ld8(vp), gf[0], dp);
      dp = mfma(ld8(vp + 32), gf[1], dp);
#pragma unroll
      for (int r = 0; r < 4; ++r) ds[kt][r] = fast_exp2(fmaf(s[r], c2, -lse)) * (dp[r] - dsum);
    }
    const bf16x8 bop = pack(ds[0], ds[1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(ld_tr(sKt, dt * 16 + col, g), bop, acc[dt]);
  }
  if (qok) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 o = {(bf16)(acc[dt][0] * a.scale), (bf16)(acc[dt][1] * a.scale), (bf16)(acc[dt][2] * a.scale),
                        (bf16)(acc[dt][3] * a.scale)};
      *reinterpret_cast<bf16x4*>(a.dq + qoff + dt * 16 + 4 * g) = o;
    }
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sQ[CH * LN];
  __shared__ __attribute__((aligned(16))) bf16 sG[CH * LN];
  __shared__ __attribute__((aligned(16))) bf16 sQt[DH * LT];
  __shared__ __attribute__((aligned(16))) bf16 sGt[DH * LT];
  __shared__ float sL[CH], sD[CH];
  int b, h, blk;
  block_coords(a, b, h, blk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, g = lane >> 4;
  const int ki = blk * 64 + w * 16 + col;
  const bool kok = ki < a.T;
  const int64_t koff = b * a.sq_b + static_cast<int64_t>(ki) * a.sq_t + h * DH;
  bf16x8 kf[2] = {}, vf[2] = {};
  if (kok) {
    kf[0] = ld8(a.k + koff + 8 * g);
    kf[1] = ld8(a.k + koff + 32 + 8 * g);
    vf[0] = ld8(a.v + koff + 8 * g);
    vf[1] = ld8(a.v + koff + 32 + 8 * g);
  }
  const bf16* qbase = a.q + b * a.sq_b + h * DH;
  const bf16* gbase = a.dout + b * a.sg_b + h * DH;
  const float* st = a.stats + (static_cast<int64_t>(b) * a.H + h) * a.T * 2;
  const int nch = (a.T + CH - 1) / CH;
  const float c2 = a.scale * kLog2e;
  f32x4 accK[4] = {}, accV[4] = {};
  auto fetch_stats = [&](int c, float& lv, float& dv) {
    const int qq = c * CH + static_cast<int>(threadIdx.x);
    lv = kInf;
    dv = 0.f;
    if (threadIdx.x < CH && qq < a.T) {
      lv = st[2 * qq];
      dv = st[2 * qq + 1];
    }
  };
  bf16x8 qx = fetch(qbase, a.sq_t, 0, a.T), gx = fetch(gbase, a.sg_t, 0, a.T);
  float lx, dx;
  fetch_stats(0, lx, dx);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();
    put(qx, sQ, sQt);
    put(gx, sG, sGt);
    if (threadIdx.x < CH) {
      sL[threadIdx.x] = lx;
      sD[threadIdx.x] = dx;
    }
    __syncthreads();
    if (c + 1 < nch) {
      qx = fetch(qbase, a.sq_t, (c + 1) * CH, a.T);
      gx = fetch(gbase, a.sg_t, (c + 1) * CH, a.T);
      fetch_stats(c + 1, lx, dx);
    }
    f32x4 p[2], ds[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const bf16* qp = sQ + (qt * 16 + col) * LN + 8 * g;
      const bf16* gp = sG + (qt * 16 + col) * LN + 8 * g;
      f32x4 s = {}, dp = {};
      s = mfma(ld8(qp), kf[0], s);
      s = mfma(ld8(qp + 32), kf[1], s);
      dp = mfma(ld8(gp), vf[0], dp);
      dp = mfma(ld8(gp + 32), vf[1], dp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = qt * 16 + 4 * g + r;
        const float pv = fast_exp2(fmaf(s[r], c2, -sL[qq]));
        p[qt][r] = pv;
        ds[qt][r] = pv * (dp[r] - sD[qq]);
      }
    }
    const bf16x8 pb = pack(p[0], p[1]), db = pack(ds[0], ds[1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      accV[dt] = mfma(ld_tr(sGt, dt * 16 + col, g), pb, accV[dt]);
      accK[dt] = mfma(ld_tr(sQt, dt * 16 + col, g), db, accK[dt]);
    }
  }
  if (kok) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 v = {(bf16)accV[dt][0], (bf16)accV[dt][1], (bf16)accV[dt][2], (bf16)accV[dt][3]};
      const bf16x4 k = {(bf16)(accK[dt][0] * a.scale), (bf16)(accK[dt][1] * a.scale),
                        (bf16)(accK[dt][2] * a.scale), (bf16)(accK[dt][3] * a.scale)};
      *reinterpret_cast<bf16x4*>(a.dv + koff + dt * 16 + 4 * g) = v;
      *reinterpret_cast<bf16x4*>(a.dk + koff + dt * 16 + 4 * g) = k;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Forward with the whole (b, h) resident: one workgroup per (batch, head), one wave per 16
// queries (T <= 256: up to 16 waves). K and V of the head are staged ONCE into LDS by
// LDS-DMA (8-row x 128-B pieces, zero rows past T), so each is read from HBM exactly once
// (the 64-query-block kernel above re-stages them for every query block, and its last block
// of a T = 197 head holds 5 real queries of 64). A wave then computes all of its query
// column's scores S^T = K Q^T (every key tile), the exact softmax in registers (no online
// rescale: the whole row is there), and O^T = V^T P^T with V^T fragments taken by
// ds_read_b64_tr_b16 from the row-major V image (no transposed LDS writes).
// Chunk-slot swizzle of the 128-B-row images, slot = chunk ^ (row & 6): conflict-free for both
// reads under the instructions' real lane groups (MI355X_MICROARCH.md §LDS; model:
// scripts/lds_banks.py attention_swizzles): ds_read_b128's four NON-contiguous 16-lane groups
// ({0-3,12-15,20-27}, ...) of a row read (16 rows, chunks g / 4 + g) and ds_read_b64_tr_b16's two
// 32-lane halves of a transposed read (8 rows x one 32-B column pair). The previous swizzle,
// ((row >> 1) & 3) << 1 | ((row >> 3) & 1), was built for contiguous 16-lane groups: 2-way
// conflicts on every row read, measured 28-39 % of the attention kernels' LDS cycles
// (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/rd3t_attention_pmc.md).
constexpr int kResMaxT = 256;

__device__ __forceinline__ int swz_b(int r) { return r & 6; }
__device__ __forceinline__ int swz_k(int r) { return swz_b(r); }
__device__ __forceinline__ int swz_v(int r) { return swz_b(r); }

// 16-B row-read fragment (8 consecutive columns from logical chunk ch) of a swizzled image
__device__ __forceinline__ bf16x8 img_row(const char* img, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(img + row * 128 + ((ch ^ swz_b(row)) << 4));
}

// transposed fragment of a swizzled image for the accumulator-pair k order: lane l gets
// column c0 + (l & 15) of rows r0 + 4 (l >> 4) + j (j < 4) and r0 + 16 + 4 (l >> 4) + j - 4
__device__ __forceinline__ bf16x8 img_tr(const char* img, int r0, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const int ra = r0 + 4 * g + q, rb = ra + 16;
  const int ch = (c0 >> 3) + (p >> 1);
  const char* a0 = img + ra * 128 + ((ch ^ swz_b(ra)) << 4) + (p & 1) * 8;
  const char* a1 = img + rb * 128 + ((ch ^ swz_b(rb)) << 4) + (p & 1) * 8;
  typedef short short4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4v lds_short4v;
  short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(a0));
  short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(a1));
  bf16x8 out;
  __builtin_memcpy(&out, &lo, 8);
  __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
  return out;
}

__device__ __attribute__((aligned(16))) uint4 g_attn_zero[4];

// LDS-DMA of rows [0, rows) of a [T][64] head operand (row stride st) into a swizzled 128-B-row
// image; rows >= T read a zero line. Pieces are spread over the workgroup's waves.
template <bool V>
__device__ __forceinline__ void stage_rows(char* img, const bf16* __restrict__ base, int64_t st, int rows, int T) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int pc = wave; pc < rows / 8; pc += nw) {
    const int row = 8 * pc + (lane >> 3);
    const int chunk = (lane & 7) ^ (V ? swz_v(row) : swz_k(row));
    const void* src = row < T ? static_cast<const void*>(base + static_cast<int64_t>(row) * st + chunk * 8)
                              : static_cast<const void*>(g_attn_zero);
    typedef __attribute__((address_space(3))) char lds_char;
    typedef __attribute__((address_space(1))) void gl_void;
    __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(img + pc * 1024), 16, 0, 0);
  }
}

// (b, h, part) of this workgroup: a.nblk parts (row-tile ranges) per (b, h); the parts of one
// head get adjacent logical ids, on one XCD (their second staging of the head hits L2)
__device__ __forceinline__ void res_coords(const AttnBwdArgs& a, int& b, int& h, int& part) {
  int id = blockIdx.x;
  const int total = a.B * a.H * a.nblk;
  if ((total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
  part = id % a.nblk;
  const int bh = id / a.nblk;
  h = bh % a.H;
  b = bh / a.H;
}

// this wave's row of a.colpart, slot (0 q, 1 k, 2 v) and head h
__device__ __forceinline__ float* colpart_row(const AttnBwdArgs& a, int b, int h, int part, int w, int slot) {
  const int nw = blockDim.x >> 6;
  return a.colpart + (static_cast<int64_t>(b * a.nblk + part) * nw + w) * (3 * a.H * DH) + slot * a.H * DH + h * DH;
}

// sums over the wave's 16 rows (lane & 15) of acc[dt][r] = gradient[row][16 dt + 4 (lane >> 4) + r],
// rows with ok == false excluded; one float4 store per (dt, lane group)
__device__ __forceinline__ void colpart_store(float* row, const f32x4 (&acc)[4], float scale, bool ok) {
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const float keep = ok ? scale : 0.f;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    float4 v;
    v.x = row_sum16(acc[dt][0] * keep);
    v.y = row_sum16(acc[dt][1] * keep);
    v.z = row_sum16(acc[dt][2] * keep);
    v.w = row_sum16(acc[dt][3] * keep);
    if ((lane & 15) == 0) *reinterpret_cast<float4*>(row + 16 * dt + 4 * g) = v;
  }
}

__device__ __forceinline__ void colpart_zero(float* row) {
  const int lane = threadIdx.x & 63;
  row[lane] = 0.f;
}

// NT > 0: the head's key-tile count (TP / 16) at compile time — loops without runtime guards are
// straight-line code the scheduler can pipeline (LDS reads ahead of the MFMAs); 0: any T <= 256
// LDS: the V image's TP rows, then the K image's TP rows (2 TP x 128 B: 53,248 B at T = 197, so
// three workgroups fit a CU's 160 KB). The P V k-steps read V rows up to TV - 1 >= TP: those rows
// are the K image's first TV - TP (0 or 16) rows, finite values multiplied by P = 0 (keys >= TP).
template <int NT>
__global__ __launch_bounds__(1024) void attn_fwd_res_kernel(AttnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int TP = (a.T + 15) & ~15, TV = (a.T + 31) & ~31;
  char* vimg = smem;
  char* kimg = smem + TP * 128;
  int part, h, b;
  res_coords(a, b, h, part);
  stage_rows<false>(kimg, a.k + b * a.sq_b + h * DH, a.sq_t, TP, a.T);
  stage_rows<true>(vimg, a.v + b * a.sq_b + h * DH, a.sq_t, TP, a.T);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, g = lane >> 4;
  const int q0 = 16 * (part * (blockDim.x >> 6) + w);
  const int qi = q0 + col;
  const bool qok = qi < a.T;
  const int64_t qoff = b * a.sq_b + static_cast<int64_t>(qi) * a.sq_t + h * DH;
  bf16x8 qf[2] = {};
  if (qok) {  // issued before the wait: the Q loads fly with the staging DMA
    qf[0] = ld8(a.q + qoff + 8 * g);
    qf[1] = ld8(a.q + qoff + 32 + 8 * g);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (q0 >= a.T) return;  // wave-uniform: no partial EXEC below (the transposed reads need all lanes)
  const int nt = NT > 0 ? NT : TP / 16;
  const float c2 = a.scale * kLog2e;
  f32x4 x[kResMaxT / 16];
  float m = -kInf;
  float l = 0.f;
  f32x4 acc[4] = {};
  if constexpr (NT > 0) {
    // software-pipelined: the K fragments of tile kt + 2 are read while tile kt's MFMAs run, the
    // scale / mask / max pass comes after all S tiles (no VALU between the reads and the MFMAs),
    // and the V^T fragments of k-step ks + 1 are read during k-step ks (PMC rd3t: ~45 % of the
    // wave cycles waited on a one-tile-at-a-time read -> wait -> MFMA chain)
    constexpr int KS = (NT + 1) / 2;
    bf16x8 fk[2][2];
#pragma unroll
    for (int t = 0; t < (NT < 2 ? NT : 2); ++t) {
      fk[t][0] = img_row(kimg, 16 * t + col, g);
      fk[t][1] = img_row(kimg, 16 * t + col, 4 + g);
    }
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      f32x4 sacc = {};
      sacc = mfma(fk[kt & 1][0], qf[0], sacc);
      sacc = mfma(fk[kt & 1][1], qf[1], sacc);
      if (kt + 2 < NT) {
        fk[kt & 1][0] = img_row(kimg, 16 * (kt + 2) + col, g);
        fk[kt & 1][1] = img_row(kimg, 16 * (kt + 2) + col, 4 + g);
      }
      x[kt] = sacc;
    }
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * kt + 4 * g + r;
        x[kt][r] = (kt < NT - 1 || key < a.T) ? x[kt][r] * c2 : -kInf;  // only the last tile pads
        m = fmaxf(m, x[kt][r]);
      }
    }
    m = xor_max<32>(xor_max<16>(m));  // permlane swaps (common.h)
#pragma unroll
    for (int kt = 0; kt < 2 * KS; ++kt) {
      if (kt < NT) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = fast_exp2(x[kt][r] - m);  // -inf (padded key) -> 0
          x[kt][r] = pv;
          l += pv;
        }
      } else {
        x[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    l = butterfly_from<16>(l);  // permlane swaps (common.h)
    bf16x8 fv[2][4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) fv[0][dt] = img_tr(vimg, 0, 16 * dt);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) fv[(ks + 1) & 1][dt] = img_tr(vimg, 32 * (ks + 1), 16 * dt);
      }
      const bf16x8 bop = pack(x[2 * ks], x[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(fv[ks & 1][dt], bop, acc[dt]);
    }
  } else {
#pragma unroll
    for (int kt = 0; kt < (NT > 0 ? NT : kResMaxT / 16); ++kt) {
      x[kt] = f32x4{-kInf, -kInf, -kInf, -kInf};
      if (NT > 0 || kt < nt) {
        const int row = 16 * kt + col;
        f32x4 s = {};
        s = mfma(img_row(kimg, row, g), qf[0], s);
        s = mfma(img_row(kimg, row, 4 + g), qf[1], s);
        if (16 * kt + 16 <= a.T) {  // wave-uniform: only the last tile has padded keys
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            x[kt][r] = s[r] * c2;
            m = fmaxf(m, x[kt][r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = 16 * kt + 4 * g + r;
            x[kt][r] = key < a.T ? s[r] * c2 : -kInf;
            m = fmaxf(m, x[kt][r]);
          }
        }
      }
    }
    m = xor_max<32>(xor_max<16>(m));  // permlane swaps (common.h)
#pragma unroll
    for (int kt = 0; kt < (NT > 0 ? NT : kResMaxT / 16); ++kt) {
      if (NT > 0 || kt < nt) {  // wave-uniform
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = fast_exp2(x[kt][r] - m);  // -inf (padded key) -> 0
          x[kt][r] = pv;
          l += pv;
        }
      } else {
        x[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    l = butterfly_from<16>(l);  // permlane swaps (common.h)
    // O^T[d][q] = sum over keys of V^T[d][key] P^T[key][q]; k-step ks covers keys 32ks .. +31 in
    // the accumulator-pair order (j < 4: 32ks + 4g + j, j >= 4: 32ks + 16 + 4g + j - 4)
#pragma unroll
    for (int ks = 0; ks < (NT > 0 ? (NT + 1) / 2 : kResMaxT / 32); ++ks) {
      if (NT > 0 || 32 * ks < TV) {
        const bf16x8 bop = pack(x[2 * ks], x[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(img_tr(vimg, 32 * ks, 16 * dt), bop, acc[dt]);
      }
    }
  }
  if (qok) {
    const float inv = 1.f / l;
    bf16* op = a.o_out + b * a.so_b + static_cast<int64_t>(qi) * a.so_t + h * a.so_h;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 o = {(bf16)(acc[dt][0] * inv), (bf16)(acc[dt][1] * inv), (bf16)(acc[dt][2] * inv),
                        (bf16)(acc[dt][3] * inv)};
      *reinterpret_cast<bf16x4*>(op + dt * 16 + 4 * g) = o;
    }
    if (g == 0) a.stats[((static_cast<int64_t>(b) * a.H + h) * a.T + qi) * 2] = m + __log2f(l);
  }
}

// Backward with the head resident (T <= 256), two kernels like the blocked pair above:
//   attn_bwd_dq_res   K, V images; one wave per 16 queries: D = rowsum(dO * O) (written to
//                     stats[.., 1] for the next kernel), S^T = K Q^T, dP^T = V dO^T,
//                     dS^T = P^T (dP^T - D), dQ^T = K^T dS^T (K^T by transposed reads).
//   attn_bwd_dkv_res  Q, dO images + the per-query lse / D rows; one wave per 16 keys:
//                     S = Q K^T, dP = dO V^T, dS = P (dP - D), dV^T += dO^T P, dK^T += Q^T dS.
// Each image is read by rows (ds_read_b128) and by columns (ds_read_b64_tr_b16), one
// swizzle for both (swz_b). Padded rows (>= T) are zero; padded queries get lse = +inf.
template <int NT>
__global__ __launch_bounds__(1024) void attn_bwd_dq_res_kernel(AttnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int TP = (a.T + 15) & ~15, TV = (a.T + 31) & ~31;
  char* kimg = smem;              // TV rows (transposed reads in k-steps of 32 keys)
  char* vimg = smem + TV * 128;   // TP rows
  int part, h, b;
  res_coords(a, b, h, part);
  stage_rows<false>(kimg, a.k + b * a.sq_b + h * DH, a.sq_t, TV, a.T);
  stage_rows<false>(vimg, a.v + b * a.sq_b + h * DH, a.sq_t, TP, a.T);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, g = lane >> 4;
  const int q0 = 16 * (part * (blockDim.x >> 6) + w);
  const int qi = q0 + col;
  const bool qok = qi < a.T;
  const int64_t qoff = b * a.sq_b + static_cast<int64_t>(qi) * a.sq_t + h * DH;
  bf16x8 qf[2] = {}, gf[2] = {}, o0 = {}, o1 = {};
  float lse = 0.f;
  float* st = a.stats + ((static_cast<int64_t>(b) * a.H + h) * a.T + (qok ? qi : 0)) * 2;
  if (qok) {
    qf[0] = ld8(a.q + qoff + 8 * g);
    qf[1] = ld8(a.q + qoff + 32 + 8 * g);
    const bf16* gp = a.dout + b * a.sg_b + static_cast<int64_t>(qi) * a.sg_t + h * DH;
    gf[0] = ld8(gp + 8 * g);
    gf[1] = ld8(gp + 32 + 8 * g);
    const bf16* op = a.o + b * a.so_b + static_cast<int64_t>(qi) * a.so_t + h * a.so_h;
    o0 = ld8(op + 8 * g);
    o1 = ld8(op + 32 + 8 * g);
    lse = st[0];
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (q0 >= a.T) {  // wave-uniform
    if (a.colpart != nullptr) colpart_zero(colpart_row(a, b, h, part, w, 0));
    return;
  }
  float dsum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) dsum += (float)gf[0][j] * (float)o0[j] + (float)gf[1][j] * (float)o1[j];
  dsum = butterfly_from<16>(dsum);  // permlane swaps (common.h)
  if (qok && g == 0) st[1] = dsum;
  const int nt = NT > 0 ? NT : TP / 16;
  const float c2 = a.scale * kLog2e;
  f32x4 ds[kResMaxT / 16];
  f32x4 acc[4] = {};
  if constexpr (NT > 0) {
    // software-pipelined like the forward: the K / V fragments of tile kt + 2 are read while tile
    // kt's MFMAs run; the K^T fragments of k-step ks + 1 during k-step ks
    constexpr int KS = (NT + 1) / 2;
    if constexpr (NT & 1) ds[NT] = f32x4{0.f, 0.f, 0.f, 0.f};  // odd NT: the last k-step's pad half
    bf16x8 fk[2][2], fw[2][2];
#pragma unroll
    for (int t = 0; t < (NT < 2 ? NT : 2); ++t) {
      fk[t][0] = img_row(kimg, 16 * t + col, g);
      fk[t][1] = img_row(kimg, 16 * t + col, 4 + g);
      fw[t][0] = img_row(vimg, 16 * t + col, g);
      fw[t][1] = img_row(vimg, 16 * t + col, 4 + g);
    }
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      f32x4 sv = {}, dp = {};
      sv = mfma(fk[kt & 1][0], qf[0], sv);
      sv = mfma(fk[kt & 1][1], qf[1], sv);
      dp = mfma(fw[kt & 1][0], gf[0], dp);
      dp = mfma(fw[kt & 1][1], gf[1], dp);
      if (kt + 2 < NT) {
        fk[kt & 1][0] = img_row(kimg, 16 * (kt + 2) + col, g);
        fk[kt & 1][1] = img_row(kimg, 16 * (kt + 2) + col, 4 + g);
        fw[kt & 1][0] = img_row(vimg, 16 * (kt + 2) + col, g);
        fw[kt & 1][1] = img_row(vimg, 16 * (kt + 2) + col, 4 + g);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * kt + 4 * g + r;
        ds[kt][r] = (kt < NT - 1 || key < a.T) ? fast_exp2(fmaf(sv[r], c2, -lse)) * (dp[r] - dsum) : 0.f;
      }
    }
    bf16x8 ft[2][4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) ft[0][dt] = img_tr(kimg, 0, 16 * dt);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) ft[(ks + 1) & 1][dt] = img_tr(kimg, 32 * (ks + 1), 16 * dt);
      }
      const bf16x8 bop = pack(ds[2 * ks], ds[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(ft[ks & 1][dt], bop, acc[dt]);
    }
  } else {
#pragma unroll
  for (int kt = 0; kt < kResMaxT / 16; ++kt) {
    ds[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (NT > 0 || kt < nt) {
      const int row = 16 * kt + col;
      f32x4 sv = {}, dp = {};
      sv = mfma(img_row(kimg, row, g), qf[0], sv);
      sv = mfma(img_row(kimg, row, 4 + g), qf[1], sv);
      dp = mfma(img_row(vimg, row, g), gf[0], dp);
      dp = mfma(img_row(vimg, row, 4 + g), gf[1], dp);
      if (16 * kt + 16 <= a.T) {  // wave-uniform
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[kt][r] = fast_exp2(fmaf(sv[r], c2, -lse)) * (dp[r] - dsum);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = 16 * kt + 4 * g + r;
          ds[kt][r] = key < a.T ? fast_exp2(fmaf(sv[r], c2, -lse)) * (dp[r] - dsum) : 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int ks = 0; ks < kResMaxT / 32; ++ks) {
    if (32 * ks < TV) {
      const bf16x8 bop = pack(ds[2 * ks], ds[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(img_tr(kimg, 32 * ks, 16 * dt), bop, acc[dt]);
    }
  }
  }
  if (qok) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 o = {(bf16)(acc[dt][0] * a.scale), (bf16)(acc[dt][1] * a.scale), (bf16)(acc[dt][2] * a.scale),
                        (bf16)(acc[dt][3] * a.scale)};
      *reinterpret_cast<bf16x4*>(a.dq + qoff + dt * 16 + 4 * g) = o;
    }
  }
  if (a.colpart != nullptr) colpart_store(colpart_row(a, b, h, part, w, 0), acc, a.scale, qok);
}

// PIPE (NT > 0 only): explicit software pipeline of the k-steps (FLUXMPI_ATTN_DKV_PIPE)
template <int NT, int PIPE = 0>
__global__ __launch_bounds__(1024) void attn_bwd_dkv_res_kernel(AttnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int TV = (a.T + 31) & ~31;
  char* qimg = smem;               // TV rows
  char* gimg = smem + TV * 128;    // TV rows
  float* sL = reinterpret_cast<float*>(smem + 2 * TV * 128);
  float* sD = sL + TV;
  int part, h, b;
  res_coords(a, b, h, part);
  stage_rows<false>(qimg, a.q + b * a.sq_b + h * DH, a.sq_t, TV, a.T);
  stage_rows<false>(gimg, a.dout + b * a.sg_b + h * DH, a.sg_t, TV, a.T);
  const float* st = a.stats + (static_cast<int64_t>(b) * a.H + h) * a.T * 2;
  for (int qq = threadIdx.x; qq < TV; qq += blockDim.x) {
    sL[qq] = qq < a.T ? st[2 * qq] : kInf;
    sD[qq] = qq < a.T ? st[2 * qq + 1] : 0.f;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, g = lane >> 4;
  const int k0 = 16 * (part * (blockDim.x >> 6) + w);
  const int ki = k0 + col;
  const bool kok = ki < a.T;
  const int64_t koff = b * a.sq_b + static_cast<int64_t>(ki) * a.sq_t + h * DH;
  bf16x8 kf[2] = {}, vf[2] = {};
  if (kok) {
    kf[0] = ld8(a.k + koff + 8 * g);
    kf[1] = ld8(a.k + koff + 32 + 8 * g);
    vf[0] = ld8(a.v + koff + 8 * g);
    vf[1] = ld8(a.v + koff + 32 + 8 * g);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (k0 >= a.T) {  // wave-uniform
    if (a.colpart != nullptr) {
      colpart_zero(colpart_row(a, b, h, part, w, 1));
      colpart_zero(colpart_row(a, b, h, part, w, 2));
    }
    return;
  }
  const float c2 = a.scale * kLog2e;
  f32x4 accK[4] = {}, accV[4] = {};
  auto kstep = [&](int ks) __attribute__((always_inline)) {
    f32x4 p[2], dsv[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = 32 * ks + 16 * half + col;  // query row of the A fragment
      f32x4 sv = {}, dp = {};
      sv = mfma(img_row(qimg, row, g), kf[0], sv);
      sv = mfma(img_row(qimg, row, 4 + g), kf[1], sv);
      dp = mfma(img_row(gimg, row, g), vf[0], dp);
      dp = mfma(img_row(gimg, row, 4 + g), vf[1], dp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = 32 * ks + 16 * half + 4 * g + r;
        const float pv = fast_exp2(fmaf(sv[r], c2, -sL[qq]));  // padded query: lse = +inf -> 0
        p[half][r] = pv;
        dsv[half][r] = pv * (dp[r] - sD[qq]);
      }
    }
    const bf16x8 pb = pack(p[0], p[1]), db = pack(dsv[0], dsv[1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      accV[dt] = mfma(img_tr(gimg, 32 * ks, 16 * dt), pb, accV[dt]);
      accK[dt] = mfma(img_tr(qimg, 32 * ks, 16 * dt), db, accK[dt]);
    }
  };
  if constexpr (NT > 0 && PIPE) {
    // explicit pipeline: a k-step's row fragments are reloaded for the next k-step as soon as its
    // S / dP MFMAs have read them, its transposed fragments are issued before the softmax VALU,
    // so the LDS latency hides behind the VALU and the other half's MFMAs
    constexpr int KS = (NT + 1) / 2;
    bf16x8 fr[2][4];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = 16 * half + col;
      fr[half][0] = img_row(qimg, row, g);
      fr[half][1] = img_row(qimg, row, 4 + g);
      fr[half][2] = img_row(gimg, row, g);
      fr[half][3] = img_row(gimg, row, 4 + g);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      f32x4 sv[2], dp[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        sv[half] = mfma(fr[half][0], kf[0], f32x4{0.f, 0.f, 0.f, 0.f});
        sv[half] = mfma(fr[half][1], kf[1], sv[half]);
        dp[half] = mfma(fr[half][2], vf[0], f32x4{0.f, 0.f, 0.f, 0.f});
        dp[half] = mfma(fr[half][3], vf[1], dp[half]);
        if (ks + 1 < KS) {
          const int row = 32 * (ks + 1) + 16 * half + col;
          fr[half][0] = img_row(qimg, row, g);
          fr[half][1] = img_row(qimg, row, 4 + g);
          fr[half][2] = img_row(gimg, row, g);
          fr[half][3] = img_row(gimg, row, 4 + g);
        }
      }
      bf16x8 tg[4], tq[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        tg[dt] = img_tr(gimg, 32 * ks, 16 * dt);
        tq[dt] = img_tr(qimg, 32 * ks, 16 * dt);
      }
      f32x4 p[2], dsv[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const float4 lv = *reinterpret_cast<const float4*>(sL + 32 * ks + 16 * half + 4 * g);
        const float4 dv = *reinterpret_cast<const float4*>(sD + 32 * ks + 16 * half + 4 * g);
        const float lq[4] = {lv.x, lv.y, lv.z, lv.w}, dq[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = fast_exp2(fmaf(sv[half][r], c2, -lq[r]));  // padded query: lse = +inf -> 0
          p[half][r] = pv;
          dsv[half][r] = pv * (dp[half][r] - dq[r]);
        }
      }
      const bf16x8 pb = pack(p[0], p[1]), db = pack(dsv[0], dsv[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        accV[dt] = mfma(tg[dt], pb, accV[dt]);
        accK[dt] = mfma(tq[dt], db, accK[dt]);
      }
    }
  } else if constexpr (NT > 0) {  // compile-time trip count: fully unrolled, next k-step's reads hoisted
#pragma unroll
    for (int ks = 0; ks < (NT + 1) / 2; ++ks) kstep(ks);
  } else {
#pragma unroll 2
    for (int ks = 0; ks < TV / 32; ++ks) kstep(ks);
  }
  if (kok) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 v = {(bf16)accV[dt][0], (bf16)accV[dt][1], (bf16)accV[dt][2], (bf16)accV[dt][3]};
      const bf16x4 k = {(bf16)(accK[dt][0] * a.scale), (bf16)(accK[dt][1] * a.scale),
                        (bf16)(accK[dt][2] * a.scale), (bf16)(accK[dt][3] * a.scale)};
      *reinterpret_cast<bf16x4*>(a.dv + koff + dt * 16 + 4 * g) = v;
      *reinterpret_cast<bf16x4*>(a.dk + koff + dt * 16 + 4 * g) = k;
    }
  }
  if (a.colpart != nullptr) {
    colpart_store(colpart_row(a, b, h, part, w, 1), accK, a.scale, kok);
    colpart_store(colpart_row(a, b, h, part, w, 2), accV, 1.f, kok);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused backward, one workgroup per (batch, head), one wave per 16 keys / 16 queries (NT waves):
//   phase 1  the dK / dV sweep of attn_bwd_dkv_res (each wave: its 16 keys against every query in
//            k-steps of 32: S = Q K^T, dP = dO V^T, P, dS = P (dP - D), dV^T += dO^T P,
//            dK^T += Q^T dS) that ALSO writes dS into an LDS image [query][key] (bf16);
//   phase 2  with K staged into the Q image's slot: dQ^T = K^T dS^T per wave of 16 queries (A = K^T
//            by transposed reads of the K image, B = dS^T from two 8-B reads of a dS row, in the
//            accumulator-pair k order of img_tr).
// S, P, dP and dS are computed ONCE (the dq / dkv pair computes S and dP in both kernels), Q, K, V,
// dO and O are read once, and D = rowsum(dO * O) is formed in the prologue (no stats round trip).
// LDS: Q (then K) and dO images 2 x TV x 128 B, the dS image 16 NT x 464 B, lse / D 2 x TV floats:
// 152 KB at T = 197, one workgroup of NT = 13 waves per CU (the pair holds 2 x 7).
// dS rows are 464 B (116 dwords = 4 x 29 mod 64: a 32-lane half of the phase-2 ds_read_b64 pair
// touches 16 rows x 2 groups on distinct 4-dword bank slots); keys >= 16 NT are zero columns (their
// K rows are zero, and 0 * uninitialised could be NaN).
constexpr int kDsRow = 464;

template <int NT>
__global__ __launch_bounds__(1024) void attn_bwd_fused_kernel(AttnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TV = ((16 * NT + 31) / 32) * 32;  // key / query rows of the images (224 at NT = 13)
  constexpr int NQ = 16 * NT;                      // dS rows = queries the waves own (208)
  constexpr int KS = TV / 32;
  char* qimg = smem;               // phase 1: Q image; phase 2: K image
  char* gimg = smem + TV * 128;    // dO image
  char* dsimg = smem + 2 * TV * 128;
  float* sL = reinterpret_cast<float*>(dsimg + NQ * kDsRow);
  float* sD = sL + TV;
  int part, h, b;
  res_coords(a, b, h, part);  // a.nblk == 1
  stage_rows<false>(qimg, a.q + b * a.sq_b + h * DH, a.sq_t, TV, a.T);
  stage_rows<false>(gimg, a.dout + b * a.sg_b + h * DH, a.sg_t, TV, a.T);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, g = lane >> 4;
  // zero dS columns NQ .. TV - 1 of every row (32 B per row: two 16-B pieces)
  for (int i = threadIdx.x; i < NQ * 2; i += blockDim.x)
    *reinterpret_cast<uint4*>(dsimg + (i >> 1) * kDsRow + NQ * 2 + (i & 1) * 16) = uint4{0, 0, 0, 0};
  // phase-1 keys of this wave
  const int k0 = 16 * w, ki = k0 + col;
  const bool kok = ki < a.T;
  const int64_t koff = b * a.sq_b + static_cast<int64_t>(ki) * a.sq_t + h * DH;
  bf16x8 kf[2] = {}, vf[2] = {};
  if (kok) {
    kf[0] = ld8(a.k + koff + 8 * g);
    kf[1] = ld8(a.k + koff + 32 + 8 * g);
    vf[0] = ld8(a.v + koff + 8 * g);
    vf[1] = ld8(a.v + koff + 32 + 8 * g);
  }
  // phase-2 queries of this wave: D = rowsum(dO * O) and lse into LDS for every query
  const int q0 = 16 * w, qi = q0 + col;
  const bool qok = qi < a.T;
  const int64_t qoff = b * a.sq_b + static_cast<int64_t>(qi) * a.sq_t + h * DH;
  bf16x8 gf[2] = {}, o0 = {}, o1 = {};
  float lse = kInf;
  if (qok) {
    const bf16* gp = a.dout + b * a.sg_b + static_cast<int64_t>(qi) * a.sg_t + h * DH;
    gf[0] = ld8(gp + 8 * g);
    gf[1] = ld8(gp + 32 + 8 * g);
    const bf16* op = a.o + b * a.so_b + static_cast<int64_t>(qi) * a.so_t + h * a.so_h;
    o0 = ld8(op + 8 * g);
    o1 = ld8(op + 32 + 8 * g);
    lse = a.stats[((static_cast<int64_t>(b) * a.H + h) * a.T + qi) * 2];
  }
  float dsum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) dsum += (float)gf[0][j] * (float)o0[j] + (float)gf[1][j] * (float)o1[j];
  dsum = butterfly_from<16>(dsum);  // over the 4 lane groups of the query
  if (g == 0) {
    sL[qi] = lse;
    sD[qi] = qok ? dsum : 0.f;
  }
  for (int qq = NQ + threadIdx.x; qq < TV; qq += blockDim.x) {
    sL[qq] = kInf;
    sD[qq] = 0.f;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  // ---- phase 1: dK^T, dV^T of this wave's keys; dS into the image
  const float c2 = a.scale * kLog2e;
  f32x4 accK[4] = {}, accV[4] = {};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    f32x4 p[2], dsv[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = 32 * ks + 16 * half + col;  // query row of the A fragment
      f32x4 sv = {}, dp = {};
      sv = mfma(img_row(qimg, row, g), kf[0], sv);
      sv = mfma(img_row(qimg, row, 4 + g), kf[1], sv);
      dp = mfma(img_row(gimg, row, g), vf[0], dp);
      dp = mfma(img_row(gimg, row, 4 + g), vf[1], dp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = 32 * ks + 16 * half + 4 * g + r;
        const float pv = fast_exp2(fmaf(sv[r], c2, -sL[qq]));  // padded query: lse = +inf -> 0
        p[half][r] = pv;
        dsv[half][r] = pv * (dp[r] - sD[qq]);
      }
      if (32 * ks + 16 * half < NQ) {  // compile-time: rows past the waves' queries are not in the image
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<bf16*>(dsimg + (32 * ks + 16 * half + 4 * g + r) * kDsRow + (k0 + col) * 2) =
              static_cast<bf16>(dsv[half][r]);
      }
    }
    const bf16x8 pb = pack(p[0], p[1]), db = pack(dsv[0], dsv[1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      accV[dt] = mfma(img_tr(gimg, 32 * ks, 16 * dt), pb, accV[dt]);
      accK[dt] = mfma(img_tr(qimg, 32 * ks, 16 * dt), db, accK[dt]);
    }
  }
  if (kok) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 v = {(bf16)accV[dt][0], (bf16)accV[dt][1], (bf16)accV[dt][2], (bf16)accV[dt][3]};
      const bf16x4 k = {(bf16)(accK[dt][0] * a.scale), (bf16)(accK[dt][1] * a.scale),
                        (bf16)(accK[dt][2] * a.scale), (bf16)(accK[dt][3] * a.scale)};
      *reinterpret_cast<bf16x4*>(a.dv + koff + dt * 16 + 4 * g) = v;
      *reinterpret_cast<bf16x4*>(a.dk + koff + dt * 16 + 4 * g) = k;
    }
  }
  if (a.colpart != nullptr) {
    colpart_store(colpart_row(a, b, h, 0, w, 1), accK, a.scale, kok);
    colpart_store(colpart_row(a, b, h, 0, w, 2), accV, 1.f, kok);
  }
  __syncthreads();  // dS complete, the Q image's last reads done
  stage_rows<false>(qimg, a.k + b * a.sq_b + h * DH, a.sq_t, TV, a.T);  // the K image
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  // ---- phase 2: dQ^T[d][q] = sum over keys of K^T[d][key] dS^T[key][q], this wave's 16 queries
  f32x4 acc[4] = {};
  const char* drow = dsimg + qi * kDsRow;  // qi < NQ always (16 NT rows)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const bf16x4 lo = *reinterpret_cast<const bf16x4*>(drow + (32 * ks + 4 * g) * 2);
    const bf16x4 hi = *reinterpret_cast<const bf16x4*>(drow + (32 * ks + 16 + 4 * g) * 2);
    const bf16x8 bop = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(img_tr(qimg, 32 * ks, 16 * dt), bop, acc[dt]);
  }
  if (qok) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 o = {(bf16)(acc[dt][0] * a.scale), (bf16)(acc[dt][1] * a.scale), (bf16)(acc[dt][2] * a.scale),
                        (bf16)(acc[dt][3] * a.scale)};
      *reinterpret_cast<bf16x4*>(a.dq + qoff + dt * 16 + 4 * g) = o;
    }
  }
  if (a.colpart != nullptr) colpart_store(colpart_row(a, b, h, 0, w, 0), acc, a.scale, qok);
}

constexpr size_t fused_lds(int nt) {
  return static_cast<size_t>(2 * (((16 * nt + 31) / 32) * 32) * 128 + 16 * nt * kDsRow +
                             2 * (((16 * nt + 31) / 32) * 32) * 4);
}

// the one-kernel backward for 13 key / query tiles (T 193..208: ViT's 197), default; measured 286-289
// vs 340-343 us per call for the dq / dkv pair, ViT-B/16 7698 / 7694 vs 7549 / 7588 img/s on one box
// (profiles/rd6o_attn_fused_ab.jsonl). FLUXMPI_ATTN_BWD=pair keeps the pair (A/B), =blocked the
// non-resident kernels.
bool attn_fused_env() {
  static const bool on = [] {
    const char* e = std::getenv("FLUXMPI_ATTN_BWD");
    return e == nullptr || (std::string(e) != "pair" && std::string(e) != "blocked");
  }();
  return on;
}

// FLUXMPI_ATTN_GENERIC=1: the runtime-tile-count kernels for every T (A/B of the NT = 13 instances)
// explicitly pipelined dkv k-steps for the compile-time-tile-count kernel (FLUXMPI_ATTN_DKV_PIPE=0: off)
bool dkv_pipe() {
  static const bool on = [] {
    const char* e = std::getenv("FLUXMPI_ATTN_DKV_PIPE");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

bool attn_generic() {
  static const bool on = [] {
    const char* e = std::getenv("FLUXMPI_ATTN_GENERIC");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// workgroups per (b, h) of the resident kernels (FLUXMPI_ATTN_PARTS, default 2): with the head's
// ~55 KB of LDS and <= 8 waves each, two workgroups share a CU, so one stages its head while
// the other computes (one workgroup of 13 waves per CU left every staging exposed)
int res_parts(int tiles) {
  static const int parts = [] {
    const char* e = std::getenv("FLUXMPI_ATTN_PARTS");
    const int v = e != nullptr ? std::atoi(e) : 2;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  return parts < tiles ? parts : tiles;
}

// workgroups per (b, h) of the resident forward (FLUXMPI_ATTN_FWD_PARTS, default 2). At 53 KB of
// LDS three fit a CU, but three parts measured slower than two (101-102 vs 94-95 us per call at
// the ViT-B/16 shape, one part 103, four 110-111; ViT-B/16 equal: profiles/rd6w_attn_fwd_parts.jsonl)
int fwd_parts(int tiles) {
  static const int parts = [] {
    const char* e = std::getenv("FLUXMPI_ATTN_FWD_PARTS");
    const int v = e != nullptr ? std::atoi(e) : 2;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  return parts < tiles ? parts : tiles;
}

}  // namespace

namespace {
// FLUXMPI_ATTN_BWD=blocked / FLUXMPI_ATTN_FWD=blocked: the non-resident kernels for every T (A/B)
bool blocked_env(const char* name) {
  const char* e = std::getenv(name);
  return e != nullptr && std::string(e) == "blocked";
}
}  // namespace

int attn_bwd_colpart_rows(int B, int T, int H, int64_t sq_t, int64_t sg_t) {
  // the resident dq / dkv pair writes the column-sum partials; every other variant does not
  if (blocked_env("FLUXMPI_ATTN_BWD") || T > kResMaxT || T <= 0 || (sq_t % 8) != 0 || (sg_t % 8) != 0) return 0;
  const int tiles = (T + 15) / 16;
  if (attn_fused_env() && tiles == 13 && !attn_generic()) return B * tiles;  // the fused kernel: one part of 13 waves
  const int nblk = res_parts(tiles);
  const int waves = (tiles + nblk - 1) / nblk;
  (void)H;
  return B * nblk * waves;
}

void attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, void* dq, void* dk,
              void* dv, float* stats, int64_t sq_b, int64_t sq_t, int64_t so_b, int64_t so_t, int64_t so_h,
              int64_t sg_b, int64_t sg_t, int B, int T, int H, int Dh, float scale, hipStream_t s, float* colpart) {
  if (Dh != DH) throw std::runtime_error("attn_bwd: head dim must be 64");
  if (B <= 0 || T <= 0 || H <= 0) throw std::runtime_error("attn_bwd: empty problem");
  for (const void* p : {q, k, v, o, dout, static_cast<const void*>(dq), static_cast<const void*>(dk),
                        static_cast<const void*>(dv)})
    if (!al16(p)) throw std::runtime_error("attn_bwd: operands must be 16-byte aligned");
  for (int64_t st : {sq_b, sq_t, so_b, so_t, so_h, sg_b, sg_t})
    if (st % 8 != 0) throw std::runtime_error("attn_bwd: strides must be multiples of 8 elements");
  AttnBwdArgs a{static_cast<const bf16*>(q), static_cast<const bf16*>(k), static_cast<const bf16*>(v),
                static_cast<const bf16*>(o), static_cast<const bf16*>(dout), nullptr, static_cast<bf16*>(dq),
                static_cast<bf16*>(dk), static_cast<bf16*>(dv), stats, sq_b, sq_t, so_b, so_t, so_h, sg_b, sg_t,
                B, T, H, (T + 63) / 64, scale};
  static const bool resident = !blocked_env("FLUXMPI_ATTN_BWD");
  if (resident && T <= kResMaxT && (sq_t % 8) == 0 && (sg_t % 8) == 0) {
    const int tiles = (T + 15) / 16;
    if (attn_fused_env() && tiles == 13 && !attn_generic()) {
      a.nblk = 1;
      const int64_t bh = static_cast<int64_t>(B) * H;
      if (bh > 0x7fffffff) throw std::runtime_error("attn_bwd: grid too large");
      a.colpart = colpart;  // [B * 13][3 * H * 64] (attn_bwd_colpart_rows), or nullptr
      static const bool attr = [] {
        FLUXMPI_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_fused_kernel<13>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              static_cast<int>(fused_lds(13))));
        return true;
      }();
      (void)attr;
      attn_bwd_fused_kernel<13><<<static_cast<unsigned>(bh), 13 * 64, fused_lds(13), s>>>(a);
      FLUXMPI_HIP_CHECK(hipGetLastError());
      return;
    }
    a.nblk = res_parts(tiles);
    const int64_t bh = static_cast<int64_t>(B) * H * a.nblk;
    if (bh > 0x7fffffff) throw std::runtime_error("attn_bwd: grid too large");
    const int waves = (tiles + a.nblk - 1) / a.nblk;
    const int TP = (T + 15) & ~15, TV = (T + 31) & ~31;
    a.colpart = colpart;  // [B * nblk * waves][3 * H * 64] (attn_bwd_colpart_rows), or nullptr
    const bool vit = tiles == 13 && !attn_generic();  // T 193..208 (ViT: 197): compile-time tile count
    auto kdq = vit ? attn_bwd_dq_res_kernel<13> : attn_bwd_dq_res_kernel<0>;
    auto kdkv = !vit ? attn_bwd_dkv_res_kernel<0> : (dkv_pipe() ? attn_bwd_dkv_res_kernel<13, 1> : attn_bwd_dkv_res_kernel<13, 0>);
    kdq<<<static_cast<unsigned>(bh), waves * 64, static_cast<size_t>(TV + TP) * 128, s>>>(a);
    FLUXMPI_HIP_CHECK(hipGetLastError());
    kdkv<<<static_cast<unsigned>(bh), waves * 64, static_cast<size_t>(2 * TV) * 128 + 2 * TV * 4,
                              s>>>(a);
    FLUXMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  const int64_t total = static_cast<int64_t>(B) * H * a.nblk;
  if (total > 0x7fffffff) throw std::runtime_error("attn_bwd: grid too large");
  attn_bwd_dq_kernel<<<static_cast<unsigned>(total), 256, 0, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
  attn_bwd_dkv_kernel<<<static_cast<unsigned>(total), 256, 0, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void attn_fwd(const void* q, const void* k, const void* v, void* o, float* stats, int64_t sq_b, int64_t sq_t,
              int64_t so_b, int64_t so_t, int64_t so_h, int B, int T, int H, int Dh, float scale, hipStream_t s) {
  if (Dh != DH) throw std::runtime_error("attn_fwd: head dim must be 64");
  if (B <= 0 || T <= 0 || H <= 0) throw std::runtime_error("attn_fwd: empty problem");
  for (const void* p : {q, k, v, static_cast<const void*>(o)})
    if (!al16(p)) throw std::runtime_error("attn_fwd: operands must be 16-byte aligned");
  for (int64_t st : {sq_b, sq_t, so_b, so_t, so_h})
    if (st % 8 != 0) throw std::runtime_error("attn_fwd: strides must be multiples of 8 elements");
  AttnBwdArgs a{};
  a.q = static_cast<const bf16*>(q);
  a.k = static_cast<const bf16*>(k);
  a.v = static_cast<const bf16*>(v);
  a.o_out = static_cast<bf16*>(o);
  a.stats = stats;
  a.sq_b = sq_b;
  a.sq_t = sq_t;
  a.so_b = so_b;
  a.so_t = so_t;
  a.so_h = so_h;
  a.B = B;
  a.T = T;
  a.H = H;
  a.nblk = (T + 63) / 64;
  a.scale = scale;
  static const bool resident = !blocked_env("FLUXMPI_ATTN_FWD");
  if (resident && T <= kResMaxT && (sq_t % 8) == 0) {
    // whole head resident in LDS: fwd_parts() workgroups per (b, h), one wave per 16 queries
    const int tiles = (T + 15) / 16;
    a.nblk = fwd_parts(tiles);
    const int64_t total = static_cast<int64_t>(B) * H * a.nblk;
    if (total > 0x7fffffff) throw std::runtime_error("attn_fwd: grid too large");
    const int waves = (tiles + a.nblk - 1) / a.nblk;
    const size_t lds = static_cast<size_t>(2 * ((T + 15) & ~15)) * 128;
    auto kf = (tiles == 13 && !attn_generic()) ? attn_fwd_res_kernel<13> : attn_fwd_res_kernel<0>;
    kf<<<static_cast<unsigned>(total), waves * 64, lds, s>>>(a);
    FLUXMPI_HIP_CHECK(hipGetLastError());
    return;
  }
  const int64_t total = static_cast<int64_t>(B) * H * a.nblk;
  if (total > 0x7fffffff) throw std::runtime_error("attn_fwd: grid too large");
  attn_fwd_kernel<<<static_cast<unsigned>(total), 256, 0, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
