// The DEQ cell as ONE kernel per evaluation — gfx950.
//
//   f(z, x) = GN3(relu(z + GN2(x + conv2(GN1(relu(conv1 z))))))      (models/deq.py ResidualCell)
//
// The unfused evaluation is 2 implicit-GEMM convolutions + 3 GroupNorm passes (~115 us at the
// MNIST DEQ's 256 x 28 x 28 x 48, every intermediate a 19 MB round trip through HBM), and the
// adjoint VJP 2 input-gradient convolutions + 3 GroupNorm backwards (~100 us). Both are
// per-sample computations whose working set fits one CU: a 28 x 28 x 48 bf16 image is 75 KB,
// a 3x3 48 -> 48 filter 41 KB, and every GroupNorm statistic is a reduction over ONE sample.
// So one workgroup owns one sample (a batch of 256 fills the 256 CUs once) and keeps it in LDS:
//
//   LDS  image  (H+2) x (W+2) x C bf16 with a zero halo (the convolution input: z, then
//               GN1's output; in the VJP d2, then d1), rows padded by 32 elements so that the
//               B-fragment reads are bank-conflict free (scripts/lds_banks.py model),
//        filter [C][9C] bf16, K-major (k = tap * C + ci), rows padded to 14*32 + 16 elements
//               (conflict-free A fragments), zero-filled K tail,
//        per-wave channel partial sums for the GroupNorm reductions.
//   conv  implicit GEMM C^T[co][px] = W[co][k] . X^T[k][px] on v_mfma_f32_16x16x32_bf16: the
//         A fragment (16 co x 32 k) is one ds_read_b128 per lane from the filter, the B
//         fragment (32 k x 16 px) one ds_read_b128 per lane from the halo image at
//         (pixel + tap offset, 8 channels) — no im2col anywhere. 8 waves x 7 pixel blocks of 16
//         (784 = 49 blocks) x 3 co blocks; per K chunk a wave reads 3 A + 7 B fragments for 21
//         MFMAs. The accumulator layout (lane: 4 consecutive channels of one pixel) is then the
//         layout of every elementwise GroupNorm step, so nothing is transposed.
//   GN    each lane sums its 12 channels over its 7 pixels, a 16-lane DPP row sum and an LDS
//         pass over the 8 waves give the per-group statistics; normalisation is applied in
//         registers and written straight into the next convolution's LDS image.
//
// Numerics mirror the unfused kernels (ops/fused_block.py conv3x3_*_raw + ops/groupnorm.py
// gn_*_raw): the convolution outputs are rounded to bf16, GroupNorm statistics are taken over the
// bf16-rounded inputs (var = E[h^2] - mean^2), every stored activation is bf16; the VJP's final
// convolution adds the d3 residual before its one rounding (the dgrad residual epilogue).
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 dc_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 dc_bf16x4 __attribute__((ext_vector_type(4)));
typedef float dc_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kC = 48;                 // channels (in = out)
constexpr int kK = 9 * kC;             // 432: GEMM K = taps x channels
constexpr int kKC = (kK + 31) / 32;    // 14 K chunks of 32 (the last half zero-filled)
constexpr int kWS = kKC * 32 + 16;     // 464: filter row stride in LDS (elements)
constexpr int kMB = kC / 16;           // 3 output-channel blocks of 16
constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kNBW = 7;                // pixel blocks (of 16) per wave: 8 x 7 = 56 >= 49
constexpr int kMaxG = 16;
constexpr int kRowPad = 32;            // image row padding (elements): conflict-free B fragments

struct CellGN {
  const float* w[3];  // fp32 affine per GroupNorm (nullable: identity)
  const float* b[3];
};

struct CellStats {    // per-sample group statistics, [N][G] fp32 each
  float* mean[3];
  float* rstd[3];
};

struct CellShape {
  int N, H, W, HW, G, RP;  // RP: image row stride (elements)
  float eps;
};

__device__ __forceinline__ int img_bytes(const CellShape& s) { return (s.H + 2) * s.RP * 2; }

__device__ __forceinline__ dc_f32x4 mfma32(dc_bf16x8 a, dc_bf16x8 b, dc_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float rbf(float v) { return static_cast<float>(static_cast<bf16>(v)); }

// ---- staging -------------------------------------------------------------------------------------

// zero the halo ring of the image (rows 0 and H+1, columns 0 and W+1)
__device__ void zero_halo(char* img, const CellShape& s) {
  const int rowc = (s.W + 2) * kC / 8;  // 16-B chunks per image row
  const uint4 z = {0u, 0u, 0u, 0u};
  for (int i = threadIdx.x; i < 2 * rowc; i += kThreads) {
    const int r = i < rowc ? 0 : s.H + 1, c = i < rowc ? i : i - rowc;
    *reinterpret_cast<uint4*>(img + (r * s.RP + c * 8) * 2) = z;
  }
  constexpr int pc = kC / 8;
  for (int i = threadIdx.x; i < 2 * s.H * pc; i += kThreads) {
    const int side = i / (s.H * pc), rem = i % (s.H * pc), r = 1 + rem / pc, c = rem % pc;
    const int x = side ? s.W + 1 : 0;
    *reinterpret_cast<uint4*>(img + (r * s.RP + x * kC + c * 8) * 2) = z;
  }
}

// one NHWC sample [HW][C] bf16 from global memory into the image interior (16-B chunks, 4 in flight)
__device__ void load_image(char* img, const bf16* __restrict__ src, const CellShape& s) {
  constexpr int pc = kC / 8;
  const int n = s.HW * pc;
  int i = threadIdx.x;
  for (; i + 3 * kThreads < n; i += 4 * kThreads) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = reinterpret_cast<const uint4*>(src)[i + u * kThreads];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = i + u * kThreads, px = j / pc, c = j % pc, y = px / s.W, x = px % s.W;
      *reinterpret_cast<uint4*>(img + ((y + 1) * s.RP + (x + 1) * kC + c * 8) * 2) = v[u];
    }
  }
  for (; i < n; i += kThreads) {
    const uint4 v = reinterpret_cast<const uint4*>(src)[i];
    const int px = i / pc, c = i % pc, y = px / s.W, x = px % s.W;
    *reinterpret_cast<uint4*>(img + ((y + 1) * s.RP + (x + 1) * kC + c * 8) * 2) = v;
  }
}

// a [C][9C] bf16 filter into the LDS rows of stride kWS, zero-filling the K tail
__device__ void load_filter(char* wl, const bf16* __restrict__ w) {
  constexpr int rc = kWS / 8;  // 16-B chunks per LDS row
  constexpr int src_rc = kK / 8;
  for (int i = threadIdx.x; i < kC * rc; i += kThreads) {
    const int r = i / rc, c = i % rc;
    uint4 v = {0u, 0u, 0u, 0u};
    if (c < src_rc) v = reinterpret_cast<const uint4*>(w)[r * src_rc + c];
    *reinterpret_cast<uint4*>(wl + (r * kWS + c * 8) * 2) = v;
  }
}

// ---- the convolution -----------------------------------------------------------------------------

struct Lane {
  int l, w, g, col;
  int pb[kNBW];     // image offset (elements) of each owned pixel's top-left tap
  bool ok[kNBW];    // wave-uniform: pixel block exists
  int px[kNBW];     // owned pixel per block
};

__device__ __forceinline__ Lane make_lane(const CellShape& s) {
  Lane L;
  L.l = threadIdx.x & 63;
  L.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: ok[] branches are scalar
  L.g = L.l >> 4;
  L.col = L.l & 15;
  const int nblk = s.HW / 16;
#pragma unroll
  for (int i = 0; i < kNBW; ++i) {
    const int nb = L.w + kWaves * i;
    L.ok[i] = nb < nblk;
    const int p = L.ok[i] ? 16 * nb + L.col : 0;
    L.px[i] = p;
    L.pb[i] = (p / s.W) * s.RP + (p % s.W) * kC;
  }
  return L;
}

// acc[mb][i] = sum_k W[16 mb + row][k] X[k][pixel block i]
__device__ __forceinline__ void conv(dc_f32x4 (&acc)[kMB][kNBW], const char* img, const char* wl, const Lane& L,
                                     const CellShape& s) {
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int i = 0; i < kNBW; ++i) acc[mb][i] = dc_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int kc = 0; kc < kKC; ++kc) {
    const int k = 32 * kc + 8 * L.g;
    dc_bf16x8 a[kMB];
#pragma unroll
    for (int mb = 0; mb < kMB; ++mb)
      a[mb] = *reinterpret_cast<const dc_bf16x8*>(wl + ((16 * mb + L.col) * kWS + k) * 2);
    // tap of this lane's 8 K values (the zero-filled tail reuses tap 8: finite data x 0 weights)
    const int t = k < kK ? k / kC : 8, ci = k < kK ? k % kC : 0;
    const int toff = (t / 3) * s.RP + (t % 3) * kC + ci;
#pragma unroll
    for (int i = 0; i < kNBW; ++i) {
      if (!L.ok[i]) continue;
      const dc_bf16x8 b = *reinterpret_cast<const dc_bf16x8*>(img + (L.pb[i] + toff) * 2);
#pragma unroll
      for (int mb = 0; mb < kMB; ++mb) acc[mb][i] = mfma32(a[mb], b, acc[mb][i]);
    }
  }
  // no global load of the next phase is hoisted into the MFMA loop (its registers would sit
  // beside the 84 accumulators and spill)
  asm volatile("" ::: "memory");
}

// ---- GroupNorm reductions ------------------------------------------------------------------------

// Per-channel sums of two lane-partial arrays over the sample: 16-lane DPP row sums, then the
// waves' partials through LDS. Returns nothing; red[2][C] holds the totals after the call.
__device__ __forceinline__ void channel_sums(float (&p)[kMB][4], float (&q)[kMB][4], float* part, float* red,
                                             const Lane& L) {
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = row_sum16(p[mb][j]), b = row_sum16(q[mb][j]);
      if (L.col == 0) {
        const int c = 16 * mb + 4 * L.g + j;
        part[(L.w * 2) * kC + c] = a;
        part[(L.w * 2 + 1) * kC + c] = b;
      }
    }
  __syncthreads();
  if (threadIdx.x < 2 * kC) {
    const int which = threadIdx.x / kC, c = threadIdx.x % kC;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += part[(w * 2 + which) * kC + c];
    red[threadIdx.x] = t;
  }
  __syncthreads();
}

// The lane's values are kept as packed bf16 (every stored activation is bf16-rounded anyway):
// half the registers of fp32, so a VJP phase holds its operand, a saved input and d3 at once.
typedef dc_bf16x4 Pk[kMB][kNBW];

__device__ __forceinline__ float fv(const Pk& v, int mb, int i, int j) { return static_cast<float>(v[mb][i][j]); }

// An empty asm that "modifies" the packed registers: the apply pass after a reduction re-unpacks
// them instead of keeping the statistics pass's 84 unpacked fp32 copies alive across the barrier
// (which doubled the VJP's register demand and spilled).
__device__ __forceinline__ void opaque(Pk& v) {
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int i = 0; i < kNBW; ++i) asm volatile("" : "+v"(*reinterpret_cast<uint2*>(&v[mb][i])));
}

// GroupNorm forward on the lane's values (the bf16 GN inputs, in place -> the bf16 outputs).
// Statistics over the sample (gn_fwd_kernel's arithmetic); the 48 channel threads turn them into
// per-channel scale / shift in LDS (coef[2][C]) and write mean / rstd of sample n when asked.
__device__ __forceinline__ void gn_forward(Pk& v, const float* __restrict__ w, const float* __restrict__ b,
                                           float* part, float* red, float* coef, const Lane& L,
                                           const CellShape& s, float* mean_out, float* rstd_out, int n) {
  float ps[kMB][4], pq[kMB][4];
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < kNBW; ++i)
        if (L.ok[i]) {
          const float t = fv(v, mb, i, j);
          a += t;
          q += t * t;
        }
      ps[mb][j] = a;
      pq[mb][j] = q;
    }
  channel_sums(ps, pq, part, red, L);
  if (threadIdx.x < kC) {
    const int c = threadIdx.x, cpg = kC / s.G, gi = c / cpg;
    float gs = 0.f, gq = 0.f;
    for (int k = gi * cpg; k < (gi + 1) * cpg; ++k) {
      gs += red[k];
      gq += red[kC + k];
    }
    const float inv_m = 1.f / (static_cast<float>(s.HW) * cpg);
    const float mu = gs * inv_m;
    const float var = fmaxf(gq * inv_m - mu * mu, 0.f);
    const float r = rsqrtf(var + s.eps);
    const float sc = r * (w ? w[c] : 1.f);
    coef[c] = sc;
    coef[kC + c] = (b ? b[c] : 0.f) - mu * sc;
    if (mean_out != nullptr && c % cpg == 0) {
      mean_out[static_cast<int64_t>(n) * s.G + gi] = mu;
      rstd_out[static_cast<int64_t>(n) * s.G + gi] = r;
    }
  }
  __syncthreads();
  opaque(v);
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb) {
    const int c0 = 16 * mb + 4 * L.g;
    const float4 sc = *reinterpret_cast<const float4*>(coef + c0);
    const float4 sh = *reinterpret_cast<const float4*>(coef + kC + c0);
    const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
    for (int i = 0; i < kNBW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[mb][i][j] = static_cast<bf16>(fv(v, mb, i, j) * scv[j] + shv[j]);
  }
  __syncthreads();  // part / red / coef are reused by the next reduction
}

// GroupNorm backward: dy (in place -> the bf16 input gradient) from the saved inputs h; ReLU
// mask on h > 0. gn_bwd_kernel's arithmetic, folded per channel into
// d = A_c dy + B_c + C_c h  with A = r w, C = -r^2 s2, B = -r s1 - C mu  (coef[3][C]).
template <bool RELU>
__device__ __forceinline__ void gn_backward(Pk& dy, Pk& h, const float* __restrict__ w,
                                            const float* __restrict__ mean, const float* __restrict__ rstd,
                                            float* part, float* red, float* coef, const Lane& L, const CellShape& s,
                                            int n) {
  float ps[kMB][4], pq[kMB][4];
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < kNBW; ++i)
        if (L.ok[i]) {
          const float d = fv(dy, mb, i, j);
          a += d;
          q += d * fv(h, mb, i, j);
        }
      ps[mb][j] = a;
      pq[mb][j] = q;
    }
  channel_sums(ps, pq, part, red, L);
  if (threadIdx.x < kC) {
    const int c = threadIdx.x, cpg = kC / s.G, gi = c / cpg;
    const float inv_m = 1.f / (static_cast<float>(s.HW) * cpg);
    const float mu = mean[static_cast<int64_t>(n) * s.G + gi], r = rstd[static_cast<int64_t>(n) * s.G + gi];
    float s1 = 0.f, s2 = 0.f;  // sum dy w, sum dy w xhat over the group
    for (int k = gi * cpg; k < (gi + 1) * cpg; ++k) {
      const float wk = w ? w[k] : 1.f;
      s1 += wk * red[k];
      s2 += wk * r * (red[kC + k] - mu * red[k]);
    }
    s1 *= inv_m;
    s2 *= inv_m;
    const float A = r * (w ? w[c] : 1.f), Cc = -r * r * s2;
    coef[c] = A;
    coef[kC + c] = -r * s1 - Cc * mu;
    coef[2 * kC + c] = Cc;
  }
  __syncthreads();
  opaque(dy);
  opaque(h);
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb) {
    const int c0 = 16 * mb + 4 * L.g;
    const float4 A4 = *reinterpret_cast<const float4*>(coef + c0);
    const float4 B4 = *reinterpret_cast<const float4*>(coef + kC + c0);
    const float4 C4 = *reinterpret_cast<const float4*>(coef + 2 * kC + c0);
    const float Av[4] = {A4.x, A4.y, A4.z, A4.w}, Bv[4] = {B4.x, B4.y, B4.z, B4.w};
    const float Cv[4] = {C4.x, C4.y, C4.z, C4.w};
#pragma unroll
    for (int i = 0; i < kNBW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float hf = fv(h, mb, i, j);
        float d = fmaf(Av[j], fv(dy, mb, i, j), fmaf(Cv[j], hf, Bv[j]));
        if (RELU && !(hf > 0.f)) d = 0.f;
        dy[mb][i][j] = static_cast<bf16>(d);
      }
  }
  __syncthreads();  // part / red / coef are reused by the next reduction
}

// ---- lane-layout global / LDS access (4 consecutive channels of one pixel) -----------------------

__device__ __forceinline__ void load_lane(Pk& v, const bf16* __restrict__ src, const Lane& L) {
#pragma unroll
  for (int i = 0; i < kNBW; ++i)
#pragma unroll
    for (int mb = 0; mb < kMB; ++mb)
      v[mb][i] = L.ok[i] ? *reinterpret_cast<const dc_bf16x4*>(src + L.px[i] * kC + 16 * mb + 4 * L.g)
                         : dc_bf16x4{};
}

__device__ __forceinline__ void store_lane(bf16* __restrict__ dst, const Pk& v, const Lane& L) {
#pragma unroll
  for (int i = 0; i < kNBW; ++i)
    if (L.ok[i])
#pragma unroll
      for (int mb = 0; mb < kMB; ++mb)
        *reinterpret_cast<dc_bf16x4*>(dst + L.px[i] * kC + 16 * mb + 4 * L.g) = v[mb][i];
}

// the lane's values into the LDS image interior (the next convolution's input)
__device__ __forceinline__ void store_image(char* img, const Pk& v, const Lane& L, const CellShape& s) {
#pragma unroll
  for (int i = 0; i < kNBW; ++i)
    if (L.ok[i])
#pragma unroll
      for (int mb = 0; mb < kMB; ++mb)
        *reinterpret_cast<dc_bf16x4*>(img + (L.pb[i] + s.RP + kC + 16 * mb + 4 * L.g) * 2) = v[mb][i];
}

// the convolution output rounded to bf16 (what the unfused conv kernels store)
__device__ __forceinline__ void round_acc(Pk& v, const dc_f32x4 (&acc)[kMB][kNBW]) {
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int i = 0; i < kNBW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[mb][i][j] = static_cast<bf16>(acc[mb][i][j]);
}

struct FwdArgs {
  const bf16* z;
  const bf16* x;
  const bf16* w1;  // [C][9C], k = tap * C + ci
  const bf16* w2;
  CellGN gn;
  bf16* out;            // nullable, sample stride out_stride (an Anderson bf16 history slot, or dense)
  float* out32;         // nullable: fp32 copy of the output, sample stride out32_stride
  int64_t out32_stride;
  int64_t out_stride;
  bf16* h[3];           // nullable: the GroupNorm inputs (the VJP's state)
  CellStats st;         // mean / rstd pointers nullable
};

__global__ __launch_bounds__(kThreads) void deq_cell_fwd_kernel(FwdArgs a, CellShape s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* img = smem;
  char* wl = img + img_bytes(s);
  float* part = reinterpret_cast<float*>(wl + kC * kWS * 2);  // [waves][2][C]
  float* red = part + kWaves * 2 * kC;                        // [2][C]
  float* coef = red + 2 * kC;                                 // [3][C] per-channel GN coefficients
  const int n = blockIdx.x;
  const int64_t so = static_cast<int64_t>(n) * s.HW * kC;
  const Lane L = make_lane(s);
  zero_halo(img, s);
  load_image(img, a.z + so, s);
  load_filter(wl, a.w1);
  __syncthreads();

  dc_f32x4 acc[kMB][kNBW];
  Pk v;
  conv(acc, img, wl, L, s);
  __syncthreads();  // every wave is done reading z and W1
  load_filter(wl, a.w2);
  // GN1(relu(c1))
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int i = 0; i < kNBW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[mb][i][j] = static_cast<bf16>(fmaxf(rbf(acc[mb][i][j]), 0.f));
  if (a.h[0] != nullptr) store_lane(a.h[0] + so, v, L);
  gn_forward(v, a.gn.w[0], a.gn.b[0], part, red, coef, L, s, a.st.mean[0], a.st.rstd[0], n);
  store_image(img, v, L, s);
  __syncthreads();

  conv(acc, img, wl, L, s);
  // GN2(c2 + x)
  load_lane(v, a.x + so, L);
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int i = 0; i < kNBW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[mb][i][j] = static_cast<bf16>(rbf(acc[mb][i][j]) + fv(v, mb, i, j));
  if (a.h[1] != nullptr) store_lane(a.h[1] + so, v, L);
  gn_forward(v, a.gn.w[1], a.gn.b[1], part, red, coef, L, s, a.st.mean[1], a.st.rstd[1], n);
  // GN3(relu(z + a2))
  {
    Pk zv;
    load_lane(zv, a.z + so, L);
#pragma unroll
    for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
      for (int i = 0; i < kNBW; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[mb][i][j] = static_cast<bf16>(fmaxf(fv(zv, mb, i, j) + fv(v, mb, i, j), 0.f));
  }
  if (a.h[2] != nullptr) store_lane(a.h[2] + so, v, L);
  gn_forward(v, a.gn.w[2], a.gn.b[2], part, red, coef, L, s, a.st.mean[2], a.st.rstd[2], n);
  if (a.out != nullptr) store_lane(a.out + static_cast<int64_t>(n) * a.out_stride, v, L);
  if (a.out32 != nullptr) {
    float* o = a.out32 + static_cast<int64_t>(n) * a.out32_stride;
#pragma unroll
    for (int i = 0; i < kNBW; ++i)
      if (L.ok[i])
#pragma unroll
        for (int mb = 0; mb < kMB; ++mb)
          *reinterpret_cast<float4*>(o + L.px[i] * kC + 16 * mb + 4 * L.g) =
              float4{fv(v, mb, i, 0), fv(v, mb, i, 1), fv(v, mb, i, 2), fv(v, mb, i, 3)};
  }
}

struct VjpArgs {
  const bf16* u;
  const bf16* h[3];
  const bf16* w2t;  // transposed, tap-flipped filters [C][9C] (k = tap * C + co)
  const bf16* w1t;
  const float* gw[3];
  const float* mean[3];
  const float* rstd[3];
  bf16* out;
  const bf16* grad;  // nullable: fuse the adjoint update, out = bf16(J^T u + grad), and
  float* ss_part;    //   ss_part[n] = sum over the sample of (out - u)^2 (adjoint_step_kernel's numerics)
};

__global__ __launch_bounds__(kThreads) void deq_cell_vjp_kernel(VjpArgs a, CellShape s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* img = smem;
  char* wl = img + img_bytes(s);
  float* part = reinterpret_cast<float*>(wl + kC * kWS * 2);
  float* red = part + kWaves * 2 * kC;
  float* coef = red + 2 * kC;
  const int n = blockIdx.x;
  const int64_t so = static_cast<int64_t>(n) * s.HW * kC;
  const Lane L = make_lane(s);
  zero_halo(img, s);
  load_filter(wl, a.w2t);

  Pk v, hv;
  load_lane(v, a.u + so, L);
  load_lane(hv, a.h[2] + so, L);
  gn_backward<true>(v, hv, a.gw[2], a.mean[2], a.rstd[2], part, red, coef, L, s, n);  // d3 = d(z + a2)
  // d3 is parked in the output (the same lanes read it back for the final residual): holding it
  // in registers across both convolutions spilled
  store_lane(a.out + so, v, L);
  load_lane(hv, a.h[1] + so, L);
  gn_backward<false>(v, hv, a.gw[1], a.mean[1], a.rstd[1], part, red, coef, L, s, n);  // d conv2 output
  store_image(img, v, L, s);
  __syncthreads();

  dc_f32x4 acc[kMB][kNBW];
  conv(acc, img, wl, L, s);  // d a1 = conv2^T(d2)
  round_acc(v, acc);
  load_lane(hv, a.h[0] + so, L);
  gn_backward<true>(v, hv, a.gw[0], a.mean[0], a.rstd[0], part, red, coef, L, s, n);  // d conv1 output
  // gn_backward's barriers follow this wave's conv: every wave is done reading d2 / W2^T
  load_filter(wl, a.w1t);
  store_image(img, v, L, s);
  __syncthreads();

  conv(acc, img, wl, L, s);  // conv1^T(d1) + d3 (n3's direct path to z), one rounding
  load_lane(hv, a.out + so, L);
#pragma unroll
  for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
    for (int i = 0; i < kNBW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[mb][i][j] = static_cast<bf16>(acc[mb][i][j] + fv(hv, mb, i, j));
  if (a.grad != nullptr) {  // the adjoint iteration's update u <- J^T u + grad and its step size
    load_lane(hv, a.grad + so, L);
    Pk uv;
    load_lane(uv, a.u + so, L);
    float ss = 0.f;
#pragma unroll
    for (int mb = 0; mb < kMB; ++mb)
#pragma unroll
      for (int i = 0; i < kNBW; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16 r = static_cast<bf16>(fv(v, mb, i, j) + fv(hv, mb, i, j));
          const float dlt = static_cast<float>(r) - fv(uv, mb, i, j);  // zero on absent blocks
          ss = fmaf(dlt, dlt, ss);
          v[mb][i][j] = r;
        }
    ss = wave_sum_dpp(ss);
    if (L.l == 0) part[L.w] = ss;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) t += part[w];
      a.ss_part[n] = t;
    }
  }
  store_lane(a.out + so, v, L);
}

// sum of the per-sample step sizes; flag = (sum <= *thresh2) — the adjoint's convergence test
__global__ __launch_bounds__(256) void deq_adjoint_check_kernel(const float* __restrict__ part, int n,
                                                                const float* __restrict__ thresh2,
                                                                float* __restrict__ ss_out, float* __restrict__ flag) {
  __shared__ float red[4];
  float t = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) t += part[i];
  t = wave_sum_dpp(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    if (ss_out != nullptr) ss_out[0] = tot;
    if (flag != nullptr) flag[0] = tot <= thresh2[0] ? 1.f : 0.f;
  }
}

CellShape cell_shape(int64_t N, int64_t H, int64_t W, int64_t C, int64_t G, float eps) {
  if (C != kC) throw std::runtime_error("deq_cell: channels must be " + std::to_string(kC));
  if (G < 1 || G > kMaxG || C % G != 0) throw std::runtime_error("deq_cell: bad group count");
  if (N < 1 || N > 2147483647LL || H < 1 || W < 1 || (H * W) % 16 != 0 || H * W / 16 > kWaves * kNBW)
    throw std::runtime_error("deq_cell: need H*W a multiple of 16 and <= " + std::to_string(16 * kWaves * kNBW));
  CellShape s;
  s.N = static_cast<int>(N);
  s.H = static_cast<int>(H);
  s.W = static_cast<int>(W);
  s.HW = s.H * s.W;
  s.G = static_cast<int>(G);
  s.RP = (s.W + 2) * kC + kRowPad;
  s.eps = eps;
  return s;
}

size_t cell_lds(const CellShape& s) {
  return static_cast<size_t>(s.H + 2) * s.RP * 2 + kC * kWS * 2 + sizeof(float) * (kWaves * 2 * kC + 2 * kC + 3 * kC);
}

void check16(std::initializer_list<const void*> ps) {
  for (const void* p : ps)
    if (p != nullptr && (reinterpret_cast<uintptr_t>(p) & 15u) != 0)
      throw std::runtime_error("deq_cell: tensors must be 16-byte aligned");
}

template <typename K>
void set_lds(K kernel, size_t lds) {
  if (lds > 160 * 1024) throw std::runtime_error("deq_cell: sample does not fit in LDS");
  FLUXMPI_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
}

}  // namespace

bool deq_cell_supported(int64_t H, int64_t W, int64_t C, int64_t G) {
  if (C != kC || G < 1 || G > kMaxG || C % G != 0 || (H * W) % 16 != 0 || H * W / 16 > kWaves * kNBW) return false;
  const CellShape s = cell_shape(1, H, W, C, G, 0.f);
  return cell_lds(s) <= 160 * 1024;
}

void deq_cell_fwd(const void* z, const void* x, const void* w1, const void* w2, const float* const* gn_w,
                  const float* const* gn_b, void* out, float* out32, int64_t out32_stride, void* const* h,
                  float* const* mean, float* const* rstd, int64_t N, int64_t H, int64_t W, int64_t C, int64_t G,
                  float eps, hipStream_t stream, int64_t out_stride) {
  const CellShape s = cell_shape(N, H, W, C, G, eps);
  check16({z, x, w1, w2, out, out32, h[0], h[1], h[2]});
  if (out == nullptr && out32 == nullptr) throw std::runtime_error("deq_cell_fwd: no output");
  if (out32 != nullptr && out32_stride % 4 != 0) throw std::runtime_error("deq_cell_fwd: out32 stride % 4");
  if (out_stride == 0) out_stride = H * W * C;
  if (out_stride % 8 != 0 || out_stride < H * W * C) throw std::runtime_error("deq_cell_fwd: out stride");
  FwdArgs a{static_cast<const bf16*>(z), static_cast<const bf16*>(x), static_cast<const bf16*>(w1),
            static_cast<const bf16*>(w2), {}, static_cast<bf16*>(out), out32, out32_stride, out_stride, {}, {}};
  for (int i = 0; i < 3; ++i) {
    a.gn.w[i] = gn_w[i];
    a.gn.b[i] = gn_b[i];
    a.h[i] = static_cast<bf16*>(h[i]);
    a.st.mean[i] = mean[i];
    a.st.rstd[i] = rstd[i];
  }
  const size_t lds = cell_lds(s);
  static bool attr = false;
  if (!attr) {
    set_lds(deq_cell_fwd_kernel, 160 * 1024);
    attr = true;
  }
  deq_cell_fwd_kernel<<<s.N, kThreads, lds, stream>>>(a, s);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void deq_cell_vjp(const void* u, const void* const* h, const void* w2t, const void* w1t, const float* const* gn_w,
                  const float* const* mean, const float* const* rstd, void* out, const void* grad, float* ss_part,
                  int64_t N, int64_t H, int64_t W, int64_t C, int64_t G, hipStream_t stream) {
  const CellShape s = cell_shape(N, H, W, C, G, 0.f);
  check16({u, h[0], h[1], h[2], w2t, w1t, out, grad});
  if ((grad == nullptr) != (ss_part == nullptr)) throw std::runtime_error("deq_cell_vjp: grad and ss_part go together");
  if (out == u) throw std::runtime_error("deq_cell_vjp: out must not alias u");
  for (int i = 0; i < 3; ++i)
    if (mean[i] == nullptr || rstd[i] == nullptr || h[i] == nullptr)
      throw std::runtime_error("deq_cell_vjp: missing state");
  VjpArgs a{static_cast<const bf16*>(u), {}, static_cast<const bf16*>(w2t), static_cast<const bf16*>(w1t), {}, {}, {},
            static_cast<bf16*>(out), static_cast<const bf16*>(grad), ss_part};
  for (int i = 0; i < 3; ++i) {
    a.h[i] = static_cast<const bf16*>(h[i]);
    a.gw[i] = gn_w[i];
    a.mean[i] = mean[i];
    a.rstd[i] = rstd[i];
  }
  const size_t lds = cell_lds(s);
  static bool attr = false;
  if (!attr) {
    set_lds(deq_cell_vjp_kernel, 160 * 1024);
    attr = true;
  }
  deq_cell_vjp_kernel<<<s.N, kThreads, lds, stream>>>(a, s);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

void deq_adjoint_check(const float* part, int64_t n, const float* thresh2, float* ss_out, float* flag,
                       hipStream_t stream) {
  if (n < 1 || n > 2147483647LL) throw std::runtime_error("deq_adjoint_check: bad n");
  if (flag != nullptr && thresh2 == nullptr) throw std::runtime_error("deq_adjoint_check: flag needs thresh2");
  deq_adjoint_check_kernel<<<1, 256, 0, stream>>>(part, static_cast<int>(n), thresh2, ss_out, flag);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
