// A token-major Linear's whole backward GEMM work in ONE launch — gfx950.
//
//   input gradient   dX[m][kk] = sum_n dY[m][n] W[n][kk]      (M tokens x K_in, reduction N_out)
//   weight gradient  dW[n][kk] = sum_m dY[m][n] X[m][kk]      (N_out x K_in, reduction M = tokens)
//
// The two are independent. Run as two launches (round 5: hipBLASLt stream-K for the input
// gradient, wgrad256.hip for the weight gradient) each one has its own partial last round — the
// ViT-B/16 input gradients with K_in = 768 are 591 tiles of 256 x 256 = 2.31 rounds of 256 CUs
// — and a drain / refill at the boundary. Here every job is ONE 512-thread workgroup on a
// 256 x 256 output tile (one workgroup per CU: 128 KiB of LDS), and the grid lists the weight-
// gradient split-K jobs and the input-gradient tiles in the order the host picks (the dispatcher
// hands CUs out in grid order as they free up; ops/linear.py simulates that greedy schedule per
// shape to choose the split count and which kind goes first). A weight-gradient job writes an fp32 partial [split][N_out][K_in] (summed
// by gemm_splitk_reduce, as wgrad256.hip's); an input-gradient job writes its bf16 tile.
//
// Both job kinds run wgrad256.hip's ping-pong pipeline (BK = 32, four LDS stages, LDS-DMA three
// steps ahead, 8 waves as 2 x 4 with 128 x 64 outputs each, waves 4-7 one barrier behind waves
// 0-3). The MFMA rows (A operand, transposed reads of a [k][256] image) are
//   weight gradient: n  (A = dY as [k = m][n]),     columns kk (B = X as [k = m][kk], transposed reads)
//   input gradient:  kk (A = W  as [k = n][kk]),    columns m  (B = dY rows [m][k = n]: a [256][32]
//                    image of 64-B rows read by ds_read_b128 — chunk slot q ^ 2 ((row >> 3) & 1),
//                    conflict-free for all four lane groups, model in the commit's check)
// so W is read as stored (no transpose pass) and a lane's input-gradient accumulators are 4
// consecutive kk of one token: the epilogue stages the bf16 tile in LDS ([256 m][256 kk], 16-B
// units XOR-swizzled by the row) and writes 16-B pieces, 512 B per row.
//
// Reference: /root/reference has no kernels; this is the compute behind the gradient each
// Linear leaf contributes to DistributedOptimizer's reduction (src/optimizer.jl:20-23), for
// the ViT-B/16 config of BASELINE.json.
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4v;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void gl_void;

constexpr int kThreads = 512;
constexpr int kTile = 256;
constexpr int BK = 32, ST = 4;
constexpr int kImgBytes = BK * kTile * 2;  // 16 KiB: a [32][256] (transposed) or [256][32] (row) image
constexpr int kStageBytes = 2 * kImgBytes;
constexpr int kP = kImgBytes / 1024 / 8;   // 2 DMA pieces (1 KiB each) per wave per operand per step
constexpr int kRowT = kTile * 2;           // 512-B rows of a transposed-read image
constexpr int kSmem = ST * kStageBytes;    // 128 KiB

__device__ __attribute__((aligned(16))) uint4 g_zero_lb[4];

// transposed-read images: chunk slot = chunk ^ swz(k row) (wgrad256.hip)
__device__ __forceinline__ int swz(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }
// row images ([256][32], 64-B rows): chunk slot = chunk ^ rsw(row)
__device__ __forceinline__ int rsw(int row) { return ((row >> 3) & 1) << 1; }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

struct LBArgs {
  const bf16* dy;  // [M][ldy]
  const bf16* x;   // [M][ldx]
  const bf16* w;   // [N][ldw]
  bf16* dx;        // [M][lddx]
  float* ws;       // [splits][N][K]
  int64_t M, N, K;
  int64_t ldy, ldx, ldw, lddx;
  int64_t k_per_split;  // weight gradient: tokens per split (a multiple of BK)
  int wg_jobs;          // weight-gradient jobs (tiles x splits; 0: none)
  int wg_tiles;         // (N / 256) * (K / 256)
  int dg_tiles;         // (M / 256) * (K / 256) (0: no input gradient)
  int dg_first;         // grid order: input-gradient tiles first (else weight-gradient jobs first)
};

// bijective XCD-aware order inside a segment [s0, s0 + n) of the grid: the blocks that share an
// XCD (b % 8, a speed assumption only) take a contiguous range of job ids
__device__ __forceinline__ int seg_order(int b, int s0, int n) {
  const int x = b % 8, local = b - s0;
  const int off0 = ((x - s0 % 8) % 8 + 8) % 8;  // first local index on XCD x
  int start = 0;
  for (int y = 0; y < x; ++y) {
    const int oy = ((y - s0 % 8) % 8 + 8) % 8;
    start += n > oy ? (n - oy + 7) / 8 : 0;
  }
  return start + (local - off0) / 8;
}

template <bool DG>
__device__ __forceinline__ void job(const LBArgs& p, char* smem, int id) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;
  // the job: rows r0 (MFMA rows), columns c0, reduction range [kbeg, kend)
  int64_t r0, c0, kbeg, kend;
  int split = 0;
  const int tk = static_cast<int>(p.K / kTile);
  if (DG) {
    const int tm = id / tk, tc = id - tm * tk;
    r0 = static_cast<int64_t>(tc) * kTile;  // kk
    c0 = static_cast<int64_t>(tm) * kTile;  // m
    kbeg = 0, kend = p.N;
  } else {
    split = id / p.wg_tiles;
    const int bid = id - split * p.wg_tiles;
    const int tn = bid / tk, tc = bid - tn * tk;
    r0 = static_cast<int64_t>(tn) * kTile;  // n
    c0 = static_cast<int64_t>(tc) * kTile;  // kk
    kbeg = static_cast<int64_t>(split) * p.k_per_split;
    kend = kbeg + p.k_per_split < p.M ? kbeg + p.k_per_split : p.M;
  }
  const int nk = kend > kbeg ? static_cast<int>((kend - kbeg + BK - 1) / BK) : 0;
  const int klim = static_cast<int>(kend - kbeg);

  // A (transposed reads of a [k][256] image): DG: W rows n, columns kk; else dY rows m, columns n
  const bf16* ga = DG ? p.w : p.dy;
  const int64_t lda = DG ? p.ldw : p.ldy;
  // B: DG: dY as a [256 m][32 n] row image; else X as a [k = m][256 kk] transposed image
  const bf16* gb = DG ? p.dy : p.x;
  const int64_t ldb = DG ? p.ldy : p.ldx;
  const bf16* pa[kP];
  const bf16* pb[kP];
  int krow[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const int piece = wave * kP + j;
    const int row = 2 * piece + (lane >> 5);  // transposed image: 2 k-rows of 512 B per piece
    const int chunk = (lane & 31) ^ swz(row);
    krow[j] = row;
    pa[j] = ga + (kbeg + row) * lda + r0 + chunk * 8;
    if (DG) {
      const int rr = 16 * piece + (lane >> 2);  // row image: 16 rows of 64 B per piece
      pb[j] = gb + (c0 + rr) * ldb + kbeg + (((lane & 3) ^ rsw(rr)) << 3);
    } else {
      pb[j] = gb + (kbeg + row) * ldb + c0 + chunk * 8;
    }
  }
  const int64_t stepA = static_cast<int64_t>(BK) * lda;
  const int64_t stepB = DG ? static_cast<int64_t>(BK) : static_cast<int64_t>(BK) * ldb;
  auto issue = [&](int t, bool b_op) {
    char* img = smem + (t % ST) * kStageBytes + (b_op ? kImgBytes : 0);
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      // k rows past the job's end read a zero line (same instruction count: the waits stay exact);
      // the row image's k is the step's column range: the whole 32 are in range or none
      const bool ok = b_op && DG ? t * BK < klim : krow[j] + t * BK < klim;
      const void* src = ok ? static_cast<const void*>(b_op ? pb[j] + t * stepB : pa[j] + t * stepA)
                           : static_cast<const void*>(g_zero_lb);
      __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(img + (wave * kP + j) * 1024), 16, 0, 0);
    }
  };

  // fragment offsets (k-step 0)
  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pq = li & 3;
  const int k0 = 8 * g + qq;
  const int sw = swz(k0);
  int offA[8], offB[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int col = wm * 128 + i * 16 + 4 * pq;
    offA[i] = k0 * kRowT + ((((col >> 3) ^ sw)) << 4) + (col & 7) * 2;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (DG) {
      const int row = wn * 64 + j * 16 + li;  // token row of the [256][32] image, chunk g
      offB[j] = row * 64 + ((g ^ rsw(row)) << 4);
    } else {
      const int col = wn * 64 + j * 16 + 4 * pq;
      offB[j] = k0 * kRowT + ((((col >> 3) ^ sw)) << 4) + (col & 7) * 2;
    }
  }
  auto frag_t = [&](const char* __restrict__ img, int off) {
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + off + 4 * kRowT));
    bf16x8 out;
    __builtin_memcpy(&out, &lo, 8);
    __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
    return out;
  };
  auto frag_r = [&](const char* __restrict__ img, int off) { return *reinterpret_cast<const bf16x8*>(img + off); };

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
        for (int j = 0; j < 4; ++j) fb[j] = DG ? frag_r(tb, offB[j]) : frag_t(tb, offB[j]);
      }
      bf16x8 fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_t(ta, offA[4 * ph + i]);
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
  // acc[i][j][r]: MFMA row R = wm*128 + i*16 + 4g + r, column C = wn*64 + j*16 + li
  if (!DG) {
    float* c = p.ws + static_cast<int64_t>(split) * p.N * p.K;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = c0 + wn * 64 + j * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = r0 + wm * 128 + i * 16 + 4 * g + r;
          c[row * p.K + col] = acc[i][j][r];
        }
      }
    return;
  }
  // input gradient: [256 m][256 kk] bf16 in LDS (512-B rows, 16-B unit u of row m at u ^ (m & 15)),
  // then 16-B coalesced stores
  __syncthreads();  // every wave's last fragment reads are done: the stages are free
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = wn * 64 + j * 16 + li;
      const int kk = wm * 128 + i * 16 + 4 * g;  // 4 consecutive kk: half of 16-B unit kk / 8
      bf16 o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = static_cast<bf16>(acc[i][j][r]);
      uint2 v;
      __builtin_memcpy(&v, o, 8);
      const int u = (kk >> 3) ^ (m & 15);
      *reinterpret_cast<uint2*>(smem + m * 512 + u * 16 + (kk & 4) * 2) = v;
    }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kTile * 32 / kThreads; ++q) {  // 16 pieces per thread
    const int idx = q * kThreads + threadIdx.x;
    const int m = idx >> 5, u = idx & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(smem + m * 512 + ((u ^ (m & 15)) << 4));
    *reinterpret_cast<uint4*>(p.dx + (c0 + m) * p.lddx + r0 + u * 8) = v;
  }
}

__global__ __launch_bounds__(kThreads, 2) void linbwd_kernel(LBArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  if (p.dg_first) {
    if (b < p.dg_tiles) job<true>(p, smem, seg_order(b, 0, p.dg_tiles));
    else job<false>(p, smem, seg_order(b, p.dg_tiles, p.wg_jobs));
  } else {
    if (b < p.wg_jobs) job<false>(p, smem, seg_order(b, 0, p.wg_jobs));
    else job<true>(p, smem, seg_order(b, p.wg_jobs, p.dg_tiles));
  }
}

}  // namespace

bool linear_bwd_supported(int64_t M, int64_t N, int64_t K, int64_t ldy, int64_t ldx, int64_t ldw, int64_t lddx) {
  return M > 0 && N > 0 && K > 0 && M % kTile == 0 && N % kTile == 0 && K % kTile == 0 && M < (int64_t(1) << 31) &&
         ldy % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0 && lddx % 8 == 0 && ldy >= N && ldx >= K && ldw >= K &&
         lddx >= K && (M / kTile) * (K / kTile) < (int64_t(1) << 30);
}

int linear_bwd_splits(int64_t M, int64_t N, int64_t K, int splits) {
  if (splits < 1) splits = 1;
  const int64_t nk = (M + BK - 1) / BK;
  const int64_t kps = (nk + splits - 1) / splits * BK;
  return static_cast<int>((M + kps - 1) / kps);
}

void linear_bwd(const void* dy, const void* x, const void* w, void* dx, float* ws, int64_t M, int64_t N, int64_t K,
                int64_t ldy, int64_t ldx, int64_t ldw, int64_t lddx, int splits, int dg_first, hipStream_t stream) {
  if (!linear_bwd_supported(M, N, K, ldy, ldx, ldw, lddx))
    throw std::runtime_error("linear_bwd: need M, N, K multiples of 256 and 8-aligned leading dimensions (M=" +
                             std::to_string(M) + " N=" + std::to_string(N) + " K=" + std::to_string(K) + ")");
  if (((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) |
        reinterpret_cast<uintptr_t>(dx)) & 15u) != 0)
    throw std::runtime_error("linear_bwd: operands must be 16-byte aligned");
  LBArgs p{};
  p.dy = static_cast<const bf16*>(dy), p.x = static_cast<const bf16*>(x), p.w = static_cast<const bf16*>(w);
  p.dx = static_cast<bf16*>(dx), p.ws = ws;
  p.M = M, p.N = N, p.K = K, p.ldy = ldy, p.ldx = ldx, p.ldw = ldw, p.lddx = lddx;
  p.wg_tiles = static_cast<int>((N / kTile) * (K / kTile));
  if (ws != nullptr) {
    if (splits < 1) splits = 1;
    const int64_t nk = (M + BK - 1) / BK;
    p.k_per_split = (nk + splits - 1) / splits * BK;
    const int s = static_cast<int>((M + p.k_per_split - 1) / p.k_per_split);
    p.wg_jobs = s * p.wg_tiles;
  }
  p.dg_tiles = dx != nullptr ? static_cast<int>((M / kTile) * (K / kTile)) : 0;
  p.dg_first = dg_first;
  const int64_t grid = static_cast<int64_t>(p.wg_jobs) + p.dg_tiles;
  if (grid == 0) return;
  static bool attr = false;
  if (!attr) {
    FLUXMPI_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&linbwd_kernel),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, kSmem));
    attr = true;
  }
  linbwd_kernel<<<static_cast<unsigned>(grid), kThreads, kSmem, stream>>>(p);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
