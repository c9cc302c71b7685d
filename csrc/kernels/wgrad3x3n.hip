// Weight gradient of the narrow-channel 3x3 / stride 1 / pad 1 convolution, NHWC bf16 — gfx950.
//
//   dW[co][tap][ci] = sum over pixels p of dY[p][co] * X[p + shift(tap)][ci],  tap = 3 (dr + 1) + (ds + 1)
//
// ResNet-50's stage-1 (C = 64, 56 x 56) and stage-2 (C = 128, 28 x 28) 3x3 weight gradients ran at
// 18 / 25 % of the bf16 peak on the split-K LDS-DMA kernel (profiles/rd5g_roofline_resnet50.md):
// its B operand is the implicit im2col, so each input pixel crosses L2 -> LDS once per tap and dY
// once per 128-column tile (~1.5 GB of L2 -> LDS traffic for 0.2 GB of operands). Here a workgroup
// walks blocks of kR image rows:
//   * the block's dY rows and the kR + 2 input rows around them (zeros outside the image) are
//     staged ONCE into LDS, the input in a layout with zero columns either side of each row, so the
//     nine taps are nine constant offsets into one image: no masks, no per-tap loads;
//   * both MFMA operands run along pixels (the GEMM's k) and are read with ds_read_b64_tr_b16. A
//     read's 32-lane half takes two runs of 4 consecutive pixels, and pixel slots lie C * 2 + 32
//     bytes apart (an odd multiple of 8 banks): the 8 rows of a half land on 8 disjoint 8-bank
//     windows whatever the tap offset, provided the second run starts 4 slots (mod 8) after the
//     first — true inside an image row, and across rows once the row pitch P == W (mod 8);
//   * the next block's rows are loaded into registers during this block's MFMAs (ds_write after a
//     barrier: an LDS-DMA ring makes the waitcnt pass drain it in front of the reads, conv3x3n.hip);
//     DEPTH 2 keeps the next two blocks in flight in two register sets.
// The workgroup's output is COB (64 / 128) co x TG taps x C ci. Its 4 or 8 waves split the columns (and with 8
// the co rows in halves) and keep fp32 sums in registers across all blocks of their K-split;
// partials [splits][Cout][9 C] go through the shared split-K reduce (gemm_splitk_reduce).
// Reference: /root/reference has no kernels — this is the compute under the per-step gradient work
// of the ResNet-50 DDP configuration (BASELINE.json, src/optimizer.jl:20-23).
#include <cstdint>
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

constexpr int kR = 4;       // image rows per block
constexpr uint32_t kOOB = 0x80000000u;  // a buffer offset past every operand: the load returns zeros

// COB: output channels per workgroup (64, or 128 for the 128-channel layers: half the input
// re-reads of two 64-channel workgroups)
template <int C, int COB> struct Geo3 {
  static constexpr int kW = C == 64 ? 56 : 28;            // widest supported image row
  static constexpr int kP = kW % 8 == 0 ? kW + 2 : kW + 8;  // its padded row pitch
  static constexpr int kSB = C * 2 + 32;                  // input slot stride: 40 / 72 banks
  static constexpr int kSA = COB * 2 + 32;                // dY slot stride: 40 / 72 banks
  static constexpr int kXBytes = (kR + 2) * kP * kSB;
  static constexpr int kDBytes = kR * kW * kSA;
  static constexpr int kBytes = kXBytes + kDBytes + kSA;  // + one zero dY slot
};

__host__ __device__ constexpr int pitch_of(int W) { return W % 8 == 0 ? W + 2 : W + 8; }

struct W3Args {
  const bf16* dy;  // [N][H][W][CO]
  const bf16* x;   // [N][H][W][C]
  float* ws;       // [splits][CO][9 C]
  uint32_t dy_bytes, x_bytes;
  int H, W, CO;
  int nblocks;     // N * H / kR
  int per_split;   // blocks per K-split
  int groups;      // (CO / COB) * (9 / TG) output blocks per split
};

__device__ __forceinline__ short4v tr_read(const char* lds, int byte) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(lds + byte));
}

__device__ __forceinline__ bf16x8 join(short4v lo, short4v hi) {
  bf16x8 out;
  __builtin_memcpy(&out, &lo, 8);
  __builtin_memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
  return out;
}

template <int C, int TG, int NWM, int DEPTH, int COB>
__global__ __launch_bounds__(256 * NWM, 1) void wgrad3x3n_kernel(W3Args p) {
  using G = Geo3<C, COB>;
  constexpr int kSA = G::kSA;
  constexpr int DPP = COB / 8;               // 16-B dY pieces per pixel
  constexpr int NT = 256 * NWM;
  constexpr int CW = COB / NWM;              // co rows per wave
  constexpr int FI = CW / 16;                // A fragments per wave
  constexpr int CF = C / 16;                 // 16-column fragments per tap
  constexpr int NF = TG * CF / 4;            // B fragments per wave
  static_assert(TG * CF % 4 == 0, "tap group split");
  constexpr int kXP = (kR + 2) * G::kW * C / 8;  // 16-B input pieces of a block (widest row)
  constexpr int kDP = kR * G::kW * COB / 8;      // 16-B dY pieces
  constexpr int JX = (kXP + NT - 1) / NT, JD = (kDP + NT - 1) / NT;
  constexpr int DB = G::kXBytes, ZB = G::kXBytes + G::kDBytes;
  __shared__ __attribute__((aligned(1024))) char lds[G::kBytes];

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wm = wave / 4, wn = wave % 4;
  const int H = p.H, W = p.W, P = pitch_of(W), CO = p.CO;
  const int hb = H / kR;
  // (split, group) of this workgroup; XCD-aware: the workgroups of one XCD take a contiguous range,
  // so the groups of one split (same pixels, other output columns) share that XCD's L2
  int lid = blockIdx.x;
  const int total = static_cast<int>(gridDim.x);
  if (total >= 8) {
    const int q = total / 8, r = total % 8, xcd = lid % 8, pos = lid / 8;
    lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  lid = __builtin_amdgcn_readfirstlane(lid);
  const int split = lid / p.groups, grp = lid - split * p.groups;
  constexpr int NTG = 9 / TG;
  const int co0 = (grp / NTG) * COB, t0 = (grp % NTG) * TG;
  const int b0 = split * p.per_split;
  const int b1 = b0 + p.per_split < p.nblocks ? b0 + p.per_split : p.nblocks;

  // ---- zero the pad columns of the input rows and the zero dY slot (never written again)
  {
    constexpr int SP = G::kSB / 16;  // 16-B pieces per input slot
    const int padc = P - W;          // pad slots per row: column 0 and W + 1 .. P - 1
    const int npad = (kR + 2) * padc * SP;
    for (int i = tid; i < npad + kSA / 16; i += NT) {
      int off;
      if (i < npad) {
        const int s = i / SP, piece = i - s * SP;
        const int rr = s / padc, k = s - rr * padc;
        off = (rr * P + (k == 0 ? 0 : W + k)) * G::kSB + piece * 16;
      } else {
        off = ZB + (i - npad) * 16;
      }
      *reinterpret_cast<uint4*>(lds + off) = uint4{0, 0, 0, 0};
    }
  }

  // ---- staging: this thread's 16-B pieces (the same LDS places for every block)
  const int NX = (kR + 2) * W * C / 8, ND = kR * W * COB / 8;
  int xl[JX];
#pragma unroll
  for (int j = 0; j < JX; ++j) {
    const int i = j * NT + tid;
    const int pi = i / (C / 8), c = i - pi * (C / 8);
    const int rr = pi / W, w = pi - rr * W;
    xl[j] = (rr * P + w + 1) * G::kSB + c * 16;
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.x), 0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.dy), 0, p.dy_bytes, 0x00020000);
  using XV = uint4[JX];
  using DV = uint4[JD];
  XV xa, xb;
  DV da, db;
  auto load = [&](int b, XV& xv, DV& dv) {
    const int n = b / hb, h0 = (b - n * hb) * kR;
    const int64_t xbase = (static_cast<int64_t>(n) * H + h0 - 1) * W * C * 2;
#if W3N_DIAG_NOHALO  // diagnostics: the halo rows not loaded (wrong results; their traffic's price)
    const int lo = W * C / 8, hi = (kR + 1) * W * C / 8;
#else
    const int lo = h0 == 0 ? W * C / 8 : 0;
    const int hi = h0 + kR == H ? (kR + 1) * W * C / 8 : NX;
#endif
#pragma unroll
    for (int j = 0; j < JX; ++j) {
      const int i = j * NT + tid;
#if W3N_DIAG_NOLOAD  // diagnostics: every load out of bounds (no memory traffic)
      const uint32_t off = i > (1 << 30) ? static_cast<uint32_t>(xbase + i * 16 + lo + hi) : kOOB;
#else
      const uint32_t off = i >= lo && i < hi ? static_cast<uint32_t>(xbase + i * 16) : kOOB;
#endif
      xv[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
    const int64_t dbase = (static_cast<int64_t>(n) * H + h0) * W * CO * 2 + co0 * 2;
#pragma unroll
    for (int j = 0; j < JD; ++j) {
      const int i = j * NT + tid;
#if W3N_DIAG_NOLOAD
      const uint32_t off = i > (1 << 30) ? static_cast<uint32_t>(dbase) : kOOB;
#else
      const uint32_t off = i < ND ? static_cast<uint32_t>(dbase + (i / DPP) * CO * 2 + (i % DPP) * 16) : kOOB;
#endif
      dv[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dr, off, 0, 0));
    }
  };
  auto store = [&](const XV& xv, const DV& dv) {
#pragma unroll
    for (int j = 0; j < JX; ++j)
      if (j * NT + tid < NX) *reinterpret_cast<uint4*>(lds + xl[j]) = xv[j];
#pragma unroll
    for (int j = 0; j < JD; ++j) {
      const int i = j * NT + tid;
      if (i < ND) *reinterpret_cast<uint4*>(lds + DB + (i / DPP) * kSA + (i % DPP) * 16) = dv[j];
    }
  };

  // ---- the lane's pixels: read r of step s takes pixel 32 s + 8 r + c0 of the block for MFMA row
  // k = 8 g + 4 r + q (g = lane / 16, q = (lane / 4) % 4): each 32-lane half reads two runs of 4
  // consecutive pixels; pc = lane % 4 picks the 4 columns of the 16 that the lane fetches
  const int g = lane >> 4, q = (lane >> 2) & 3, pc = lane & 3;
  const int c0 = 16 * (g >> 1) + 4 * (g & 1) + q;
#if W3N_DIAG_NOCOMPUTE  // diagnostics: no k-steps (the staging alone)
  const int RW = kR * W, nstep = W < 0 ? 1 : 0;
#else
  const int RW = kR * W, nstep = (RW + 31) / 32;
#endif
  // pixel px -> (row, column) without a divide: px < 2^9 and W <= 56, so px * ceil(2^20 / W) >> 20
  // is exact
  const uint32_t invw = ((1u << 20) + W - 1) / W;
  // B fragments: wave wn takes the 16-channel blocks wn + 4 j of every tap of the group, so a
  // fragment's offset from the wave's base is (filter row) x P + (filter column) slots + 128 j bytes:
  // compile-time except the row term (P is the runtime pitch), one base per filter row
  constexpr int TR = TG / 3;  // filter rows per workgroup (the tap group is whole rows)
  constexpr int JB = CF / 4;  // channel blocks per wave and tap
  const int bwave = __builtin_amdgcn_readfirstlane((t0 / 3) * P * G::kSB + wn * 32);
  f32x4 acc[FI][NF];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the fragments of step s (issue only: the waitcnt pass waits for them at their first MFMA)
  auto read = [&](int s, bf16x8 (&fa)[FI], bf16x8 (&fb)[NF]) {
    int aa[2], bb[2][TR];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int px = 32 * s + 8 * r + c0;
      const int row = static_cast<int>((static_cast<uint32_t>(px) * invw) >> 20), col = px - row * W;
      const bool ok = px < RW;  // a partial last step reads zero dY rows (and finite input)
      aa[r] = (ok ? DB + px * kSA : ZB) + wm * CW * 2 + pc * 8;
      const int base = (ok ? (row * P + col) * G::kSB : 0) + bwave + pc * 8;
#pragma unroll
      for (int d = 0; d < TR; ++d) bb[r][d] = base + d * P * G::kSB;
    }
#pragma unroll
    for (int i = 0; i < FI; ++i) fa[i] = join(tr_read(lds, aa[0] + i * 32), tr_read(lds, aa[1] + i * 32));
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int tl = f / JB, j = f % JB;
      const int off = (tl % 3) * G::kSB + j * 128;
      fb[f] = join(tr_read(lds, bb[0][tl / 3] + off), tr_read(lds, bb[1][tl / 3] + off));
    }
  };
  auto mma = [&](const bf16x8 (&fa)[FI], const bf16x8 (&fb)[NF]) {
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f)
        acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[f], acc[i][f], 0, 0, 0);
  };
  // software-pipelined k-steps: step s + 1's fragment reads are interleaved with step s's MFMAs
  // (two fragment sets), so the LDS latency hides under the matrix work and fewer than 16 reads
  // are ever outstanding (lgkmcnt's range: a burst of all 2 (FI + NF) reads made the waitcnt pass
  // drain most of the next step's reads before this step's first MFMA). The tail step re-reads the
  // last one into the spare set (harmless) to keep the loop body free of branches.
  auto compute = [&]() {
    bf16x8 fa0[FI], fb0[NF], fa1[FI], fb1[NF];
    read(0, fa0, fb0);
    int s = 0;
    for (; s + 1 < nstep; s += 2) {
      read(s + 1, fa1, fb1);
      mma(fa0, fb0);
      interleave_mfma_ds<0, FI * NF, 2 * (FI + NF)>();
      read(s + 2 < nstep ? s + 2 : nstep - 1, fa0, fb0);
      mma(fa1, fb1);
      interleave_mfma_ds<0, FI * NF, 2 * (FI + NF)>();
    }
    if (s < nstep) mma(fa0, fb0);
  };

  // the next block's rows are in flight during this block's MFMAs (DEPTH 1), or the next two blocks'
  // (DEPTH 2: two register sets, so a load has two blocks' time to arrive)
  if (b0 < b1) {
    load(b0, xa, da);
    store(xa, da);
  }
  if (DEPTH == 2 && b0 + 1 < b1) load(b0 + 1, xb, db);
  __syncthreads();
  if constexpr (DEPTH == 1) {
    for (int b = b0; b < b1; ++b) {
      const bool more = b + 1 < b1;
      if (more) load(b + 1, xa, da);
      __builtin_amdgcn_sched_barrier(0);  // keep the loads at the top: their latency hides under the MFMAs
      compute();
      if (more) {
        __syncthreads();  // every wave is done reading this block
        store(xa, da);
      }
      __syncthreads();
    }
  } else {
    for (int b = b0; b < b1; b += 2) {
      if (b + 2 < b1) load(b + 2, xa, da);  // set b holds block b + 1
      __builtin_amdgcn_sched_barrier(0);
      compute();
      if (b + 1 < b1) {
        __syncthreads();
        store(xb, db);
      }
      __syncthreads();
      if (b + 1 >= b1) break;
      if (b + 3 < b1) load(b + 3, xb, db);  // set a holds block b + 2
      __builtin_amdgcn_sched_barrier(0);
      compute();
      if (b + 2 < b1) {
        __syncthreads();
        store(xa, da);
      }
      __syncthreads();
    }
  }

  // ---- fp32 partials: acc[i][f][r] = dW[co0 + wm CW + 16 i + 4 g + r][(t0 + tl) C + 16 (wn + 4 j) + lane % 16]
  float* out = p.ws + static_cast<int64_t>(split) * CO * 9 * C;
#if W3N_DIAG_NOSTORE  // diagnostics: only split 0 stores its partials (the partial traffic's price)
  if (split != 0) return;
#endif
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int tl = f / JB, j = f % JB;
      const int col = (t0 + tl) * C + 16 * (wn + 4 * j) + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * CW + 16 * i + 4 * g + r;
        out[static_cast<int64_t>(co) * 9 * C + col] = acc[i][f][r];
      }
    }
}

template <int C, int TG, int NWM, int DEPTH, int COB = 64>
void launch3(const W3Args& a, int splits, hipStream_t s) {
  wgrad3x3n_kernel<C, TG, NWM, DEPTH, COB><<<splits * a.groups, 256 * NWM, 0, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

bool wgrad3x3n_supported(int64_t N, int H, int W, int C, int Cout) {
  if (C != 64 && C != 128) return false;
  const int maxw = C == 64 ? Geo3<64, 64>::kW : Geo3<128, 64>::kW;
  const int maxp = C == 64 ? Geo3<64, 64>::kP : Geo3<128, 64>::kP;
  return N >= 1 && H >= kR && H % kR == 0 && W >= 4 && W % 4 == 0 && W <= maxw && pitch_of(W) <= maxp &&
         Cout >= 64 && Cout % 64 == 0 && N * H * W * static_cast<int64_t>(C > Cout ? C : Cout) * 2 < (int64_t(1) << 31);
}

int wgrad3x3n_splits(int64_t N, int H, int splits) {
  const int64_t nb = N * (H / kR);
  const int64_t s = splits < 1 ? 1 : (splits > nb ? nb : splits);
  const int64_t per = (nb + s - 1) / s;
  return static_cast<int>((nb + per - 1) / per);
}

// variant bit 2 (C = 128, Cout % 128 == 0): 128 output channels per workgroup
static int cob_of(int C, int Cout, int variant) { return C == 128 && (variant & 4) && Cout % 128 == 0 ? 128 : 64; }

int wgrad3x3n_groups(int C, int Cout, int variant) {
  return (Cout / cob_of(C, Cout, variant)) * (C == 64 ? 1 : 3);
}

void wgrad3x3n(const void* dy, const void* x, float* ws, int64_t N, int H, int W, int C, int Cout, int splits,
               int variant, hipStream_t stream) {
  if (!wgrad3x3n_supported(N, H, W, C, Cout))
    throw std::runtime_error("wgrad3x3n: unsupported shape (C in {64, 128}, Cout % 64 == 0, H % 4 == 0, W % 4 == 0, "
                             "W <= 56 / 28; N=" + std::to_string(N) + " H=" + std::to_string(H) + " W=" +
                             std::to_string(W) + " C=" + std::to_string(C) + " Cout=" + std::to_string(Cout) + ")");
  if (((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(ws)) & 15u) != 0)
    throw std::runtime_error("wgrad3x3n: operands must be 16-byte aligned");
  W3Args a{};
  a.dy = static_cast<const bf16*>(dy), a.x = static_cast<const bf16*>(x), a.ws = ws;
  a.dy_bytes = static_cast<uint32_t>(N * H * W * Cout * 2);
  a.x_bytes = static_cast<uint32_t>(N * H * W * C * 2);
  a.H = H, a.W = W, a.CO = Cout;
  a.nblocks = static_cast<int>(N * (H / kR));
  const int sp = wgrad3x3n_splits(N, H, splits);
  a.per_split = (a.nblocks + sp - 1) / sp;
  a.groups = wgrad3x3n_groups(C, Cout, variant);
  const bool w8 = variant & 1, d2 = variant & 2;
  if (C == 64) {
    if (w8) launch3<64, 9, 2, 1>(a, sp, stream);  // (8 waves with two register sets spill)
    else { if (d2) launch3<64, 9, 1, 2>(a, sp, stream); else launch3<64, 9, 1, 1>(a, sp, stream); }
  } else if (cob_of(C, Cout, variant) == 128) {
    if (w8) launch3<128, 3, 2, 1, 128>(a, sp, stream); else launch3<128, 3, 1, 1, 128>(a, sp, stream);
  } else {
    if (w8) launch3<128, 3, 2, 1>(a, sp, stream);
    else { if (d2) launch3<128, 3, 1, 2>(a, sp, stream); else launch3<128, 3, 1, 1>(a, sp, stream); }
  }
}

}  // namespace fluxmpi
