// Narrow-channel 3x3 / stride 1 / pad 1 convolution, NHWC bf16, as an implicit GEMM whose input
// halo is staged ONCE per workgroup — gfx950.
//
// Shapes: C = Cout = 64 (ResNet-50 stage 1, 56 x 56) and 128 (stage 2, 28 x 28), forward (with the
// next BatchNorm's statistics in the epilogue) and input gradient (the same convolution over dy
// with the flipped, transposed filter). These are the layers the 256 x 256 kernels cannot take
// (Cout < 256) and the 128-tile LDS-DMA kernel ran at 18-26 % of the bf16 peak
// (profiles/rd3f_roofline_resnet50.md): it stages every k-tile of the implicit im2col through
// LDS, so each input pixel crosses L2 -> LDS nine times, and its 128-wide B tile is twice the
// layer's width.
//
// Here a workgroup owns 256 consecutive output pixels (rows of the implicit GEMM) and ALL output
// channels:
//   * its input halo — pixels m0 - W - 1 .. m0 + 256 + W (the 3 x 3 neighbourhoods of its rows in
//     flattened NHWC order) — is DMA'd into LDS once (global_load_lds_dwordx4 through a buffer
//     resource: pixels before the first / after the last read as zeros), as C / 64 planes of
//     128-B rows with chunk slot q ^ (row & 7): every 16-row fragment read, whatever its start
//     row (a tap shifts the rows by (dr + 1) W + dc + 1), is bank-conflict free for
//     ds_read_b128's lane groups (model: scripts/lds_banks.py);
//   * the filter streams one tap (Cout x C) at a time through a double-buffered LDS slot, the
//     next tap's loads in flight (into registers) during this tap's MFMAs;
//   * a tap that falls outside the image (row / column / image boundary in flattened order)
//     redirects the lane's fragment read to a zero row: one address select per read, no data
//     masking.
// 8 waves x 32 rows (64 channels; 128 channels: 16 waves, two per 32-row block on half of the
// output channels each): per tap and 32-channel k-step a wave reads one filter fragment per 16 of
// its output channels and 2 activation fragments (ds_read_b128) for two MFMAs per filter fragment
// (v_mfma_f32_16x16x32_bf16).
// Reference: /root/reference has no kernels — this is the compute under the per-step gradient
// work of the ResNet-50 DDP configuration (BASELINE.json, src/optimizer.jl:20-23).
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
typedef __attribute__((address_space(3))) char lds_char;

constexpr int kTM = 256;     // output pixels per workgroup
#ifndef C3N_TAIL_CO
#define C3N_TAIL_CO 16
#endif
#ifndef C3N_W128
#define C3N_W128 16
#endif
// waves per workgroup: 8 x 32 rows; the 128-channel kernel (one workgroup per CU: 150 KB of LDS)
// runs 16, two per 32-row block, each on half of the output channels: 4 waves per SIMD instead of
// 2 (104 VGPRs), 77.5 vs 81.2 us per call at 28 x 28 x 128 x 256 images, 64.7 vs 69.0 at 240
// (profiles/rd5ax_conv3x3n_16waves_ab.jsonl)
template <int CO> constexpr int waves_of() { return CO == 128 ? C3N_W128 : 8; }
constexpr int kShards = 64;  // BatchNorm statistics shards (== batchnorm.hip)

// halo rows for the widest image each channel count supports (LDS sizing)
template <int C> struct Geo {
  static constexpr int kPlanes = C / 64;
  static constexpr int kMaxW = C == 64 ? 64 : 32;
  static constexpr int kHalo = (kTM + 2 * kMaxW + 2 + 7) / 8 * 8;  // rows, a multiple of the DMA's 8
  static constexpr int kPlaneBytes = (kHalo + 8) * 128;             // + the zero rows
  static constexpr int kZeroRow = kHalo;
};

struct CNArgs {
  const bf16* x;   // [M][C] (NHWC image batch)
  const bf16* w;   // [Cout][9][C] (tap-major: a channels_last filter, or the dgrad's flipped transpose)
  bf16* y;         // [M][Cout]
  float* stats;    // EPI 3: [kShards][2][Cout]
  int H, W;
  int tiles;
  int m_base;      // pixel of tile 0
  int ncob;        // output-channel blocks of CO per tile (workgroup b: tile b / ncob, block b % ncob)
  int ldy;         // output channels of y (and of the statistics) = ncob * CO
  uint32_t x_bytes;
};

__device__ __forceinline__ bf16x8 frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

template <int C, int CO, int EPI>
__global__ __launch_bounds__(64 * waves_of<CO>(), C == 64 ? 4 : (waves_of<CO>() == 16 ? 4 : 2)) void conv3x3n_kernel(CNArgs p) {
  using G = Geo<C>;
  constexpr int kWaves = waves_of<CO>(), kThreads = 64 * kWaves;
  constexpr int NPL = G::kPlanes;
  constexpr int KS = C / 32;               // 32-channel k-steps per tap
  constexpr int WN = kWaves / 8, WM = 8;   // wave grid: 8 row blocks of 32 x WN column blocks
  constexpr int NB = CO / WN / 16;         // 16-column blocks per wave
  constexpr int kBBytes = NPL * CO * 128;  // one tap of the filter
  __shared__ __attribute__((aligned(1024))) char halo[NPL * G::kPlaneBytes];
  __shared__ __attribute__((aligned(1024))) char bbuf[2 * kBBytes];

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  // XCD-aware tile order: the workgroups of one XCD (b % 8) take a contiguous range of tiles, so
  // neighbouring tiles' shared halo rows meet in that XCD's L2 (speed only)
  int tile = blockIdx.x / p.ncob;
  const int co0 = (blockIdx.x - tile * p.ncob) * CO;  // first output channel of this workgroup
  if (p.ncob == 1 && p.tiles % 8 == 0) tile = (blockIdx.x % 8) * (p.tiles / 8) + blockIdx.x / 8;
  tile = __builtin_amdgcn_readfirstlane(tile);
  const int W = p.W, H = p.H;
  const int m0 = p.m_base + tile * kTM;
  const int hb = m0 - W - 1;  // global pixel of halo row 0
  const int hrows = kTM + 2 * W + 2;

  // ---- prologue: zero rows, halo DMA, the first tap's filter DMA
  if (threadIdx.x < NPL * 64) {  // 8 zero rows per plane (16 B per thread)
    const int pl = threadIdx.x >> 6, q = threadIdx.x & 63;
    *reinterpret_cast<uint4*>(halo + pl * G::kPlaneBytes + G::kZeroRow * 128 + q * 16) = uint4{0, 0, 0, 0};
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.x), 0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.w) + static_cast<int64_t>(co0) * 9 * C, 0,
                                                                   0x7fffffff, 0x00020000);
  const int lrow = lane >> 3, lslot = lane & 7;
  {
    const int groups = (hrows + 7) / 8;  // DMA instructions per plane (8 rows each)
    for (int i = wave; i < groups * NPL; i += kWaves) {
      const int pl = i / groups, rg = i - pl * groups;
      const int row = rg * 8 + lrow;
      const uint32_t off = static_cast<uint32_t>((hb + row) * (C * 2) + pl * 128 + ((lslot ^ (row & 7)) << 4));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_char*)(halo + pl * G::kPlaneBytes + rg * 1024), 16, off, 0, 0, 0);
    }
  }
  auto issue_b = [&](int tap, int buf) {  // one tap of the filter: NPL * CO / 8 DMA instructions
    for (int i = wave; i < NPL * (CO / 8); i += kWaves) {
      const int pl = i / (CO / 8), rg = i - pl * (CO / 8);
      const int co = rg * 8 + lrow;
      const uint32_t off = static_cast<uint32_t>((co * 9 + tap) * (C * 2) + pl * 128 + ((lslot ^ (co & 7)) << 4));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_char*)(bbuf + buf * kBBytes + pl * CO * 128 + rg * 1024), 16, off,
                                               0, 0, 0);
    }
  };
  issue_b(0, 0);
  // taps 1..8 are prefetched through registers (global loads during the previous tap's MFMAs,
  // ds_write after them): an LDS-DMA of the next tap made the waitcnt pass drain it with a
  // vmcnt(0) in front of the current tap's reads, so nothing overlapped
  constexpr int kPieces = NPL * CO * 8;  // 16-B pieces of one tap
  constexpr int kBL = (kPieces + kThreads - 1) / kThreads;  // per lane
  static_assert(kPieces % kThreads == 0 || kPieces < kThreads, "tap staging");
  constexpr bool kAll = kPieces % kThreads == 0;  // else (16-channel tail blocks) lanes >= kPieces idle
  uint4 bpre[kBL];
  auto load_b = [&](int tap) {
#pragma unroll
    for (int j = 0; j < kBL; ++j) {
      const int idx = j * kThreads + threadIdx.x;          // (plane, co, chunk)
      const int pl = idx / (CO * 8), rem = idx - pl * CO * 8;
      const int co = rem >> 3, q = rem & 7;
      const uint32_t off = static_cast<uint32_t>((co * 9 + tap) * (C * 2) + pl * 128 + (q << 4));
      if (kAll || idx < kPieces) bpre[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int j = 0; j < kBL; ++j) {
      const int idx = j * kThreads + threadIdx.x;
      const int pl = idx / (CO * 8), rem = idx - pl * CO * 8;
      const int co = rem >> 3, q = rem & 7;
      if (kAll || idx < kPieces)
        *reinterpret_cast<uint4*>(bbuf + buf * kBBytes + pl * CO * 128 + co * 128 + ((q ^ (co & 7)) << 4)) = bpre[j];
    }
  };

  // ---- the lane's rows: local row lr = 32 wave + 16 mb + (lane & 15); in-image taps as 9-bit masks
  const int fr = lane & 15, fg = lane >> 4;
  const int wm = wave % WM, wn = wave / WM;  // the wave's 32-row block and column block
  uint32_t vmask[2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int m = m0 + wm * 32 + mb * 16 + fr;
    const int hw = m % (H * W), h = hw / W, w = hw - h * W;
    const uint32_t rm = (h > 0 ? 1u : 0u) | 2u | (h < H - 1 ? 4u : 0u);
    const uint32_t cm = (w > 0 ? 1u : 0u) | 2u | (w < W - 1 ? 4u : 0u);
    vmask[mb] = ((rm & 1u) ? cm : 0u) | ((rm & 2u) ? cm << 3 : 0u) | ((rm & 4u) ? cm << 6 : 0u);
  }
  f32x4 acc[2][NB];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int tap = 0; tap < 9; ++tap) {
    if (tap < 8) load_b(tap + 1);
    __builtin_amdgcn_sched_barrier(0);  // keep the loads at the top: their latency hides under this tap
    const int dr = tap / 3, dc = tap - 3 * dr;     // 0..2
    const char* bb = bbuf + (tap & 1) * kBBytes;
    int arow[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
      arow[mb] = (vmask[mb] >> tap) & 1u ? wm * 32 + mb * 16 + fr + dr * W + dc : G::kZeroRow;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int pl = ks / 2, ch = (ks & 1) * 4 + fg;  // plane, 16-B chunk within its 128-B row
      bf16x8 fb[NB], fa[2];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int co = wn * (NB * 16) + nb * 16 + fr;
        fb[nb] = frag(bb + pl * CO * 128 + co * 128 + ((ch ^ (co & 7)) << 4));
      }
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
        fa[mb] = frag(halo + pl * G::kPlaneBytes + arow[mb] * 128 + ((ch ^ (arow[mb] & 7)) << 4));
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nb], fa[mb], acc[mb][nb], 0, 0, 0);
    }
    if (tap < 8) store_b((tap + 1) & 1);  // that slot was last read in tap - 1 (barrier since)
    __syncthreads();
  }

  // ---- epilogue: acc[mb][nb][r] = y[m0 + 32 wave + 16 mb + (lane & 15)][16 nb + 4 (lane >> 4) + r]
  float cs[NB][4], cq[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[nb][r] = cq[nb][r] = 0.f;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    bf16* yrow = p.y + static_cast<int64_t>(m0 + wm * 32 + mb * 16 + fr) * p.ldy + co0 + wn * (NB * 16) + 4 * fg;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      bf16 o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        o[r] = static_cast<bf16>(acc[mb][nb][r]);
        if (EPI == 3) {
          const float f = static_cast<float>(o[r]);  // the statistics of the rounded output
          cs[nb][r] += f;
          cq[nb][r] = fmaf(f, f, cq[nb][r]);
        }
      }
      uint2 v;
      __builtin_memcpy(&v, o, 8);
      *reinterpret_cast<uint2*>(yrow + nb * 16) = v;
    }
  }
  if constexpr (EPI == 3) {
    // per column: the wave's 32 rows (16 row lanes x 2 blocks), then the 8 waves through LDS
    // (the halo is free: every wave passed the last tap's barrier), one atomic per column and
    // moment per workgroup into its shard
    float* red = reinterpret_cast<float*>(halo);  // [8 waves][2][CO]
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = row_sum16(cs[nb][r]), q = row_sum16(cq[nb][r]);
        if (fr == 0) {
          red[(wm * 2 + 0) * CO + wn * (NB * 16) + nb * 16 + 4 * fg + r] = s;
          red[(wm * 2 + 1) * CO + wn * (NB * 16) + nb * 16 + 4 * fg + r] = q;
        }
      }
    __syncthreads();
    if (threadIdx.x < 2 * CO) {
      const int mom = threadIdx.x / CO, col = threadIdx.x - mom * CO;
      float t = 0.f;
#pragma unroll
      for (int wv = 0; wv < WM; ++wv) t += red[(wv * 2 + mom) * CO + col];
      atomicAdd(p.stats + (static_cast<int64_t>(tile % kShards) * 2 + mom) * p.ldy + co0 + col, t);
    }
  }
}

template <int C, int CO>
void launch(const CNArgs& p, int epi, hipStream_t s) {
  const int grid = p.tiles * p.ncob;
  if (epi == 3) conv3x3n_kernel<C, CO, 3><<<grid, 64 * waves_of<CO>(), 0, s>>>(p);
  else conv3x3n_kernel<C, CO, 0><<<grid, 64 * waves_of<CO>(), 0, s>>>(p);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

// The 128-channel kernel holds one workgroup per CU (150 KB of LDS): ResNet-50's 28 x 28 x 128
// layers at batch 256 are 784 tiles = 3 rounds of 256 + 16, and that last round cost ~20 % of the
// call (profiles/rd5ah_conv3x3n_tail.jsonl: 85.0 us vs 66.5 at 735 tiles). Its tiles run as 16
// (or, for more than 32 leftover tiles, 32) output channels per workgroup instead: eight (four)
// times the workgroups, an eighth (a quarter) of each wave's MFMAs; 16 vs 32 measured 75.1-77.8
// vs 77.6-77.9 us per call (rd5az). 64-pixel tiles of a 2-wave kernel kept each wave's work and
// saved only 2 us (rd5ai).
int slots128() {  // resident 128-channel workgroups on the current device (cached per device)
  return resident_blocks(reinterpret_cast<const void*>(&conv3x3n_kernel<128, 128, 3>), 64 * waves_of<128>(), 0);
}

void launch128(CNArgs p, int epi, hipStream_t s) {
  static const bool notail = std::getenv("FLUXMPI_CONV3X3N_NOTAIL") != nullptr;
  const int slots = notail ? 0 : slots128();
  const int full = slots > 0 ? p.tiles / slots * slots : 0, rem = p.tiles - full;
  const int ncob = rem * 8 <= slots && C3N_TAIL_CO == 16 ? 8 : (rem * 4 <= slots ? 4 : 1);
  if (full == 0 || rem == 0 || ncob == 1) {
    launch<128, 128>(p, epi, s);
    return;
  }
  CNArgs t = p;
  p.tiles = full;
  launch<128, 128>(p, epi, s);
  t.m_base = full * kTM, t.tiles = rem, t.ncob = ncob;
  if (ncob == 8) launch<128, 16>(t, epi, s);  // 16 output channels per workgroup: an eighth of the MFMAs
  else launch<128, 32>(t, epi, s);
}

}  // namespace

int conv3x3n_slots128() { return slots128(); }

bool conv3x3n_supported(int64_t pixels, int C, int Cout, int H, int W) {
  if (!((C == 64 && Cout == 64) || (C == 128 && Cout == 128))) return false;
  const int maxw = C == 64 ? Geo<64>::kMaxW : Geo<128>::kMaxW;
  return pixels > 0 && pixels % kTM == 0 && W >= 1 && W <= maxw && H >= 1 && pixels % (static_cast<int64_t>(H) * W) == 0 &&
         pixels * C * 2 < (int64_t(1) << 31) && pixels / kTM < (int64_t(1) << 31);
}

void conv3x3n(const void* x, const void* w, void* y, float* stats, int64_t pixels, int H, int W, int C, int Cout,
              int epi, hipStream_t stream) {
  if (!conv3x3n_supported(pixels, C, Cout, H, W))
    throw std::runtime_error("conv3x3n: unsupported shape (C = Cout in {64, 128}, pixels % 256 == 0, W <= 64 / 32; "
                             "pixels=" + std::to_string(pixels) + " C=" + std::to_string(C) + " W=" + std::to_string(W) + ")");
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) & 15u) != 0)
    throw std::runtime_error("conv3x3n: operands must be 16-byte aligned");
  if (epi != 0 && epi != 3) throw std::runtime_error("conv3x3n: epilogue 0 (plain) or 3 (statistics)");
  if (epi == 3 && stats == nullptr) throw std::runtime_error("conv3x3n: the statistics epilogue needs the shards");
  CNArgs p{};
  p.x = static_cast<const bf16*>(x), p.w = static_cast<const bf16*>(w), p.y = static_cast<bf16*>(y);
  p.stats = stats, p.H = H, p.W = W, p.tiles = static_cast<int>(pixels / kTM);
  p.x_bytes = static_cast<uint32_t>(pixels * C * 2);
  p.m_base = 0, p.ncob = 1, p.ldy = Cout;
  if (C == 64) launch<64, 64>(p, epi, stream);
  else launch128(p, epi, stream);
}

}  // namespace fluxmpi
