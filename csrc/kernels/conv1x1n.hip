// Narrow-K 1x1 convolution forward (+ the next BatchNorm's statistics), NHWC bf16 — gfx950.
//
// y[M][N] = x[M][K] W[N][K]^T for K = 64 / 128 input channels and N a multiple of 256 output
// channels: ResNet-50's stage-1 / stage-2 expansions (conv3 64 -> 256, 128 -> 512, the stage-1
// downsample 64 -> 256). These are write-bound (the output is 4x the input) and too shallow
// for the k-loop of the tiled GEMMs to hide their epilogues: the 128-tile LDS-DMA kernel ran them
// at 4.1 TB/s (64 -> 256: 126 us) and 2.9 TB/s (128 -> 512: 88 us), MIOpen at 5.0 / 4.2 TB/s
// without the statistics (profiles/rd5g_roofline_resnet50.md).
//
// Persistent: one workgroup per CU owns one 256-column slice of the output (its filter slice,
// 256 x K, is DMA'd into LDS once) and walks 128-row tiles of x, the next tile's loads in flight
// (into registers) during this tile's MFMAs and stores. 8 waves: 4 row groups of 32 rows x 2 column halves of 128;
// per 32-channel k-step a wave reads 2 activation and 8 filter fragments (ds_read_b128, 128-B
// rows with chunk slot q ^ (row & 7): conflict-free) for 16 v_mfma_f32_16x16x32_bf16. The
// statistics accumulate in registers over ALL of the workgroup's tiles and meet in LDS once at
// the end: one atomic per column and moment per workgroup (instead of per tile).
// Reference: /root/reference has no kernels — this is compute under the per-step gradient work of
// the ResNet-50 DDP configuration (BASELINE.json, src/optimizer.jl:20-23).
#include <cstdint>
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;

constexpr int kBM = 128;     // rows per tile
constexpr int kBN = 256;     // columns per workgroup slice
constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kShards = 64;  // BatchNorm statistics shards (== batchnorm.hip)

struct C1Args {
  const bf16* x;   // [M][K]
  const bf16* w;   // [N][K]
  bf16* y;         // [M][N]
  float* stats;    // EPI 3: [kShards][2][N]
  int N;
  int tiles;       // M / kBM
  int slices;      // N / kBN
  uint32_t x_bytes;
};

// LDS reads through an address-space-3 pointer with alias scopes (__restrict__): otherwise the
// waitcnt pass puts a vmcnt(0) for the in-flight tile DMA — and the stores queued behind it — in
// front of them
typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
__device__ __forceinline__ bf16x8 frag(const char* __restrict__ p) { return *(lds_bf16x8*)(p); }

template <int K, int EPI>
__global__ __launch_bounds__(kThreads, 1) void conv1x1n_kernel(C1Args p) {
  constexpr int NPL = K / 64;                // 128-B planes per row
  constexpr int KS = K / 32;                 // 32-channel k-steps
  constexpr int kWPlane = kBN * 128;         // filter plane bytes
  constexpr int kAPlane = kBM * 128;         // activation plane bytes (one buffer)
  constexpr int kABuf = NPL * kAPlane;
  __shared__ __attribute__((aligned(1024))) char wl[NPL * kWPlane];
  // two separate tile buffers (not halves of one array): the LDS reads of one and the DMA into the
  // other are then provably disjoint, so the waitcnt pass does not drain the DMA (and the stores
  // queued behind it) before the reads
  __shared__ __attribute__((aligned(1024))) char al0[kABuf];
  __shared__ __attribute__((aligned(1024))) char al1[kABuf];

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int lrow = lane >> 3, lslot = lane & 7;
  const int fr = lane & 15, fg = lane >> 4;
  const int wr = wave & 3, wc = wave >> 2;  // row group (32 rows), column half (128 columns)

  // this workgroup's slice and its tiles: t = first, first + step, ...
  const int slice = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) % p.slices);
  const int first = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) / p.slices);
  const int step = __builtin_amdgcn_readfirstlane(static_cast<int>(gridDim.x) / p.slices);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.x), 0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.w), 0, 0x7fffffff, 0x00020000);

  // the filter slice: kBN rows x NPL planes, 8 rows (1 KB) per DMA instruction
  for (int i = wave; i < NPL * (kBN / 8); i += kWaves) {
    const int pl = i / (kBN / 8), rg = i - pl * (kBN / 8);
    const int co = rg * 8 + lrow;
    const uint32_t off = static_cast<uint32_t>((slice * kBN + co) * (K * 2) + pl * 128 + ((lslot ^ (co & 7)) << 4));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_char*)(wl + pl * kWPlane + rg * 1024), 16, off, 0, 0, 0);
  }
  // x tiles: prefetched into registers one tile ahead (global_load_dwordx4, 16 B per lane), then
  // written to LDS after this tile's stores; the compiler's own vmcnt accounting then covers the
  // stores queued between (an LDS-DMA ring made it drain them before every tile's reads)
  constexpr int kAL = NPL * (kBM / 8) / kWaves;  // 16-B loads per lane per tile
  uint4 pre[kAL];
  auto load_a = [&](int t) {
#pragma unroll
    for (int j = 0; j < kAL; ++j) {
      const int i = j * kWaves + wave;
      const int pl = i / (kBM / 8), rg = i - pl * (kBM / 8);
      const int row = rg * 8 + lrow;
      const uint32_t off = static_cast<uint32_t>((t * kBM + row) * (K * 2) + pl * 128 + (lslot << 4));
      pre[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto store_a = [&](char* dst) {
#pragma unroll
    for (int j = 0; j < kAL; ++j) {
      const int i = j * kWaves + wave;
      const int pl = i / (kBM / 8), rg = i - pl * (kBM / 8);
      const int row = rg * 8 + lrow;
      *reinterpret_cast<uint4*>(dst + pl * kAPlane + row * 128 + ((lslot ^ (row & 7)) << 4)) = pre[j];
    }
  };
  if (first < p.tiles) {
    load_a(first);
    store_a(al0);
  }

  float cs[8][4], cq[8][4];  // EPI 3: the lane's column partial sums over every tile it stores
#pragma unroll
  for (int nb = 0; nb < 8; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[nb][r] = cq[nb][r] = 0.f;

  // one tile: wait for `cur`, prefetch the next tile into registers, MFMAs, stores, then `nxt`
  auto do_tile = [&](int t, const char* __restrict__ cur, char* __restrict__ nxt) {
    // tile t is in `cur` (every wave's ds_writes, and the filter DMA on the first tile, done);
    // `nxt` was last read during the previous tile
    if (t == first) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bool more = t + step < p.tiles;
    if (more) load_a(t + step);
    __builtin_amdgcn_sched_barrier(0);  // keep the loads at the top: their latency hides under this tile
    f32x4 acc[2][8];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int pl = ks / 2, ch = (ks & 1) * 4 + fg;  // plane, 16-B chunk within its 128-B row
      bf16x8 fb[8], fa[2];
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        const int co = wc * 128 + nb * 16 + fr;
        fb[nb] = frag(wl + pl * kWPlane + co * 128 + ((ch ^ (co & 7)) << 4));
      }
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        const int row = wr * 32 + mb * 16 + fr;
        fa[mb] = frag(cur + pl * kAPlane + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nb], fa[mb], acc[mb][nb], 0, 0, 0);
    }
    // acc[mb][nb][r] = y[t kBM + 32 wr + 16 mb + (lane & 15)][slice kBN + 128 wc + 16 nb + 4 (lane >> 4) + r]
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      bf16* yrow = p.y + static_cast<int64_t>(t * kBM + wr * 32 + mb * 16 + fr) * p.N + slice * kBN + wc * 128 + 4 * fg;
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
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
    if (more) store_a(nxt);
  };
  // the tile loop unrolled by two: each half's buffers are compile-time known (see al0 / al1)
  for (int t = first; t < p.tiles; t += 2 * step) {
    do_tile(t, al0, al1);
    if (t + step < p.tiles) do_tile(t + step, al1, al0);
  }
  if constexpr (EPI == 3) {
    // per column: the wave's 16 row lanes, then the 4 row-group waves through LDS (the tile
    // buffers are free once every wave is past its last tile), one atomic per column and moment
    // per workgroup into the shard blockIdx % kShards
    __syncthreads();
    float* red = reinterpret_cast<float*>(al0);  // [4 row groups][2][kBN]
#pragma unroll
    for (int nb = 0; nb < 8; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = row_sum16(cs[nb][r]), q = row_sum16(cq[nb][r]);
        if (fr == 0) {
          const int col = wc * 128 + nb * 16 + 4 * fg + r;
          red[(wr * 2 + 0) * kBN + col] = s;
          red[(wr * 2 + 1) * kBN + col] = q;
        }
      }
    __syncthreads();
    {
      const int mom = threadIdx.x / kBN, col = threadIdx.x - mom * kBN;  // 512 threads = 2 x 256
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) t += red[(g * 2 + mom) * kBN + col];
      atomicAdd(p.stats + (static_cast<int64_t>(blockIdx.x % kShards) * 2 + mom) * p.N + slice * kBN + col, t);
    }
  }
}

template <int K>
void launch(const C1Args& p, int epi, int grid, hipStream_t s) {
  if (epi == 3) conv1x1n_kernel<K, 3><<<grid, kThreads, 0, s>>>(p);
  else conv1x1n_kernel<K, 0><<<grid, kThreads, 0, s>>>(p);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    FLUXMPI_HIP_CHECK(hipGetDevice(&dev));
    FLUXMPI_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return cus;
}

}  // namespace

bool conv1x1n_supported(int64_t M, int64_t K, int64_t N) {
  return (K == 64 || K == 128) && N >= kBN && N % kBN == 0 && N <= 4096 && M > 0 && M % kBM == 0 &&
         M * K * 2 < (int64_t(1) << 31) && M / kBM < (int64_t(1) << 30);
}

void conv1x1n(const void* x, const void* w, void* y, float* stats, int64_t M, int64_t K, int64_t N, int epi,
              hipStream_t stream) {
  if (!conv1x1n_supported(M, K, N))
    throw std::runtime_error("conv1x1n: unsupported shape (K in {64, 128}, N % 256 == 0, M % 128 == 0; M=" +
                             std::to_string(M) + " K=" + std::to_string(K) + " N=" + std::to_string(N) + ")");
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) & 15u) != 0)
    throw std::runtime_error("conv1x1n: operands must be 16-byte aligned");
  if (epi != 0 && epi != 3) throw std::runtime_error("conv1x1n: epilogue 0 (plain) or 3 (statistics)");
  if (epi == 3 && stats == nullptr) throw std::runtime_error("conv1x1n: the statistics epilogue needs the shards");
  C1Args p{};
  p.x = static_cast<const bf16*>(x), p.w = static_cast<const bf16*>(w), p.y = static_cast<bf16*>(y);
  p.stats = stats, p.N = static_cast<int>(N), p.tiles = static_cast<int>(M / kBM), p.slices = static_cast<int>(N / kBN);
  p.x_bytes = static_cast<uint32_t>(M * K * 2);
  // one workgroup per CU (LDS: the filter slice + two tiles), a whole number of them per slice
  int per = device_cus() / p.slices;
  if (per < 1) per = 1;
  if (per > p.tiles) per = p.tiles;
  const int grid = per * p.slices;
  if (K == 64) launch<64>(p, epi, grid, stream);
  else launch<128>(p, epi, grid, stream);
}

}  // namespace fluxmpi
