// 3x3 / stride-1 / pad-1 convolution over NHWC bf16 on MFMA with LDS image halos — gfx950.
//
// gemm_glds.hip's implicit GEMM gathers the im2col rows chunk by chunk through LDS-DMA: every
// input pixel is fetched from L2 nine times (once per tap) and a 128x128 tile stages 1 B of
// operands per 64 FLOP — the DMA rate caps it near 600 TF/s on ResNet-50's 3x3 layers
// (scripts/bench_conv3x3.py). Here a workgroup stages the input rows its 256 output pixels
// touch ONCE per 32-channel chunk (a "halo": virtual rows of W + 2 pixels, image borders and
// the rows between two images of the batch as zero pixels) and reads the nine taps' MFMA
// fragments straight out of it at shifted addresses; with 64 output channels per tile that is
// ~1 B per 127 FLOP.
//
//   tile: 256 consecutive output pixels (flattened n, y, x: a tile may span image rows and
//     images) x 64 output channels; 8 waves = 4 (pixels: 64 each) x 2 (channels: 32 each);
//   K: chunks of 32 input channels x 9 taps; one v_mfma_f32_16x16x32_bf16 k-step per tap;
//   A = filter rows (output channels; LDS [tap][64 rows][4 x 16 B]), B = pixels (LDS halo
//     [virtual row][W + 2][4 x 16 B]): a 16-B entry = 8 channels of one pixel (row), so the
//     LDS-DMA of a pixel's 64 B is four consecutive lanes (coalesced, like the source); the
//     8-channel group of entry (p, g) is stored at slot g ^ 2 ((p >> 2) & 1) — searched
//     exhaustively: conflict-free for every ds_read_b128 lane group and ANY start pixel (the taps
//     shift the start by dy (W + 2) + dx);
//   filter row R of a tile holds output channel 32 (R >> 5) + 8 ((R >> 2) & 3) + 4 ((R >> 4) & 1)
//     + (R & 3): a lane's 8 accumulators of one pixel are 8 consecutive channels (one 16-B store);
//   persistent workgroups (one per CU: two LDS stages of halo + filter chunk) walk their tiles'
//     (tile, chunk) steps with the next step's LDS-DMA in flight under the current MFMAs;
//   epilogue: bf16 store, optional per-channel sum / sum of squares (BatchNorm statistics) into
//     the sharded workspace, accumulated in registers across the workgroup's tiles of one
//     channel block.
// The input gradient is the same convolution of dY with the flipped, transposed filter.
#include <stdexcept>
#include <string>

#include "../api.h"
#include "common.h"

namespace fluxmpi {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void gl_void;

constexpr int kT = 512;
constexpr int kBM = 256;   // output pixels per tile
constexpr int kCOT = 64;   // output channels per tile
constexpr int kCK = 32;    // input channels per K chunk
constexpr int kWSlots = 9 * 4 * kCOT;              // 2304 16-B filter entries per chunk
constexpr int kWInstr = kWSlots / 64;              // 36
constexpr int kWBytes = kWSlots * 16;              // 36864
constexpr int kMaxHaloBytes = 44 * 1024;          // two stages of halo + filter chunk in 160 KiB
constexpr int kShards = 64;  // == batchnorm.hip

__device__ __attribute__((aligned(16))) uint4 g_halo_zero[4];

__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8)); }

__device__ __forceinline__ void dma16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((gl_void*)(src), (lds_char*)(lds_base), 16, 0, 0);
}

struct HaloArgs {
  const bf16* x;    // [N][H][W][C]
  const bf16* w;    // [Co][9][C] (tap-major K)
  bf16* y;          // [N][H][W][Co]
  float* stats;     // [kShards][2][Co] or nullptr
  int N, H, W, C, Co;
  int M;            // N * H * W (the last tile may be partial)
  int nv;           // halo virtual rows per tile (host: max over tiles)
  int halo_bytes;   // nv * (W + 2) * 64 rounded up to 1 KiB
  int halo_instr;   // halo_bytes / 1024
  int tiles_m, tiles;
  int per_block;    // tiles per workgroup
};

// filter row R of a tile -> output channel offset within the tile
__device__ __forceinline__ int row_channel(int R) {
  return 32 * (R >> 5) + 8 * ((R >> 2) & 3) + 4 * ((R >> 4) & 1) + (R & 3);
}

// byte offset of 8-channel group g of entry p (pixel / filter row) in a [entries][4 x 16 B] array
__device__ __forceinline__ int ent_off(int p, int g) { return (p << 6) | ((g ^ ((p >> 1) & 2)) << 4); }

// MODE (bottleneck experiments, FLUXMPI_HALO_MODE): 0 = normal, 1 = no DMA after the first
// step (MFMA + LDS reads only), 2 = no MFMA phase (DMA only)
template <int MODE>
__global__ __launch_bounds__(kT, 2) void conv3x3_halo_kernel(HaloArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int stage_bytes = p.halo_bytes + kWBytes;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;
  const int W2 = p.W + 2, HP = p.H + 2;
  const int chunks = p.C / kCK;
  const int t0 = blockIdx.x * p.per_block;
  const int t1 = t0 + p.per_block < p.tiles ? t0 + p.per_block : p.tiles;
  const int steps = (t1 - t0) * chunks;
  const float inv_w = 1.f / static_cast<float>(p.W), inv_hw = 1.f / static_cast<float>(p.H * p.W);
  const float inv_hp = 1.f / static_cast<float>(HP);
  // halo slot s = instr * 64 + lane: entry e = s >> 2 = v * (W + 2) + px, group (s & 3) ^ swizzle
  const int used_entries = p.nv * W2;
  // filter slot s: tap, 8-channel group, tile row R -> element offset (co * 9 + tap) * C + 8 g
  auto tile_of = [&](int t, int& m0, int& n0) {
    const int nt = t / p.tiles_m;
    n0 = nt * kCOT;
    m0 = (t - nt * p.tiles_m) * kBM;
  };
  // first virtual row of a tile: the row above its first pixel
  auto vr_lo_of = [&](int m0) {
    const int n = static_cast<int>((static_cast<float>(m0) + 0.5f) * inv_hw);
    const int y = static_cast<int>((static_cast<float>(m0 - n * p.H * p.W) + 0.5f) * inv_w);
    return n * HP + y;  // vr(n, y) - 1 with vr(n, y) = n (H + 2) + y + 1
  };
  auto issue = [&](int step, int st) {
    const int t = t0 + step / chunks, ck = step - (step / chunks) * chunks;
    int m0, n0;
    tile_of(t, m0, n0);
    const int vlo = vr_lo_of(m0);
    const int ci0 = ck * kCK;
    char* sh = smem + st * stage_bytes;
    for (int i = wave; i < p.halo_instr; i += kT / 64) {
      const int sl = i * 64 + lane;
      const int e = sl >> 2, gs = (sl & 3) ^ ((e >> 1) & 2);
      const void* src = g_halo_zero;
      if (e < used_entries) {
        const int v = static_cast<int>((static_cast<float>(e) + 0.5f) * (1.f / static_cast<float>(W2)));
        const int px = e - v * W2;
        const int vrow = vlo + v;
        const int n = static_cast<int>((static_cast<float>(vrow) + 0.5f) * inv_hp);
        const int yy = vrow - n * HP - 1;
        if (n < p.N && static_cast<unsigned>(yy) < static_cast<unsigned>(p.H) && px >= 1 && px <= p.W)
          src = p.x + ((static_cast<int64_t>(n) * p.H + yy) * p.W + px - 1) * p.C + ci0 + 8 * gs;
      }
      dma16(src, sh + i * 1024);
    }
    char* sw = sh + p.halo_bytes;
    for (int i = wave; i < kWInstr; i += kT / 64) {
      const int sl = i * 64 + lane;
      const int tap = sl >> 8, R = (sl >> 2) & 63, gq = (sl & 3) ^ ((R >> 1) & 2);
      const int co = n0 + row_channel(R);
      dma16(p.w + (static_cast<int64_t>(co) * 9 + tap) * p.C + ci0 + 8 * gq, sw + i * 1024);
    }
  };

  f32x4 acc[4][2];
  float cs[8], cq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = cq[e] = 0.f;
  int boff[9][4];  // halo byte offset of this lane's B-fragment entry, per tap and fragment
  int aoff[2];     // filter byte offset (tap 0) of this lane's A-fragment rows
#pragma unroll
  for (int j = 0; j < 2; ++j) aoff[j] = ent_off(32 * wn + 16 * j + li, g);
  int stat_n0 = -1;
  auto flush_stats = [&](int n0) {
    // lanes with equal g hold the same 8 channels: reduce over li, then one atomic per channel
    // per wave (the 4 pixel-waves of a channel half add into the same shard)
#pragma unroll
    for (int off = 1; off < 16; off <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], off, 64);
        cq[e] += __shfl_xor(cq[e], off, 64);
      }
    if (li == 0) {
      float* shard = p.stats + static_cast<size_t>((blockIdx.x * 4 + wm) % kShards) * 2 * p.Co;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = n0 + 32 * wn + 8 * g + e;
        atomicAdd(shard + c, cs[e]);
        atomicAdd(shard + p.Co + c, cq[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] = cq[e] = 0.f;
  };

  if (steps > 0) issue(0, 0);
  for (int step = 0; step < steps; ++step) {
    const int st = step & 1;
    const int t = t0 + step / chunks, ck = step - (step / chunks) * chunks;
    int m0, n0;
    tile_of(t, m0, n0);
    wait_vm0();
    __syncthreads();  // stage st landed; every wave is done with the other stage
    if (MODE != 1 && step + 1 < steps) issue(step + 1, st ^ 1);
    if (ck == 0) {
      const int vlo = vr_lo_of(m0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pixr = m0 + 64 * wm + 16 * i + li;
        const int pix = pixr < p.M ? pixr : p.M - 1;  // past the end: any valid address (not stored)
        const int n = static_cast<int>((static_cast<float>(pix) + 0.5f) * inv_hw);
        const int r = pix - n * p.H * p.W;
        const int y = static_cast<int>((static_cast<float>(r) + 0.5f) * inv_w);
        const int x = r - y * p.W;
        const int v = n * HP + y + 1 - vlo;  // >= 1
        const int hb = (v - 1) * W2 + x;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) boff[tap][i] = ent_off(hb + (tap / 3) * W2 + tap % 3, g);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    const char* shp = smem + st * stage_bytes;
    const char* swp = shp + p.halo_bytes;
#pragma unroll
    for (int tap = 0; tap < (MODE == 2 ? 0 : 9); ++tap) {
      bf16x8 a[2], b[4];
#pragma unroll
      for (int j = 0; j < 2; ++j) a[j] = *reinterpret_cast<const bf16x8*>(swp + tap * (kCOT * 64) + aoff[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = *reinterpret_cast<const bf16x8*>(shp + boff[tap][i]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[i], acc[i][j], 0, 0, 0);
    }
    if (ck == chunks - 1) {
      // lane (g, li): channels n0 + 32 wn + 8g .. + 7 of pixel m0 + 64 wm + 16 i + li
      if (p.stats != nullptr && stat_n0 != n0) {
        if (stat_n0 >= 0) flush_stats(stat_n0);
        stat_n0 = n0;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf16 v8[8];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) v8[4 * j + r] = static_cast<bf16>(acc[i][j][r]);
        const int64_t pix = m0 + 64 * wm + 16 * i + li;
        if (pix < p.M) {
          if (p.stats != nullptr) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float f = static_cast<float>(v8[e]);
              cs[e] += f;
              cq[e] = fmaf(f, f, cq[e]);
            }
          }
          uint4 w4;
          __builtin_memcpy(&w4, v8, 16);
          *reinterpret_cast<uint4*>(p.y + pix * p.Co + n0 + 32 * wn + 8 * g) = w4;
        }
      }
    }
  }
  if (p.stats != nullptr && stat_n0 >= 0) flush_stats(stat_n0);
  wait_vm0();
}

// virtual halo rows a tile of kBM pixels starting at m0 needs
int tile_rows(int64_t m0, int64_t M, int H, int W) {
  const int64_t m1 = m0 + kBM - 1 < M ? m0 + kBM - 1 : M - 1;
  const int64_t hw = static_cast<int64_t>(H) * W;
  const int64_t n0 = m0 / hw, n1 = m1 / hw;
  const int64_t y0 = (m0 - n0 * hw) / W, y1 = (m1 - n1 * hw) / W;
  const int64_t v0 = n0 * (H + 2) + y0, v1 = n1 * (H + 2) + y1 + 2;  // vr - 1 .. vr + 1
  return static_cast<int>(v1 - v0 + 1);
}

// the largest halo (virtual rows) over the tiles of an (N, H, W) batch, cached
int halo_rows(int64_t N, int H, int W) {
  static std::mutex mu;
  static std::map<std::tuple<int64_t, int, int>, int> cache;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_tuple(N, H, W);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const int64_t M = N * H * W;
  int nv = 0;
  for (int64_t m0 = 0; m0 < M; m0 += kBM) {
    const int r = tile_rows(m0, M, H, W);
    nv = r > nv ? r : nv;
  }
  cache.emplace(key, nv);
  return nv;
}

int halo_bytes_of(int nv, int W) {
  return static_cast<int>(((static_cast<int64_t>(nv) * (W + 2) * 64 + 1023) / 1024) * 1024);
}

}  // namespace

bool conv3x3_halo_supported(int64_t N, int H, int W, int C, int Co) {
  if (N < 1 || H < 1 || W < 1 || C % kCK != 0 || Co % kCOT != 0) return false;
  if (N * H * W * static_cast<int64_t>(C > Co ? C : Co) >= (int64_t(1) << 31)) return false;
  if (N * H * W >= (int64_t(1) << 24)) return false;  // float index math in the kernel
  return halo_bytes_of(halo_rows(N, H, W), W) <= kMaxHaloBytes;
}

void conv3x3_halo(const void* x, const void* w, void* y, float* stats, int64_t N, int H, int W, int C, int Co,
                  hipStream_t s) {
  if (!conv3x3_halo_supported(N, H, W, C, Co)) throw std::runtime_error("conv3x3_halo: unsupported shape");
  for (const void* q : {x, w, static_cast<const void*>(y)})
    if (q == nullptr || reinterpret_cast<uintptr_t>(q) % 16 != 0)
      throw std::runtime_error("conv3x3_halo: x, w, y must be 16-byte aligned");
  const int64_t M = N * H * W;
  const int nv = halo_rows(N, H, W);
  HaloArgs a{};
  a.x = static_cast<const bf16*>(x);
  a.w = static_cast<const bf16*>(w);
  a.y = static_cast<bf16*>(y);
  a.stats = stats;
  a.N = static_cast<int>(N);
  a.H = H;
  a.W = W;
  a.C = C;
  a.Co = Co;
  a.nv = nv;
  a.halo_bytes = halo_bytes_of(nv, W);
  a.halo_instr = a.halo_bytes / 1024;
  a.M = static_cast<int>(M);
  a.tiles_m = static_cast<int>((M + kBM - 1) / kBM);
  a.tiles = a.tiles_m * (Co / kCOT);
  const int smem = 2 * (a.halo_bytes + kWBytes);
  static int attr_bytes = 0;
  if (attr_bytes < 2 * (kMaxHaloBytes + kWBytes)) {
    for (const void* k : {reinterpret_cast<const void*>(&conv3x3_halo_kernel<0>),
                          reinterpret_cast<const void*>(&conv3x3_halo_kernel<1>),
                          reinterpret_cast<const void*>(&conv3x3_halo_kernel<2>)})
      FLUXMPI_HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (kMaxHaloBytes + kWBytes)));
    attr_bytes = 2 * (kMaxHaloBytes + kWBytes);
  }
  int cus = 0, dev = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  const int blocks = a.tiles < cus ? a.tiles : cus;
  a.per_block = (a.tiles + blocks - 1) / blocks;
  static const int mode = [] {
    const char* e = std::getenv("FLUXMPI_HALO_MODE");
    return e != nullptr ? std::atoi(e) : 0;
  }();
  const unsigned grid = static_cast<unsigned>((a.tiles + a.per_block - 1) / a.per_block);
  if (mode == 1) conv3x3_halo_kernel<1><<<grid, kT, smem, s>>>(a);
  else if (mode == 2) conv3x3_halo_kernel<2><<<grid, kT, smem, s>>>(a);
  else conv3x3_halo_kernel<0><<<grid, kT, smem, s>>>(a);
  FLUXMPI_HIP_CHECK(hipGetLastError());
}

}  // namespace fluxmpi
