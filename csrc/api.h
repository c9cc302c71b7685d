// Host-side launch API of the fluxmpi_amd native library (no ATen dependency:
// raw device pointers + a hipStream_t, so callers can launch on any PyTorch
// stream, inside or outside HIP-graph capture).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

namespace fluxmpi {

// ---- multi-tensor copy / cast / scale (pack, unpack, scale) -----------------
// dst[i][k] = (Tout)(src[i][k] * scale) for k < numel[i]. src[i] may equal dst[i]
// (in-place scale / cast is not allowed when the element sizes differ).
void mt_copy(const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst,
             const std::vector<int64_t>& numel, int in_dtype, int out_dtype, float scale,
             hipStream_t stream);

// Fill every tensor with `value` (zeroing flat grad buckets).
void mt_fill(const std::vector<uintptr_t>& dst, const std::vector<int64_t>& numel, int dtype,
             float value, hipStream_t stream);

// Sum of squares of all tensors into out[0] (fp32, atomically accumulated; out must be
// zeroed by the caller). Used by ClipNorm and by debug checksums.
void mt_sumsq(const std::vector<uintptr_t>& src, const std::vector<int64_t>& numel, int dtype,
              float* out, hipStream_t stream);

// ---- fused optimisers ---------------------------------------------------------
struct AdamHyper {
  float lr, beta1, beta2, eps;
  float bc1, bc2;     // 1 - beta1^t, 1 - beta2^t (host mode)
  float weight_decay;  // Optimisers.jl WeightDecay after Adam (AdamW = chain)
  float grad_scale;    // multiplies the incoming gradient (e.g. 1/world for mean)
  const float* dev;    // optional device hyper block {lr, beta1^t, beta2^t} (graph mode)
  const float* dev_gscale;  // optional device gradient scale (e.g. 1/loss_scale)
};

// master: optional fp32 master weights (mixed precision); when given, param is
// the low-precision copy that is re-written from the master after the update.
void mt_adam(const std::vector<uintptr_t>& param, const std::vector<uintptr_t>& grad,
             const std::vector<uintptr_t>& m, const std::vector<uintptr_t>& v,
             const std::vector<uintptr_t>& master, const std::vector<int64_t>& numel,
             int p_dtype, int g_dtype, int s_dtype, const AdamHyper& h, hipStream_t stream);

// dev[1] *= beta1, dev[2] *= beta2 (advance the bias-correction powers on device).
void adam_advance(float* dev, float beta1, float beta2, hipStream_t stream);

struct SgdHyper {
  float lr, momentum, weight_decay, grad_scale;
  int nesterov;  // 0: heavy ball (Optimisers.Momentum), 1: Optimisers.Nesterov
  const float* dev_lr;
};
// buf: momentum buffers (ignored when momentum == 0 -> Optimisers.Descent).
void mt_sgd(const std::vector<uintptr_t>& param, const std::vector<uintptr_t>& grad,
            const std::vector<uintptr_t>& buf, const std::vector<uintptr_t>& master,
            const std::vector<int64_t>& numel, int p_dtype, int g_dtype, int s_dtype,
            const SgdHyper& h, hipStream_t stream);

// ---- BatchNorm (NHWC, channels innermost) + ReLU / residual-add fusions ----------
// Training forward: per-channel batch statistics over rows = N*H*W, then
//   y = act(x * scale_c + shift_c [+ residual]).
// Writes mean/invstd (fp32 [C]) for the backward and updates running stats.
void bn_fwd_train(const void* x, void* y, const void* residual, const float* weight,
                  const float* bias, float* running_mean, float* running_var, float* save_mean,
                  float* save_invstd, float* workspace, int64_t rows, int64_t C, float momentum,
                  float eps, int relu, uint8_t* relu_mask, int dtype, hipStream_t stream, int64_t* num_batches_tracked = nullptr);
// Backward: given dy (and y when relu, to mask), computes dx, dweight, dbias and
// (when residual was fused) d_residual = masked dy.
// y == nullptr with relu: the ReLU mask is recomputed from x (bit-identical to forward).
// relu_mask (optional): the 1-bit-per-element mask written by bn_fwd_train.
void bn_bwd(const void* dy, const void* x, const void* y, const uint8_t* relu_mask, const float* weight,
            const float* bias,
            const float* save_mean, const float* save_invstd, void* dx, void* dres,
            float* dweight, float* dbias, float* workspace, int64_t rows, int64_t C, int relu,
            int dtype, hipStream_t stream, int stats_ready = 0);
size_t bn_workspace_floats(int64_t rows, int64_t C);
// Split forward for producer/consumer fusion with the GEMM:
// bn_stats_finalize: [stats pass over x unless stats_ready (a GEMM epilogue already
// accumulated them into ws)] + finalize (mean/invstd, running stats, and optionally the
// per-channel scale/shift a consumer GEMM applies on load). bn_apply: the normalise pass.
void bn_stats_finalize(const void* x, const float* w, const float* b, float* running_mean,
                       float* running_var, float* save_mean, float* save_invstd, float* scale,
                       float* shift, float* workspace, int64_t rows, int64_t C, float momentum,
                       float eps, int stats_ready, int dtype, hipStream_t stream, int64_t* num_batches_tracked = nullptr);
void bn_apply(const void* x, void* y, const void* residual, const float* w, const float* b,
              const float* save_mean, const float* save_invstd, int64_t rows, int64_t C, int relu,
              uint8_t* relu_mask, int dtype, hipStream_t stream);
// Dual BatchNorm of a downsample block: y = relu(BN(x) + BN2(x2)) (+ 1-bit ReLU mask), and its
// backward: dx, dx2 and both BatchNorms' dweight/dbias from one reduce + one dx pass over
// (dy, mask, x, x2). ws/ws2: two zeroed statistics workspaces. C/8 must divide 256.
void bn_apply_dual(const void* x, const void* x2, void* y, const float* w, const float* b, const float* save_mean,
                   const float* save_invstd, const float* w2, const float* b2, const float* save_mean2,
                   const float* save_invstd2, int64_t rows, int64_t C, uint8_t* relu_mask, int dtype,
                   hipStream_t stream);
void bn_bwd_dual(const void* dy, const uint8_t* relu_mask, const void* x, const void* x2, const float* w,
                 const float* save_mean, const float* save_invstd, const float* w2, const float* save_mean2,
                 const float* save_invstd2, void* dx, void* dx2, float* dweight, float* dbias, float* dweight2,
                 float* dbias2, float* ws, float* ws2, int64_t rows, int64_t C, int dtype, hipStream_t stream);
// Inference: y = act(x * scale + shift [+ residual]) from running statistics.
void bn_fwd_infer(const void* x, void* y, const void* residual, const float* weight,
                  const float* bias, const float* running_mean, const float* running_var,
                  int64_t rows, int64_t C, float eps, int relu, int dtype, hipStream_t stream);

// ---- fused stem: BN affine + ReLU + max-pool (NHWC) ---------------------------------
// y = relu(max over KxK/S window (pad P) of x*scale+shift), idx = window index (0xFF: max <= 0)
void bn_relu_maxpool_fwd(const void* x, const float* scale, const float* shift, void* y, uint8_t* idx, int64_t N,
                         int64_t H, int64_t W, int64_t C, int K, int S, int P, int dtype, hipStream_t stream);
// y[p][0..3] = (x[p][0], x[p][1], x[p][2], 0) for npix 16-bit NHWC pixels (stem channel pad)
void pad_c3_to_c4(const void* x, void* y, int64_t npix, int dtype, hipStream_t stream);

// ---- ResNet stem on MFMA (stem.hip): 7x7/2 conv of NHWC4 224x224 images + BN statistics;
// the fused backward (pool gather + BN backward + filter gradient)
void stem_fwd(const void* x, const void* wp, void* y, float* stats, int64_t n, hipStream_t stream);
int stem_bwd_blocks(int64_t n);
int64_t stem_part_floats();
void stem_bwd(const void* x, const void* c, const void* dp, const uint8_t* idx, const float* w, const float* mean,
              const float* inv, float* part, int blocks, float* stats, float* dw_bn, float* db_bn, float* dwp,
              int64_t n, hipStream_t stream);
// Softmax attention, head dim 64, bf16 (csrc/kernels/attention.hip). q/k/v and dq/dk/dv share
// strides (sq_b, sq_t; head stride 64), o has (so_b, so_t, so_h), dout (sg_b, sg_t; head stride
// 64); stats is fp32 [B][H][T][2]: attn_fwd writes [..][0] = base-2 log-sum-exp of the scaled
// scores, attn_bwd reads it and writes [..][1] = rowsum(dO*O).
void attn_fwd(const void* q, const void* k, const void* v, void* o, float* stats, int64_t sq_b, int64_t sq_t,
              int64_t so_b, int64_t so_t, int64_t so_h, int B, int T, int H, int Dh, float scale, hipStream_t stream);
void attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, void* dq, void* dk,
              void* dv, float* stats, int64_t sq_b, int64_t sq_t, int64_t so_b, int64_t so_t, int64_t so_h,
              int64_t sg_b, int64_t sg_t, int B, int T, int H, int Dh, float scale, hipStream_t stream,
              float* colpart = nullptr);
// rows of attn_bwd's optional column-sum partials ([rows][3*H*64] fp32: per-wave sums of the dQ /
// dK / dV rows it writes; their reduce is the packed QKV bias gradient), 0 if this call's variant
// does not write them
int attn_bwd_colpart_rows(int B, int T, int H, int64_t sq_t, int64_t sg_t);
// dx[n,h,w,c] = sum of dy over the windows whose idx points at (h,w) (gather; dx fully written)
void maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int64_t N, int64_t H, int64_t W, int64_t C, int K,
                 int S, int P, int dtype, hipStream_t stream);

// ---- fused LayerNorm (+ residual add), rows of D (D % 8 == 0, D <= 8192) ----------------
// forward: [h = x + residual] (h written when residual != nullptr); y = LN(h) * w + b;
// mean / rstd per row (fp32) saved. w/b: fp32 or the activation dtype (wdtype), 16-byte aligned.
void layernorm_fwd(const void* x, const void* residual, void* h, void* y, const void* w, const void* b, float* mean,
                   float* rstd, int64_t rows, int64_t D, float eps, int dtype, int wdtype, hipStream_t stream);
// backward: dx = LN backward of dy [+ dh_ext]; per-workgroup [2][D] fp32 partials of (dw, db)
// stored into `partials` (capacity max_blocks x 2D); returns the number of partial rows written
// (sum them with gemm_splitk_reduce). colsum (dh_ext required): [3][D] rows, the third the
// column sums of dx.
int layernorm_bwd(const void* dy, const void* x, const void* dh_ext, const float* mean, const float* rstd,
                  const void* w, void* dx, float* partials, int max_blocks, int64_t rows, int64_t D, int dtype,
                  int wdtype, bool colsum, hipStream_t stream);

// ---- MFMA bf16 GEMM with BatchNorm fusions (1x1 convolutions) --------------------
// C[M,N] = A[M,K] * B[N,K]^T. a_kmajor: A stored [M][lda] (K contiguous), else [K][lda]
// (M contiguous); b_kmajor likewise for B. mode 0: C bf16; mode 1: C bf16 + per-column
// sum/sumsq into stats[64][2][N] (sharded, caller-zeroed); mode 2: C fp32 += (atomics,
// allows split-K over `splits`); mode 3: split s stores its fp32 partial to C + s*M*ldc. a_scale/a_shift: relu(A*s+t) per k applied on load
// (K-major A); b_scale/b_shift: per n on load (N-major B).
struct GemmProblem {
  const void* a;
  const void* b;
  void* c;
  int64_t lda, ldb, ldc, M, N, K;
  bool a_kmajor, b_kmajor;
  int mode, splits;
  const float* a_scale;
  const float* a_shift;
  const float* b_scale;
  const float* b_shift;
  float* stats;
  int tile_m, tile_n;  // 0 = auto, 64 forces the 64 tile
  int nbuf;            // LDS buffers: 0 = auto (2), 1, 2
  const void* res;     // optional bf16 residual [M][ldr] added in the epilogue (modes 0/1)
  int64_t ldr;
  // mode 1 + bnb_x: stats = BatchNorm-backward reductions (sum dy_eff, sum dy_eff*xhat) of a BN
  // whose input is bnb_x ([M][N] dense) and whose output gradient is C (see gemm.hip)
  const void* bnb_x;
  const float* bnb_w;
  const float* bnb_b;
  const float* bnb_mean;
  const float* bnb_inv;
  const uint8_t* bnb_mask;
  int bnb_rm;
  // conv_h > 0: A is implicit — the 3x3 / stride 1 / pad 1 im2col of an NHWC image batch
  // [M/(H*W)][H][W][conv_c] (K = 9*conv_c, K-major B = [N][3][3][conv_c] filter)
  int conv_h = 0, conv_w = 0, conv_c = 0;
  int engine = 0;  // 0 auto, 1 register-staged kernel (gemm.hip), 2 LDS-DMA pipelined kernel (gemm_glds.hip)
  // LDS-DMA kernel: residual element (m, n) counts only if bit n%8 of res_mask[(m*N + n)/8] is set
  // (the 1-bit ReLU mask of the BatchNorm whose output gradient the residual is)
  const uint8_t* res_mask = nullptr;
  // LDS-DMA kernel: res_sub_h > 0 — the residual is the compact stride-2 subsample of an
  // [M/(H*W)][H][W] row grid (H = res_sub_h, W = res_sub_w): output row (n, h, w) adds residual row
  // (n, h/2, w/2) when h and w are even and nothing otherwise (a stride-2 1x1 convolution's input
  // gradient, without the zero-filled full-resolution tensor). No res_mask with it.
  int res_sub_h = 0, res_sub_w = 0;
  // LDS-DMA kernel: a_sub_h > 0 — A row (n, ho, wo) of an [M/(Ho*Wo)][Ho][Wo] output grid is row
  // (n, 2*ho, 2*wo) of the NHWC image [M/(Ho*Wo)][a_sub_h][a_sub_w][lda] (Ho = ceil(H/2)): a
  // stride-2 1x1 convolution without the strided copy of its input. Plain K-major A only.
  int a_sub_h = 0, a_sub_w = 0;
  // LDS-DMA kernel, implicit conv: conv_s == 2 — a 3x3 / stride 2 / pad 1 convolution over the
  // NHWC image [M/(Ho*Wo)][conv_h][conv_w][conv_c] (conv_h / conv_w the INPUT size, Ho = ceil(H/2));
  // conv_s == 16 + (2 py + px) — parity class (py, px) of that convolution's INPUT gradient: A = dY
  // [M/(Ho*Wo)][conv_h = Ho][conv_w = Wo][conv_c = Cout], B = the flipped transposed filter
  // [N = Cin][3][3][Cout] (ldb >= 9 Cout), K = taps * Cout (1, 2, 2, 4 taps), C row (img, a, b) =
  // dX pixel (img, 2a + py, 2b + px) of [.][2 Ho][2 Wo] (even input sizes)
  int conv_s = 1;
};
void gemm_bf16(const GemmProblem& g, hipStream_t stream);
// the LDS-DMA pipelined kernel: K-major A (or implicit conv) and B, modes 0/1, optional residual,
// no prologue affine / split-K / BN-backward epilogue
bool gemm_glds_supported(const GemmProblem& g);
void gemm_glds(const GemmProblem& g, hipStream_t stream);
// weight gradient, fp32 split-K partials ws[s][M][N] = sum over split s of A[k][m] * B[k][n]
// (A: [K][lda], B: [K][ldb] or, conv_h > 0, the implicit 3x3/s1/p1 im2col of an NHWC image
// [K/(H*W)][H][W][conv_c] with N = 9*conv_c; b_sub: row k of B = pixel (n, 2ho, 2wo) of the NHWC image
// [.][conv_h][conv_w][ldb] for output pixel k = (n, ho, wo) of a stride-2 1x1 convolution, or with
// conv_c > 0 the implicit im2col of a 3x3 / stride 2 / pad 1 convolution over that grid);
// returns nothing, reduce with gemm_splitk_reduce
void gemm_wgrad(const void* a, const void* b, float* ws, int64_t lda, int64_t ldb, int64_t M, int64_t N, int64_t K,
                int splits, int conv_h, int conv_w, int conv_c, hipStream_t stream, int variant = 0, int b_sub = 0);
// out_i[ci][t][co] = in_i[co][taps-1-t][ci] (bf16) for every filter i, one launch per 40 filters:
// the K-major B operand of the input-gradient GEMMs (1x1: W^T; 3x3: transposed + flipped)
void transpose_filters(const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst,
                       const std::vector<int>& co, const std::vector<int>& ci, const std::vector<int>& taps,
                       hipStream_t stream);
// out[e] = sum over s < splits of ws[s*n + e] (mode-3 split-K partials; ws is clobbered); out fp32 or bf16
void gemm_splitk_reduce(const float* ws, int splits, int64_t n, void* out, int out_dtype, hipStream_t stream);
// the same with the reduced row split into <= 3 segments of `seg` columns, each to its own output
// (e.g. a LayerNorm's dw / db straight into two DDP bucket slices)
void gemm_splitk_reduce_seg(const float* ws, int splits, int64_t n, int64_t seg, void* out0, void* out1, void* out2,
                            int out_dtype, hipStream_t stream);
// Weight gradient on 256 x 256 tiles (wgrad256.hip): ws[split][M][N] = sum over the split's k of
// A[k][m] * B[k][n] (bf16 A [K][lda], B [K][ldb], M and N multiples of 256), fp32 partials.
bool wgrad256_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
int wgrad256_actual_splits(int64_t K, int splits);
void wgrad256_set_variant(int v);  // main-loop variant (A/B runs; 3 hoisted addressing, 4 ping-pong)
void gemm_wgrad256(const void* a, const void* b, float* ws, int64_t lda, int64_t ldb, int64_t M, int64_t N, int64_t K,
                   int splits, hipStream_t stream);
// Token-major Linear GEMM, both operands k-contiguous (gemm_nt.hip): C[M][N] = A[M][K] B[N][K]^T,
// 256 x 256 tiles, ping-pong 8-wave schedule; epi 0 (+ bias), 1 (+ bias: C = gelu'(h), C2 = gelu(h)),
// 2 (C = bf16(acc) * D, D = gelu'(h) as epi 1 stored it; colpart[2 * M / 256][N] = per-half-tile column sums of C),
// 3 (C, and its per-column sum / sum of squares added into the BatchNorm shards stats[64][2][N]).
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc);
bool gemm_nt_conv_supported(int64_t pixels, int64_t C, int64_t Cout);
int gemm_nt_colpart_rows(int64_t M);
// split-K tail: the fewest k-tiles of a workgroup's share of the last round (0: off, the default;
// FLUXMPI_GEMM_NT_SPLIT overrides it). Test/diagnostic knob, not public API.
void gemm_nt_set_split(int min_ktiles);
int gemm_nt_get_split();
void gemm_nt(const void* a, const void* b, void* c, void* c2, const void* bias, int bias_f32, const void* h,
             float* colpart, float* stats, int64_t lda, int64_t ldb, int64_t ldc, int64_t M, int64_t N, int64_t K,
             int epi, hipStream_t stream);
// 3x3 / stride 1 / pad 1 convolution on the same kernel: A = the implicit im2col of the NHWC image
// x [nimg][H][W][C] (C % 64 == 0), B = w [Cout][3][3][C]; y [nimg*H*W][Cout]; epi 0, 3 (statistics)
// or 4 (y = bf16(bf16(conv) + residual), residual laid out as y)
void gemm_nt_conv(const void* x, const void* w, void* y, float* stats, int64_t nimg, int H, int W, int C,
                  int64_t Cout, int epi, hipStream_t stream, const void* residual = nullptr);
// A token-major Linear's input and weight gradients in one launch (linbwd.hip): dx [M][K] =
// dy [M][N] W [N][K] (bf16, nullptr: skip) and the weight gradient's fp32 split-K partials
// ws [s][N][K] of dy^T x (nullptr: skip; s = linear_bwd_splits(M, N, K, splits), sum them with
// gemm_splitk_reduce). M, N, K multiples of 256.
bool linear_bwd_supported(int64_t M, int64_t N, int64_t K, int64_t ldy, int64_t ldx, int64_t ldw, int64_t lddx);
int linear_bwd_splits(int64_t M, int64_t N, int64_t K, int splits);
void linear_bwd(const void* dy, const void* x, const void* w, void* dx, float* ws, int64_t M, int64_t N, int64_t K,
                int64_t ldy, int64_t ldx, int64_t ldw, int64_t lddx, int splits, int dg_first, hipStream_t stream);
// 3x3 / pad 1 / stride 1-2 convolution over a 3-channel NHWC bf16 image (conv_c3.hip), Cout % 128 == 0:
// forward y [pixels][Cout] from w_pairs [Cout][14] (the channels_last filter's 27 taps x channels as
// packed bf16 pairs, the 28th element 0); filter gradient as fp32 partials [blocks][Cout][27]
// (reduce with gemm_splitk_reduce into the [Cout][3][3][3] channels_last filter order)
bool conv_c3_supported(int64_t N, int H, int W, int stride, int Cout);
int64_t conv_c3_wgrad_blocks(int64_t N, int H, int W, int stride);
void conv_c3_fwd(const void* x, const void* w_pairs, void* y, int64_t N, int H, int W, int stride, int Cout,
                 hipStream_t stream);
void conv_c3_wgrad(const void* x, const void* dy, float* part, int64_t N, int H, int W, int stride, int Cout,
                   hipStream_t stream);
// Narrow-channel 3x3 / stride 1 / pad 1 convolution (conv3x3n.hip): C = Cout in {64, 128}, the
// input halo staged once per 256-pixel workgroup; x [pixels][C] NHWC, w [Cout][9][C], y [pixels][Cout];
// epi 0 or 3 (BatchNorm statistics into stats[64][2][Cout])
// resident workgroups of the 128-channel kernel on the current device (its tail split's round size)
int conv3x3n_slots128();
bool conv3x3n_supported(int64_t pixels, int C, int Cout, int H, int W);
void conv3x3n(const void* x, const void* w, void* y, float* stats, int64_t pixels, int H, int W, int C, int Cout,
              int epi, hipStream_t stream);
// Weight gradient of the narrow-channel 3x3 / stride 1 / pad 1 convolution (wgrad3x3n.hip): dy
// [N][H][W][Cout], x [N][H][W][C] (C in {64, 128}); ws[split][Cout][9 C] fp32 partials (reduce with
// gemm_splitk_reduce; the actual split count is wgrad3x3n_splits). variant bit 0: 8 waves (else 4),
// bit 1: two register sets of prefetched rows (4 waves), bit 2 (C = 128): 128 Cout per workgroup.
// A workgroup owns 64 / 128 Cout x all nine taps (C = 64) or x one filter row of three taps (C = 128).
bool wgrad3x3n_supported(int64_t N, int H, int W, int C, int Cout);
int wgrad3x3n_splits(int64_t N, int H, int splits);
int wgrad3x3n_groups(int C, int Cout, int variant);
void wgrad3x3n(const void* dy, const void* x, float* ws, int64_t N, int H, int W, int C, int Cout, int splits,
               int variant, hipStream_t stream);
// dst[c][r] = src[r][c], bf16 (rows, cols, leading dims multiples of 8)
void transpose_bf16(const void* src, void* dst, int64_t rows, int64_t cols, int64_t lds, int64_t ldd,
                    hipStream_t stream);

// ---- Anderson-acceleration solver (DEQ) --------------------------------------------
// X: fp32 history, F: fp32 or bf16 history, [bsz][m rows of row_stride][d] (batch_stride between batches).
// anderson_gram: partials[b][chunk][37]: the upper-triangle pair sums of G G^T (G = F - X over
// rows < n; pair (i, j>=i) at index i*n - i*(i-1)/2 + (j-i)) and |F[last]|^2 at [36];
// sum over chunks on the host side. anderson_gram_chunks: the chunk count to allocate for.
int anderson_gram_chunks(int64_t bsz, int64_t d);
// G (nullable): stored G = F - X rows (same layout); rows with their bit set in `fresh` are
// recomputed from F - X and written to G, the others are read from G.
// F: fp32 or bf16 (f_dtype), same element layout as X; X and G: h_dtype (fp32 or bf16).
void anderson_gram(const void* X, const void* F, int f_dtype, void* G, unsigned fresh, float* partials, int64_t bsz,
                   int64_t d, int64_t row_stride, int64_t batch_stride, int n, int last, int chunks, hipStream_t stream,
                   int h_dtype = 7);
// X[b, slot] = beta * sum_i alpha[b][i] F[b, i] + (1 - beta) * sum_i alpha[b][i] X[b, i] (i < n);
// z (nullable, [bsz][d], dtype z_dtype): the new iterate cast to the model dtype.
void anderson_mix(void* X, const void* F, int f_dtype, const float* alpha, void* z, int z_dtype, int64_t bsz,
                  int64_t d, int64_t row_stride, int64_t batch_stride, int n, int slot, float beta, hipStream_t stream,
                  int h_dtype = 7);
// anderson_solve: from anderson_gram's partials, alpha[b][0..n) of the regularised Anderson system
// [[0, 1^T], [1, G G^T + lam I]] a = e_0 (a[1..n]) per batch element (bsz <= 1024, one launch),
// and (res nullable) the relative residual of row `last` into res[0].
void anderson_solve(const float* partials, int chunks, int64_t bsz, int n, int last, float lam, float* alpha,
                    float* res, hipStream_t stream);
// adjoint_step: u_new = vjp + grad (dtype), partials[blocks] = per-workgroup sums of (u_new - u)^2
// (fp32; n % 8 == 0, 16-byte aligned, same memory layout); adjoint_step_blocks: the grid size.
int adjoint_step_blocks(int64_t n);
void adjoint_step(const void* vjp, const void* grad, const void* u, void* u_new, float* partials, int blocks,
                  int64_t n, int dtype, hipStream_t stream);

// ---- fused NHWC GroupNorm (+ add, + ReLU on its input); one workgroup per sample ---------
// forward: h = [relu](x [+ add]) (stored when h != nullptr); y = GN(h) * w + b (w/b fp32, nullable);
// mean / rstd [N][G] fp32 saved. backward: dh = d(GN)/dh [* (h > 0) when relu], the gradient of
// both x and add; partials[N][2][C] = per-sample (dw, db).
// y_stride: y's sample stride in elements (0: HW * C, dense) — y can be an Anderson history slot.
void groupnorm_nhwc_fwd(const void* x, const void* add, void* h, void* y, const float* w, const float* b, float* mean,
                        float* rstd, int64_t N, int64_t HW, int64_t C, int64_t G, bool relu, float eps, int dtype,
                        hipStream_t stream, int64_t y_stride = 0);
void groupnorm_nhwc_bwd(const void* dy, const void* h, const float* mean, const float* rstd, const float* w, void* dh,
                        float* partials, int64_t N, int64_t HW, int64_t C, int64_t G, bool relu, int dtype,
                        hipStream_t stream);

// ---- the DEQ cell in one kernel per evaluation (kernels/deq_cell.hip) ----------------------
// f(z, x) = GN3(relu(z + GN2(x + conv2(GN1(relu(conv1 z)))))) on NHWC bf16 [N][H*W][48]; one
// workgroup per sample, everything LDS-resident. w1 / w2: [C][9C] bf16 with k = tap * C + ci.
// gn_w / gn_b: 3 fp32 vectors each (nullable). out (bf16, sample stride out_stride elements, 0 =
// dense) and/or out32 (fp32, sample stride out32_stride elements); h[3] (the GroupNorm inputs) and mean / rstd[3] ([N][G]) nullable.
// vjp: J_f(z)^T u from that state; w2t / w1t are the transposed tap-flipped filters (k = tap * C + co).
bool deq_cell_supported(int64_t H, int64_t W, int64_t C, int64_t G);
void deq_cell_fwd(const void* z, const void* x, const void* w1, const void* w2, const float* const* gn_w,
                  const float* const* gn_b, void* out, float* out32, int64_t out32_stride, void* const* h,
                  float* const* mean, float* const* rstd, int64_t N, int64_t H, int64_t W, int64_t C, int64_t G,
                  float eps, hipStream_t stream, int64_t out_stride = 0);
// grad / ss_part (nullable together): the adjoint update fused in, out = bf16(J^T u + grad) and
// ss_part[N] the per-sample sum of (out - u)^2; deq_adjoint_check sums them (ss_out) and tests
// flag = (sum <= *thresh2) in one tiny launch.
void deq_cell_vjp(const void* u, const void* const* h, const void* w2t, const void* w1t, const float* const* gn_w,
                  const float* const* mean, const float* const* rstd, void* out, const void* grad, float* ss_part,
                  int64_t N, int64_t H, int64_t W, int64_t C, int64_t G, hipStream_t stream);
void deq_adjoint_check(const float* part, int64_t n, const float* thresh2, float* ss_out, float* flag,
                       hipStream_t stream);

// ---- GELU backward + bias gradient (transformer MLP fc1) ---------------------------------
// dh = dy * gelu'(h) (exact erf form); partials[blocks][N] = per-workgroup column sums of dh
// (sum with gemm_splitk_reduce). N/8 must be a multiple of 64, <= 1024.
int gelu_bwd_bias_blocks(int64_t rows);
// Column sums of a row-major [rows][N] matrix (N % 8 == 0, N <= 8192) into per-workgroup fp32
// partial rows [blocks][N] (sum them with gemm_splitk_reduce): the bias gradient of a Linear.
int colsum_blocks(int64_t rows);
// Measurement tool: `blocks` workgroups holding their CU slots for `microseconds` of wall time
// on `stream` (stands in for RCCL's kernels at world size 1, where RCCL launches none).
void emulate_comm(int blocks, double microseconds, hipStream_t stream, int threads, int lds_bytes);
void colsum(const void* x, float* partials, int blocks, int64_t rows, int64_t N, int dtype, hipStream_t stream);
void gelu_bwd_bias(const void* dy, const void* h, void* dh, float* partials, int blocks, int64_t rows, int64_t N,
                   int dtype, hipStream_t stream);
// GELU form of the fused GELU kernels (gelu_bwd_bias, gemm_nt EPI 1 / 2): 1 tanh (NNlib's `gelu`,
// the default), 0 exact erf. Host-side switch read at launch.
void gelu_set_form(int tanh_form);
// g = gelu(h) (the selected form) over n bf16 / fp16 elements, n % 8 == 0, 16-B aligned
void gelu_fwd(const void* h, void* g, int64_t n, int dtype, hipStream_t stream);
int gelu_form();

}  // namespace fluxmpi
