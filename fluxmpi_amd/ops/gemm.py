"""Wrappers of the MFMA bf16 GEMM (``csrc/kernels/gemm.hip``) as the three passes of a
1x1 convolution on NHWC activations viewed as ``[M = N*H*W, C]`` matrices.

* :func:`conv1x1_fwd`   ``Y = act(X) @ W^T`` (+ optional BatchNorm statistics of Y)
* :func:`conv1x1_dgrad` ``dX = dY @ W``
* :func:`conv1x1_wgrad` ``dW = dY^T @ act(X)`` (split-K, fp32 accumulation)

``act(X) = relu(X * scale + shift)`` per input channel, when ``in_affine`` is
given: the previous BatchNorm + ReLU applied on the fly (never stored).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _ext
from . import gemm_nt as _NT
from . import graddst

SHARDS = 64  # == kShards in csrc/kernels/{batchnorm,gemm}.hip
# LDS buffering of the GEMM main loop: 0 = per-shape choice in the kernel launcher, 1 or 2 forces it
NBUF = 0
# GEMM kernel: 0 = launcher's choice, 1 = register-staged (gemm.hip), 2 = LDS-DMA pipelined (gemm_glds.hip)
ENGINE = int(os.environ.get("FLUXMPI_GEMM_ENGINE", "0"))
def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t):
    return t.data_ptr() if t is not None else 0


def gemm(a, b, c, *, M, N, K, lda, ldb, ldc, a_kmajor=True, b_kmajor=True, mode=0, splits=1, a_affine=None,
         b_affine=None, stats=None, tile_m=0, tile_n=0, nbuf=0, residual=None, bn_bwd=None, conv=None, engine=None,
         res_mask=None, res_sub=None, a_sub=None, conv_stride=1):
    """``res_sub=(H, W)``: ``residual`` is the compact stride-2 subsample of the [M/(H*W), H, W]
    row grid (added at even (h, w) only). ``a_sub=(H, W)``: A row (n, ho, wo) is pixel (n, 2ho, 2wo)
    of the NHWC image ``a`` [M/(Ho*Wo), H, W, lda] (a stride-2 1x1 convolution). ``bn_bwd``: ``(x2d, w32, b32, mean, inv, mask, relu_mode)`` of a BatchNorm whose output
    gradient is C — with ``mode=1`` the epilogue accumulates that BatchNorm's backward
    reductions into ``stats`` instead of C's sum / sum of squares. ``conv=(H, W, C)``: A is the
    implicit 3x3/s1/p1 im2col of the NHWC image batch ``a`` (K = 9*C)."""
    C = _ext.get(required=True)
    asc, ash = a_affine if a_affine is not None else (None, None)
    bsc, bsh = b_affine if b_affine is not None else (None, None)
    bx, bw, bb, bmean, binv, bmask, brm = bn_bwd if bn_bwd is not None else (None,) * 6 + (0,)
    C.gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), lda, ldb, ldc, M, N, K, a_kmajor, b_kmajor, mode, splits,
                _ptr(asc), _ptr(ash), _ptr(bsc), _ptr(bsh), _ptr(stats), tile_m, tile_n, _stream(c), nbuf or NBUF,
                _ptr(residual), residual.stride(0) if residual is not None else 0, _ptr(bx), _ptr(bw), _ptr(bb),
                _ptr(bmean), _ptr(binv), _ptr(bmask), int(brm), *(conv if conv is not None else (0, 0, 0)),
                ENGINE if engine is None else engine, _ptr(res_mask), *(res_sub if res_sub is not None else (0, 0)),
                *(a_sub if a_sub is not None else (0, 0)), int(conv_stride))
    return c


def conv1x1_fwd(x2d: torch.Tensor, w2d: torch.Tensor, in_affine=None, stats: torch.Tensor | None = None):
    """``x2d`` [M, Cin] bf16, ``w2d`` [Cout, Cin] bf16 -> [M, Cout] bf16.

    ``stats`` (fp32 [16, 2, Cout], zeroed) receives per-channel sum / sumsq of the output.
    """
    M, K = x2d.shape
    N = w2d.shape[0]
    y = torch.empty(M, N, device=x2d.device, dtype=torch.bfloat16)
    if (in_affine is None and x2d.stride(0) == K and w2d.stride(0) == K and x2d.stride(1) == 1 and w2d.stride(1) == 1
            and _NT.gemm_ok(M, N, K, x2d, w2d)):
        return _NT.gemm_plain(x2d, w2d, y, stats)  # 256x256 persistent kernel (+ statistics epilogue)
    gemm(x2d, w2d, y, M=M, N=N, K=K, lda=x2d.stride(0), ldb=w2d.stride(0), ldc=N, a_kmajor=True, b_kmajor=True,
         mode=1 if stats is not None else 0, a_affine=in_affine, stats=stats)
    return y


def conv1x1_dgrad(dy2d: torch.Tensor, w2d: torch.Tensor, residual: torch.Tensor | None = None,
                  out: torch.Tensor | None = None, bn_bwd=None, stats: torch.Tensor | None = None,
                  w4d: torch.Tensor | None = None, residual_mask: torch.Tensor | None = None, residual_sub=None):
    """``dy2d`` [M, Cout], ``w2d`` [Cout, Cin] -> dX [M, Cin] bf16 (``+ residual`` [M, Cin] bf16 fused
    into the epilogue: the gradient of a residual block's input in one pass). ``bn_bwd`` /
    ``stats``: accumulate the backward reductions of the BatchNorm that produced the conv's
    input (see :func:`gemm`) into the sharded ``stats`` workspace. ``w4d``: the filter parameter
    itself (its forward called :func:`note_filter`): enables the LDS-DMA kernel on the cached W^T.
    ``residual_sub=(H, W)``: the residual is the compact stride-2 subsample (see :func:`gemm`)."""
    M, Co = dy2d.shape
    Ci = w2d.shape[1]
    dx = out if out is not None else torch.empty(M, Ci, device=dy2d.device, dtype=torch.bfloat16)
    if residual is not None:
        rows = M if residual_sub is None else \
            M // (residual_sub[0] * residual_sub[1]) * ((residual_sub[0] + 1) // 2) * ((residual_sub[1] + 1) // 2)
        assert residual.shape == (rows, Ci) and residual.dtype == torch.bfloat16 and residual.stride(1) == 1
    if bn_bwd is not None:
        assert stats is not None and dx.stride(0) == Ci and bn_bwd[0].shape == (M, Ci) and bn_bwd[0].stride(0) == Ci
    if ENGINE != 1 and w4d is not None and dy2d.stride(0) % 8 == 0 and Ci % 8 == 0:
        # LDS-DMA kernel on the cached W^T (K-major B); the BN-backward epilogue is supported too
        if residual_mask is not None:
            assert residual is not None and residual.stride(0) == Ci and residual_mask.numel() * 8 == M * Ci
        if (residual is None and bn_bwd is None and dy2d.stride(0) == Co and dx.stride(0) == Ci
                and _NT.gemm_ok(M, Ci, Co, dy2d, w4d)):
            return _NT.gemm_plain(dy2d, filter_t(w4d), dx)  # W^T [Ci][Co]: both operands k-contiguous
        gemm(dy2d, filter_t(w4d), dx, M=M, N=Ci, K=Co, lda=dy2d.stride(0), ldb=Co, ldc=dx.stride(0),
             residual=residual, mode=1 if bn_bwd is not None else 0, stats=stats, bn_bwd=bn_bwd,
             engine=ENGINE or 2, res_mask=residual_mask, res_sub=residual_sub)
        return dx
    if residual_mask is not None or residual_sub is not None:
        raise RuntimeError("conv1x1_dgrad: a masked / stride-2 residual needs the LDS-DMA kernel "
                           "(w4d, FLUXMPI_GEMM_ENGINE != 1)")
    gemm(dy2d, w2d, dx, M=M, N=Ci, K=Co, lda=dy2d.stride(0), ldb=w2d.stride(0), ldc=dx.stride(0), a_kmajor=True,
         b_kmajor=False, residual=residual, mode=1 if bn_bwd is not None else 0, stats=stats, bn_bwd=bn_bwd,
         engine=1)
    return dx


# ---- transposed filters for the input-gradient GEMMs ------------------------------------------
# The dgrad GEMMs of the LDS-DMA kernel take the filter as a K-major B operand: W^T [ci][co] for
# a 1x1 convolution, the transposed AND flipped [ci][3][3][co] for a 3x3 one. Every forward of
# one of our convolutions marks its filter stale; the first input-gradient request of the
# backward then refreshes ALL stale filters in one launch (csrc transpose_filters), so a
# ResNet-50 step pays ~2 launches instead of one transpose per convolution. (Weights change
# only between a forward and the next one — the optimiser step — so the backward always sees
# the filters its forward used; a captured HIP graph replays the refresh launch too.)
_FILT: dict = {}  # id(w) -> [weakref(w), wt | None, fresh]


def note_filter(w: torch.Tensor) -> None:
    e = _FILT.get(id(w))
    if e is None or e[0]() is not w:
        _FILT[id(w)] = [weakref.ref(w), None, False]
    else:
        e[2] = False


def filter_t(w: torch.Tensor) -> torch.Tensor:
    """``w`` [co, ci, kh, kw] -> ``[ci, kh*kw*co]`` (taps flipped), from the batched cache."""
    e = _FILT.get(id(w))
    if e is None or e[0]() is not w:
        note_filter(w)
        e = _FILT[id(w)]
    if not e[2]:
        srcs, dsts, cos, cis, taps, keep, fresh = [], [], [], [], [], [], []
        for k, ent in list(_FILT.items()):
            t = ent[0]()
            if t is None:
                del _FILT[k]
                continue
            if ent[2] or t.device != w.device:
                continue
            co, ci = t.shape[0], t.shape[1]
            T = t.shape[2] * t.shape[3] if t.dim() == 4 else 1
            src = t.permute(0, 2, 3, 1).contiguous() if t.dim() == 4 else t.contiguous()  # [co][taps][ci]
            if ent[1] is None or ent[1].numel() != ci * T * co or ent[1].dtype != t.dtype:
                ent[1] = torch.empty(ci, T * co, device=t.device, dtype=t.dtype)
            srcs.append(src.data_ptr())
            dsts.append(ent[1].data_ptr())
            cos.append(co)
            cis.append(ci)
            taps.append(T)
            keep.append(src)  # alive until the launch is enqueued
            fresh.append(ent)
        C = _ext.get(required=True)
        C.transpose_filters(srcs, dsts, cos, cis, taps, _stream(w))
        for ent in fresh:
            ent[2] = True
    return e[1]


def conv_n_ok(pixels: int, c: int, co: int, h: int, w: int, *tensors: torch.Tensor) -> bool:
    """The narrow-channel 3x3 kernel (``conv3x3n.hip``: C = Cout in {64, 128}, ResNet-50 stages
    1-2) takes this stride-1 convolution (16-B aligned bf16 operands)."""
    if not tensors[0].is_cuda or any(t.dtype != torch.bfloat16 or t.data_ptr() % 16 for t in tensors):
        return False
    C = _ext.get(required=False)
    return C is not None and hasattr(C, "conv3x3n") and bool(C.conv3x3n_supported(pixels, c, co, h, w))


def conv3x3n(x: torch.Tensor, w_taps: torch.Tensor, y: torch.Tensor, pixels: int, h: int, w: int,
             stats: torch.Tensor | None = None) -> torch.Tensor:
    """``y [pixels, Cout] = conv3x3(x)`` on the narrow-channel kernel: ``x`` NHWC memory, ``w_taps``
    [Cout][3][3][C] (tap-major), ``stats``: BatchNorm shards [64][2][Cout] (sum / sum of squares of
    the rounded output)."""
    C = _ext.get(required=True)
    c, co = x.shape[1], w_taps.shape[0]
    C.conv3x3n(x.data_ptr(), w_taps.data_ptr(), y.data_ptr(), stats.data_ptr() if stats is not None else 0,
               pixels, h, w, c, co, 3 if stats is not None else 0, _stream(x))
    return y


def conv3x3_fwd(x: torch.Tensor, w: torch.Tensor, in_affine=None, stats: torch.Tensor | None = None,
                out: torch.Tensor | None = None, engine: int | None = None) -> torch.Tensor:
    """3x3 / stride 1 / pad 1 convolution as an implicit GEMM on the MFMA kernel.

    ``x`` [N, C, H, W] bf16 channels_last, ``w`` [Co, C, 3, 3] bf16 -> [N, Co, H, W] channels_last.
    ``in_affine=(scale, shift)``: relu(x * scale + shift) per input channel applied on load (the
    previous BatchNorm + ReLU; the zero padding stays zero). ``stats``: per-output-channel
    sum / sumsq into the sharded BatchNorm workspace. ``engine``: force a tile configuration of the
    LDS-DMA kernel (7 / 8: 256x128 tiles; see gemm_glds.hip), e.g. the one an autotune picked;
    ``None`` / 0: automatic — the 256x256 persistent kernel (``gemm_nt``) where the shape qualifies.
    """
    n, c, h, wd = x.shape
    co = w.shape[0]
    xs = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
    w2 = w.permute(0, 2, 3, 1).contiguous()  # [Co][3][3][C]: K-major over (tap, channel)
    note_filter(w)
    y = out if out is not None else torch.empty(n, h, wd, co, device=x.device, dtype=x.dtype).permute(0, 3, 1, 2)
    M = n * h * wd
    if (in_affine is None and not engine and y.is_contiguous(memory_format=torch.channels_last)
            and conv_n_ok(M, c, co, h, wd, xs, w2, y)):
        return conv3x3n(xs, w2, y, M, h, wd, stats)  # narrow channels: the halo staged once per tile
    if (in_affine is None and not engine and y.is_contiguous(memory_format=torch.channels_last)
            and _NT.conv_ok(M, c, co, xs, w2)):
        return _NT.conv3x3(xs, w2.view(co, 9 * c), y, stats)  # 256x256 persistent implicit GEMM
    gemm(xs, w2, y, M=M, N=co, K=9 * c, lda=c, ldb=9 * c, ldc=co, mode=1 if stats is not None else 0,
         a_affine=in_affine, stats=stats, conv=(h, wd, c), engine=engine or None)
    return y


def conv3x3_s2_fwd(x: torch.Tensor, w: torch.Tensor, stats: torch.Tensor | None = None) -> torch.Tensor:
    """3x3 / stride 2 / pad 1 convolution as an implicit GEMM over the output pixels (each A row
    stages the taps around input pixel (2ho, 2wo)); ``stats`` as in :func:`conv3x3_fwd`."""
    n, c, h, wd = x.shape
    co = w.shape[0]
    ho, wo = (h + 1) // 2, (wd + 1) // 2
    xs = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
    w2 = w.permute(0, 2, 3, 1).contiguous()  # [Co][3][3][C]
    y = torch.empty(n, ho, wo, co, device=x.device, dtype=x.dtype).permute(0, 3, 1, 2)
    gemm(xs, w2, y, M=n * ho * wo, N=co, K=9 * c, lda=c, ldb=9 * c, ldc=co, mode=1 if stats is not None else 0,
         stats=stats, conv=(h, wd, c), conv_stride=2)
    return y


# stride-2 3x3 input gradients on the parity-class implicit GEMM (conv3x3_s2_dgrad): OFF by
# default ("1" turns it on) — measured slower than MIOpen on ResNet-50: the four class GEMMs re-read
# dY once per tap (9x per layer) and took 141 / 156 / 193 us for the 7x7x512 / 14x14x256 / 28x28x128
# layers against ~140 us each for MIOpen's igemm_bwd + its output fill; ResNet-50 12.74k / 12.72k vs
# 12.80k / 12.76k img/s (profiles/rd6e_s2_dgrad_ab.jsonl). A one-pass kernel (each dY tile staged once
# for the 2 x 2 output parities, conv3x3n-style) is the form that would win.
S2_DGRAD = os.environ.get("FLUXMPI_S2_DGRAD", "0") == "1"


def s2_dgrad_ok(dy: torch.Tensor, w: torch.Tensor, x_shape) -> bool:
    """Shapes :func:`conv3x3_s2_dgrad` takes: even input sizes (each parity class is the dY grid),
    Cout % 32 == 0 (a K tile inside one tap), Cin % 8 == 0, bf16."""
    if not (S2_DGRAD and ENGINE != 1 and dy.is_cuda and dy.dtype == w.dtype == torch.bfloat16):
        return False
    n, co, ho, wo = dy.shape
    ci = w.shape[1]
    h, wd = x_shape[2], x_shape[3]
    return (tuple(w.shape[2:]) == (3, 3) and h == 2 * ho and wd == 2 * wo and co % 32 == 0 and ci % 8 == 0
            and n * h * wd < 2 ** 31)


def conv3x3_s2_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape) -> torch.Tensor:
    """Input gradient of the 3x3 / stride 2 / pad 1 convolution (even input sizes) as four
    implicit GEMMs, one per output parity class (py, px): dX pixel (2a + py, 2b + px) only
    receives the taps kh = 1 (py = 0) or kh = 0, 2 (py = 1) — dY rows a, and a + 1 / a — and
    likewise in columns, so the classes take 1, 2, 2 and 4 taps: exactly the convolution's
    9 Cout-deep products per 2 x 2 input block, no zero-inserted dY, no atomics, every dX element
    written once. A = the dY grid itself (rows = class pixels), B = the flipped transposed filter
    (the batched ``filter_t`` cache; each class indexes its taps), epilogue rows remapped to the
    class's dX pixels (``gemm_glds.hip``, ``conv_s = 16 + 2 py + px``). Replaces MIOpen's
    backward-data kernels (ResNet-50: 2 x 112 + 106 us per step plus a 28 us output fill each,
    ``profiles/rd5ba_resnet50_steady.md``)."""
    n, co, ho, wo = dy.shape
    ci = w.shape[1]
    h, wd = x_shape[2], x_shape[3]
    dys = dy if dy.is_contiguous(memory_format=torch.channels_last) else dy.contiguous(
        memory_format=torch.channels_last)
    wt = filter_t(w)  # [ci][3][3][co] flipped: original tap (kh, kw) at column block 8 - (3 kh + kw)
    dx = torch.empty(n, h, wd, ci, device=dy.device, dtype=dy.dtype).permute(0, 3, 1, 2)
    for cls in range(4):
        taps = (2 if cls >> 1 else 1) * (2 if cls & 1 else 1)
        gemm(dys, wt, dx, M=n * ho * wo, N=ci, K=taps * co, lda=co, ldb=9 * co, ldc=ci, conv=(ho, wo, co),
             conv_stride=16 + cls)
    return dx


def conv3x3_dgrad(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None, bn_bwd=None,
                  stats: torch.Tensor | None = None, residual: torch.Tensor | None = None) -> torch.Tensor:
    """Input gradient of the 3x3/s1/p1 convolution: the same implicit GEMM over dY with the
    filter transposed and flipped (``WT[ci][r][s][co] = W[co][ci][2-r][2-s]``). ``bn_bwd`` /
    ``stats``: the epilogue accumulates the backward reductions of the BatchNorm that produced
    the convolution's input (see :func:`gemm`). ``residual`` (NHWC, the input's shape): added in the
    epilogue — the other summand of the input's gradient when the input has a second consumer."""
    n, co, h, wd = dy.shape
    ci = w.shape[1]
    dys = dy if dy.is_contiguous(memory_format=torch.channels_last) else dy.contiguous(
        memory_format=torch.channels_last)
    if ENGINE == 1:  # register-staged kernel: transpose on the spot
        wt = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()  # [Ci][3][3][Co]
    else:
        wt = filter_t(w)
    dx = out if out is not None else torch.empty(n, h, wd, ci, device=dy.device, dtype=dy.dtype).permute(0, 3, 1, 2)
    if bn_bwd is not None:
        assert stats is not None and bn_bwd[0].shape == (n * h * wd, ci) and ENGINE != 1
    if (bn_bwd is None and residual is None and ENGINE != 1 and dx.is_contiguous(memory_format=torch.channels_last)
            and conv_n_ok(n * h * wd, co, ci, h, wd, dys, wt, dx)):
        return conv3x3n(dys, wt, dx, n * h * wd, h, wd)  # the flipped transpose [ci][3][3][co] as the filter
    r2 = None
    if residual is not None:
        assert residual.shape == dx.shape and residual.dtype == dy.dtype and bn_bwd is None
        r2 = residual.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(-1, ci)
    if (bn_bwd is None and ENGINE != 1 and dx.is_contiguous(memory_format=torch.channels_last)
            and _NT.conv_ok(n * h * wd, co, ci, dys, wt, *(() if r2 is None else (r2,)))):
        # the flipped transpose [ci][3][3][co] as B; the residual (if any) added in the epilogue
        return _NT.conv3x3(dys, wt, dx, residual=r2)
    gemm(dys, wt, dx, M=n * h * wd, N=ci, K=9 * co, lda=co, ldb=9 * co, ldc=ci, conv=(h, wd, co),
         mode=1 if bn_bwd is not None else 0, stats=stats, bn_bwd=bn_bwd, residual=r2)
    return dx


BK = 32  # K tile of the kernel (split boundaries are multiples of it)


def wgrad_splits(M: int, co: int, ci: int) -> int:
    """Split-K factor for the weight gradient (K = M pixels).

    Splits write fp32 partials with plain stores (a [splits, co, ci] workspace, then one
    reduce pass), so their cost is ~2 x splits x co*ci*4 bytes of streaming traffic: aim
    at ~512 workgroups for the 256 CUs, keep >= 256 pixels per split and the partial
    traffic under half of the operand bytes.
    """
    tiles = max(1, (co + 127) // 128) * max(1, (ci + 127) // 128)
    in_bytes = M * (co + ci) * 2
    out_bytes = co * ci * 4
    s_occ = -(-512 // tiles)
    s_bw = max(1, in_bytes // (4 * out_bytes))
    return int(max(1, min(s_occ, s_bw, M // 256)))


def _actual_splits(K: int, splits: int) -> int:
    """The kernel launcher rounds the per-split K range up to whole K tiles."""
    nk = -(-K // BK)
    kps = -(-nk // splits) * BK
    return -(-K // kps)


def conv1x1_wgrad(dy2d: torch.Tensor, x2d: torch.Tensor, in_affine=None, out: torch.Tensor | None = None,
                  out_dtype: torch.dtype = torch.float32, splits: int | None = None):
    """``dy2d`` [M, Cout], ``x2d`` [M, Cin] -> dW [Cout, Cin] (``out_dtype``, fp32 accumulation).

    Written into ``out`` (overwritten) if given. One split: the GEMM stores dW directly
    (bf16 through the staged epilogue, fp32 plainly); several: fp32 partials + one reduce
    launch that also casts to the output dtype.
    """
    M, Co = dy2d.shape
    Ci = x2d.shape[1]
    if out is not None:
        out_dtype = out.dtype
    dw = out if out is not None else graddst.empty((Co, Ci), out_dtype, dy2d.device)
    s = _actual_splits(M, splits or wgrad_splits(M, Co, Ci))
    common = dict(M=Co, N=Ci, K=M, lda=dy2d.stride(0), ldb=x2d.stride(0), ldc=Ci, a_kmajor=False, b_kmajor=False,
                  b_affine=in_affine)
    if s == 1:
        gemm(dy2d, x2d, dw, mode=0 if dw.dtype == torch.bfloat16 else 3, splits=1, **common)
        return dw
    ws = torch.empty(s, Co, Ci, device=dy2d.device, dtype=torch.float32)
    gemm(dy2d, x2d, ws, mode=3, splits=s, **common)
    C = _ext.get(required=True)
    C.gemm_splitk_reduce(ws.data_ptr(), s, Co * Ci, dw.data_ptr(), 9 if dw.dtype == torch.bfloat16 else 7,
                         _stream(dw))
    return dw


# ---- weight gradients on the LDS-DMA transposed-operand kernel --------------------------------
# workgroups the weight-gradient split-K aims at (one round of the 3-per-CU kernel on 256 CUs)
WGRAD_TARGET_WG = 768


def _wgrad_splits_v2(M: int, N: int, K: int) -> int:
    """Split-K factor: ~WGRAD_TARGET_WG workgroups, >= 256 pixels per split, and at most 64 MiB
    of fp32 partials (each is written once and read once by the reduce)."""
    tiles = max(1, -(-M // 128)) * max(1, -(-N // 128))
    s_occ = -(-WGRAD_TARGET_WG // tiles)
    s_bytes = max(1, (64 << 20) // (M * N * 4))
    return int(max(1, min(s_occ, s_bytes, K // 256)))


def _wgrad_reduce(ws, splits, dw):
    C = _ext.get(required=True)
    C.gemm_splitk_reduce(ws.data_ptr(), splits, dw.numel(), dw.data_ptr(), 9 if dw.dtype == torch.bfloat16 else 7,
                         _stream(dw))
    return dw


def _actual_splits_v2(K: int, splits: int) -> int:
    nk = -(-K // 64)
    kps = -(-nk // splits) * 64
    return -(-K // kps)


# weight-gradient kernel variant: 1 = 32-deep K-step / 3 stages, 2 = 64-deep / 2 stages
WGRAD_VARIANT = 1
# 1 (default): XCD-aware (split, tile) block order in the weight-gradient grid; 0: dispatch order
WGRAD_REMAP = True


def conv1x1_wgrad_v2(dy2d: torch.Tensor, x2d: torch.Tensor, out_dtype=torch.bfloat16, splits: int | None = None):
    """dW [Cout, Cin] = dY^T X over the pixels, split-K fp32 partials + one reduce launch."""
    K, Co = dy2d.shape
    Ci = x2d.shape[1]
    s = _actual_splits_v2(K, splits or _wgrad_splits_v2(Co, Ci, K))
    ws = torch.empty(s, Co, Ci, device=dy2d.device, dtype=torch.float32)
    C = _ext.get(required=True)
    C.gemm_wgrad(dy2d.data_ptr(), x2d.data_ptr(), ws.data_ptr(), dy2d.stride(0), x2d.stride(0), Co, Ci, K, s, 0, 0, 0,
                 _stream(dy2d), WGRAD_VARIANT | (0 if WGRAD_REMAP else 4))
    return _wgrad_reduce(ws, s, graddst.empty((Co, Ci), out_dtype, dy2d.device))


def conv1x1_wgrad_s2(dy2d: torch.Tensor, x: torch.Tensor, out_dtype=torch.bfloat16, splits: int | None = None):
    """Weight gradient of a stride-2 1x1 convolution: dW [Cout, Cin] = sum over the output pixels
    (n, ho, wo) of dY[pixel] x X[n, 2ho, 2wo] — the kernel gathers the even input pixels in its
    B staging (no strided copy of X). ``dy2d`` [N*Ho*Wo, Cout], ``x`` NCHW channels_last."""
    K, Co = dy2d.shape
    n, ci, h, w = x.shape
    xs = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
    assert K == n * ((h + 1) // 2) * ((w + 1) // 2)
    s = _actual_splits_v2(K, splits or _wgrad_splits_v2(Co, ci, K))
    ws = torch.empty(s, Co, ci, device=dy2d.device, dtype=torch.float32)
    C = _ext.get(required=True)
    C.gemm_wgrad(dy2d.data_ptr(), xs.data_ptr(), ws.data_ptr(), dy2d.stride(0), ci, Co, ci, K, s, h, w, 0,
                 _stream(dy2d), WGRAD_VARIANT | (0 if WGRAD_REMAP else 4), 1)
    return _wgrad_reduce(ws, s, graddst.empty((Co, ci), out_dtype, dy2d.device))


def conv3x3_wgrad_s2(dy: torch.Tensor, x: torch.Tensor, splits: int | None = None) -> torch.Tensor:
    """Weight gradient of the 3x3 / stride 2 / pad 1 convolution: the B operand is the implicit
    im2col over the output grid (tap (r, s) of output pixel (n, ho, wo) reads input pixel
    (n, 2ho + r - 1, 2wo + s - 1)). Returns [Co, Ci, 3, 3] in channels_last."""
    n, co, ho, wo = dy.shape
    ci, h, wd = x.shape[1], x.shape[2], x.shape[3]
    assert ho == (h + 1) // 2 and wo == (wd + 1) // 2
    dys = dy if dy.is_contiguous(memory_format=torch.channels_last) else dy.contiguous(
        memory_format=torch.channels_last)
    xs = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
    K, N = n * ho * wo, 9 * ci
    s = _actual_splits_v2(K, splits or _wgrad_splits_v2(co, N, K))
    ws = torch.empty(s, co, N, device=dy.device, dtype=torch.float32)
    C = _ext.get(required=True)
    C.gemm_wgrad(dys.data_ptr(), xs.data_ptr(), ws.data_ptr(), co, ci, co, N, K, s, h, wd, ci, _stream(dy),
                 WGRAD_VARIANT | (0 if WGRAD_REMAP else 4), 1)
    dw = graddst.empty((co, 3, 3, ci), dy.dtype, dy.device)
    _wgrad_reduce(ws, s, dw)
    return dw.permute(0, 3, 1, 2)


def wgrad3x3n_ok(x_shape, co: int) -> bool:
    """The narrow-channel 3x3 weight-gradient kernel (``wgrad3x3n.hip``: C in {64, 128}, Cout % 64
    == 0, H % 4 == 0, W % 4 == 0 up to 56 / 28 — ResNet-50 stages 1-2) takes this shape."""
    C = _ext.get()
    n, c, h, w = x_shape
    return C is not None and hasattr(C, "wgrad3x3n") and bool(C.wgrad3x3n_supported(n, h, w, c, co))


def conv3x3_wgrad_n(dy: torch.Tensor, x: torch.Tensor, variant: int = 1, target_wg: int = 256) -> torch.Tensor:
    """Weight gradient of the 3x3/s1/p1 convolution on ``wgrad3x3n.hip`` (input rows staged once
    per block of 4 image rows, the nine taps as offsets into them; variant 1: 8 waves, 0: 4):
    fp32 partials over ~``target_wg`` workgroups, then the split-K reduce. Returns [Co, Ci, 3, 3]
    in channels_last, like ``conv3x3_wgrad``."""
    n, co, h, wd = dy.shape
    ci = x.shape[1]
    dys = dy if dy.is_contiguous(memory_format=torch.channels_last) else dy.contiguous(
        memory_format=torch.channels_last)
    xs = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
    C = _ext.get(required=True)
    groups = C.wgrad3x3n_groups(ci, co, variant)
    s = C.wgrad3x3n_splits(n, h, max(1, target_wg // groups))
    ws = torch.empty(s, co, 9 * ci, device=dy.device, dtype=torch.float32)
    C.wgrad3x3n(dys.data_ptr(), xs.data_ptr(), ws.data_ptr(), n, h, wd, ci, co, s, variant, _stream(dy))
    dw = graddst.empty((co, 3, 3, ci), dy.dtype, dy.device)
    _wgrad_reduce(ws, s, dw)
    return dw.permute(0, 3, 1, 2)


def conv3x3_wgrad(dy: torch.Tensor, x: torch.Tensor, splits: int | None = None) -> torch.Tensor:
    """Weight gradient of the 3x3/s1/p1 convolution: dW[co][(r, s, ci)] = sum over pixels of
    dY[pix][co] * X[pix + (r-1)*W + (s-1)][ci] — the implicit im2col is the B operand. Returns
    [Co, Ci, 3, 3] in channels_last (the filter parameters' layout)."""
    n, co, h, wd = dy.shape
    ci = x.shape[1]
    dys = dy if dy.is_contiguous(memory_format=torch.channels_last) else dy.contiguous(
        memory_format=torch.channels_last)
    xs = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
    K, N = n * h * wd, 9 * ci
    s = _actual_splits_v2(K, splits or _wgrad_splits_v2(co, N, K))
    ws = torch.empty(s, co, N, device=dy.device, dtype=torch.float32)
    C = _ext.get(required=True)
    C.gemm_wgrad(dys.data_ptr(), xs.data_ptr(), ws.data_ptr(), co, ci, co, N, K, s, h, wd, ci, _stream(dy),
                 WGRAD_VARIANT | (0 if WGRAD_REMAP else 4))
    dw = graddst.empty((co, 3, 3, ci), dy.dtype, dy.device)
    _wgrad_reduce(ws, s, dw)
    return dw.permute(0, 3, 1, 2)
