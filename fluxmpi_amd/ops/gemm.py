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

import torch

from . import _ext

SHARDS = 64  # == kShards in csrc/kernels/{batchnorm,gemm}.hip
# LDS buffering of the GEMM main loop: 0 = per-shape choice in the kernel launcher, 1 or 2 forces it
NBUF = int(os.environ.get("FLUXMPI_GEMM_NBUF", "0"))


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t):
    return t.data_ptr() if t is not None else 0


def gemm(a, b, c, *, M, N, K, lda, ldb, ldc, a_kmajor=True, b_kmajor=True, mode=0, splits=1, a_affine=None,
         b_affine=None, stats=None, tile_m=0, tile_n=0, nbuf=0, residual=None, bn_bwd=None):
    """``bn_bwd``: ``(x2d, w32, b32, mean, inv, mask, relu_mode)`` of a BatchNorm whose output
    gradient is C — with ``mode=1`` the epilogue accumulates that BatchNorm's backward
    reductions into ``stats`` instead of C's sum / sum of squares."""
    C = _ext.get(required=True)
    asc, ash = a_affine if a_affine is not None else (None, None)
    bsc, bsh = b_affine if b_affine is not None else (None, None)
    bx, bw, bb, bmean, binv, bmask, brm = bn_bwd if bn_bwd is not None else (None,) * 6 + (0,)
    C.gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), lda, ldb, ldc, M, N, K, a_kmajor, b_kmajor, mode, splits,
                _ptr(asc), _ptr(ash), _ptr(bsc), _ptr(bsh), _ptr(stats), tile_m, tile_n, _stream(c), nbuf or NBUF,
                _ptr(residual), residual.stride(0) if residual is not None else 0, _ptr(bx), _ptr(bw), _ptr(bb),
                _ptr(bmean), _ptr(binv), _ptr(bmask), int(brm))
    return c


def conv1x1_fwd(x2d: torch.Tensor, w2d: torch.Tensor, in_affine=None, stats: torch.Tensor | None = None):
    """``x2d`` [M, Cin] bf16, ``w2d`` [Cout, Cin] bf16 -> [M, Cout] bf16.

    ``stats`` (fp32 [16, 2, Cout], zeroed) receives per-channel sum / sumsq of the output.
    """
    M, K = x2d.shape
    N = w2d.shape[0]
    y = torch.empty(M, N, device=x2d.device, dtype=torch.bfloat16)
    gemm(x2d, w2d, y, M=M, N=N, K=K, lda=x2d.stride(0), ldb=w2d.stride(0), ldc=N, a_kmajor=True, b_kmajor=True,
         mode=1 if stats is not None else 0, a_affine=in_affine, stats=stats)
    return y


def conv1x1_dgrad(dy2d: torch.Tensor, w2d: torch.Tensor, residual: torch.Tensor | None = None,
                  out: torch.Tensor | None = None, bn_bwd=None, stats: torch.Tensor | None = None):
    """``dy2d`` [M, Cout], ``w2d`` [Cout, Cin] -> dX [M, Cin] bf16 (``+ residual`` [M, Cin] bf16 fused
    into the epilogue: the gradient of a residual block's input in one pass). ``bn_bwd`` /
    ``stats``: accumulate the backward reductions of the BatchNorm that produced the conv's
    input (see :func:`gemm`) into the sharded ``stats`` workspace."""
    M, Co = dy2d.shape
    Ci = w2d.shape[1]
    dx = out if out is not None else torch.empty(M, Ci, device=dy2d.device, dtype=torch.bfloat16)
    if residual is not None:
        assert residual.shape == (M, Ci) and residual.dtype == torch.bfloat16 and residual.stride(1) == 1
    if bn_bwd is not None:
        assert stats is not None and dx.stride(0) == Ci and bn_bwd[0].shape == (M, Ci) and bn_bwd[0].stride(0) == Ci
    gemm(dy2d, w2d, dx, M=M, N=Ci, K=Co, lda=dy2d.stride(0), ldb=w2d.stride(0), ldc=dx.stride(0), a_kmajor=True,
         b_kmajor=False, residual=residual, mode=1 if bn_bwd is not None else 0, stats=stats, bn_bwd=bn_bwd)
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
    dw = out if out is not None else torch.empty(Co, Ci, device=dy2d.device, dtype=out_dtype)
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
