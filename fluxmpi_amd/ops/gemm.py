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
         b_affine=None, stats=None, tile_m=0, tile_n=0, nbuf=0):
    C = _ext.get(required=True)
    asc, ash = a_affine if a_affine is not None else (None, None)
    bsc, bsh = b_affine if b_affine is not None else (None, None)
    C.gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), lda, ldb, ldc, M, N, K, a_kmajor, b_kmajor, mode, splits,
                _ptr(asc), _ptr(ash), _ptr(bsc), _ptr(bsh), _ptr(stats), tile_m, tile_n, _stream(c), nbuf or NBUF)
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


def conv1x1_dgrad(dy2d: torch.Tensor, w2d: torch.Tensor):
    """``dy2d`` [M, Cout], ``w2d`` [Cout, Cin] -> dX [M, Cin] bf16."""
    M, Co = dy2d.shape
    Ci = w2d.shape[1]
    dx = torch.empty(M, Ci, device=dy2d.device, dtype=torch.bfloat16)
    gemm(dy2d, w2d, dx, M=M, N=Ci, K=Co, lda=dy2d.stride(0), ldb=w2d.stride(0), ldc=Ci, a_kmajor=True,
         b_kmajor=False)
    return dx


def wgrad_splits(M: int, co: int, ci: int) -> int:
    """Split-K factor for the weight gradient (K = M pixels).

    Every split adds a whole fp32 ``co x ci`` tile with float atomics, which run
    at ~1.3 TB/s chip-wide (vs ~6 TB/s for plain streams): keep the atomic bytes
    under 1/8 of the operand bytes, and use just enough splits to put ~512
    workgroups on the 256 CUs.
    """
    tiles = max(1, (co + 127) // 128) * max(1, (ci + 127) // 128)
    in_bytes = M * (co + ci) * 2
    out_bytes = co * ci * 4
    s_bw = max(1, in_bytes // (8 * out_bytes))
    s_occ = max(1, -(-512 // tiles))
    return int(max(1, min(s_bw, s_occ, max(1, M // 256))))


def conv1x1_wgrad(dy2d: torch.Tensor, x2d: torch.Tensor, in_affine=None, out: torch.Tensor | None = None):
    """``dy2d`` [M, Cout], ``x2d`` [M, Cin] -> dW [Cout, Cin] fp32 (accumulated into ``out`` if given)."""
    M, Co = dy2d.shape
    Ci = x2d.shape[1]
    dw = out if out is not None else torch.zeros(Co, Ci, device=dy2d.device, dtype=torch.float32)
    gemm(dy2d, x2d, dw, M=Co, N=Ci, K=M, lda=dy2d.stride(0), ldb=x2d.stride(0), ldc=Ci, a_kmajor=False,
         b_kmajor=False, mode=2, splits=wgrad_splits(M, Co, Ci), b_affine=in_affine)
    return dw
