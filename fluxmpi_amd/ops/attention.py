"""Packed-QKV softmax attention on our gfx950 kernels (``csrc/kernels/attention.hip``).

``attn_fwd_packed(qkv, heads) -> (out, stats)``: ``out = softmax(q k^T / 8) v`` for the
``[B, T, 3*H*64]`` packed q|k|v projection (no mask, no dropout), written as ``[B, T, H*64]``
(the layout the output projection reads: no transpose copy), plus fp32 ``stats``
``[B, H, T, 2]`` holding the row log-sum-exp for the backward.

``attn_bwd_packed(qkv, out, dy, heads, stats)``: the gradient of the packed q|k|v, written
straight into one ``[B, T, 3, H, 64]`` buffer (no per-gradient tensors, no interleaving copy).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _ext
from .fused_block import _stream


def supported(qkv: torch.Tensor, heads: int) -> bool:
    b, t, d3 = qkv.shape
    return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and d3 % 3 == 0 and d3 // 3 == 64 * heads
            and qkv.is_contiguous())


def _check(qkv, heads):
    if not supported(qkv, heads):
        raise ValueError("attention: needs a contiguous bf16 [B, T, 3*H*64] qkv on the GPU")


def attn_fwd_packed(qkv: torch.Tensor, heads: int):
    C = _ext.get(required=True)
    _check(qkv, heads)
    b, t, d3 = qkv.shape
    d = d3 // 3
    out = torch.empty((b, t, d), device=qkv.device, dtype=qkv.dtype)
    stats = torch.empty((b, heads, t, 2), device=qkv.device, dtype=torch.float32)
    p, es = qkv.data_ptr(), qkv.element_size()
    C.attn_fwd(p, p + d * es, p + 2 * d * es, out.data_ptr(), stats.data_ptr(), t * d3, d3, t * d, d, 64,
               b, t, heads, 64, 0.125, _stream(qkv))
    return out, stats


# FLUXMPI_ATTN_COLSUM=0: no column-sum partials from the backward (the bias gradient of the packed
# projection then runs its own column-sum pass over dQKV; A/B runs)
COLSUM = os.environ.get("FLUXMPI_ATTN_COLSUM", "1") != "0"


def attn_bwd_packed(qkv: torch.Tensor, out: torch.Tensor, dy: torch.Tensor, heads: int,
                    stats: torch.Tensor, colsum: bool | None = None) -> torch.Tensor:
    C = _ext.get(required=True)
    _check(qkv, heads)
    b, t, d3 = qkv.shape
    d = d3 // 3
    if out.shape != (b, t, d) or not out.is_contiguous() or out.dtype != qkv.dtype:
        raise ValueError("attn_bwd_packed: out must be attn_fwd_packed's contiguous [B, T, H*64]")
    if stats.shape != (b, heads, t, 2) or stats.dtype != torch.float32 or not stats.is_contiguous():
        raise ValueError("attn_bwd_packed: stats must be attn_fwd_packed's [B, H, T, 2] fp32")
    dy = dy.reshape(b, t, d)
    if not dy.is_contiguous():
        dy = dy.contiguous()
    if dy.dtype != qkv.dtype:
        dy = dy.to(qkv.dtype)
    dqkv = torch.empty_like(qkv)
    p, g, es = qkv.data_ptr(), dqkv.data_ptr(), qkv.element_size()
    # column-sum partials of dQKV from the kernels themselves: the packed projection's bias
    # gradient becomes a reduce over them (ops/linear.bias_grad takes them by data pointer)
    rows = C.attn_bwd_colpart_rows(b, t, heads, d3, d) if (COLSUM if colsum is None else colsum) else 0
    part = torch.empty(rows, d3, device=qkv.device, dtype=torch.float32) if rows > 0 else None
    C.attn_bwd(p, p + d * es, p + 2 * d * es, out.data_ptr(), dy.data_ptr(), g, g + d * es, g + 2 * d * es,
               stats.data_ptr(), t * d3, d3, t * d, d, 64, t * d, d, b, t, heads, 64, 0.125, _stream(qkv),
               part.data_ptr() if part is not None else 0)
    # the version pins the values: autograd may accumulate a second gradient into dQKV in place
    # (same pointer and size) before the projection's backward reads it
    _COLPART[0] = (weakref.ref(dqkv), part, dqkv._version) if part is not None else None
    return dqkv


# the latest backward's (weak reference to dQKV, column-sum partials): the next consumer of that gradient
# (the packed projection's Linear backward, the very next autograd node) takes it
_COLPART: list = [None]


def take_colpart(grad: torch.Tensor):
    """The [rows, N] fp32 column-sum partials of ``grad`` if it is the last attention backward's
    dQKV (then ``grad.sum(0) == partials.sum(0)`` up to rounding), else None; consumed once."""
    hit = _COLPART[0]
    if hit is None:
        return None
    src = hit[0]()  # the dQKV tensor itself, still alive (no reuse of a freed address)
    if src is None or src.data_ptr() != grad.data_ptr() or src.numel() != grad.numel() \
            or hit[1].shape[1] != grad.shape[-1] or src._version != hit[2]:
        return None
    _COLPART[0] = None
    return hit[1]


__all__ = ["attn_fwd_packed", "attn_bwd_packed", "supported", "take_colpart"]
