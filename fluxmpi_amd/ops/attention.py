"""Packed-QKV softmax attention backward on our gfx950 kernels (``csrc/kernels/attention.hip``).

``attn_bwd_packed(qkv, out, dy, heads)`` returns the gradient of ``[B, T, 3*D]`` packed
q|k|v for ``out = softmax(q k^T / sqrt(64)) v`` (no mask, no dropout), written straight into
one ``[B, T, 3, H, 64]`` buffer: no per-gradient tensors, no interleaving copy.
``out`` is the forward's ``[B, H, T, 64]`` (any strides with a contiguous head dim);
``dy`` the ``[B, T, D]`` output gradient. The softmax statistics are recomputed from q and
k, so the forward's log-sum-exp is not needed.
"""
from __future__ import annotations

import math

import torch

from . import _ext
from .fused_block import _stream


def supported(qkv: torch.Tensor, heads: int) -> bool:
    b, t, d3 = qkv.shape
    return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and d3 % 3 == 0 and d3 // 3 == 64 * heads
            and qkv.is_contiguous())


def attn_bwd_packed(qkv: torch.Tensor, out: torch.Tensor, dy: torch.Tensor, heads: int) -> torch.Tensor:
    C = _ext.get(required=True)
    b, t, d3 = qkv.shape
    d = d3 // 3
    dh = d // heads
    if not supported(qkv, heads):
        raise ValueError("attn_bwd_packed: needs a contiguous bf16 [B, T, 3*H*64] qkv")
    if out.shape != (b, heads, t, dh) or out.stride(3) != 1 or out.dtype != qkv.dtype:
        raise ValueError(f"attn_bwd_packed: out must be [B, H, T, {dh}] with a contiguous head dim")
    dy = dy.reshape(b, t, d)
    if not dy.is_contiguous():
        dy = dy.contiguous()
    if dy.dtype != qkv.dtype:
        dy = dy.to(qkv.dtype)
    dqkv = torch.empty_like(qkv)
    stats = torch.empty((b, heads, t, 2), device=qkv.device, dtype=torch.float32)
    p = qkv.data_ptr()
    g = dqkv.data_ptr()
    es = qkv.element_size()
    C.attn_bwd(p, p + d * es, p + 2 * d * es, out.data_ptr(), dy.data_ptr(), g, g + d * es, g + 2 * d * es,
               stats.data_ptr(), t * d3, d3, out.stride(0), out.stride(2), out.stride(1), t * d, d,
               b, t, heads, dh, 1.0 / math.sqrt(dh), _stream(qkv))
    return dqkv


__all__ = ["attn_bwd_packed", "supported"]
