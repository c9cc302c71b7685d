"""ViT-Base/16 (Dosovitskiy et al. 2021) — BASELINE.json config "ViT-Base/16 Lux.jl DDP bf16".

224x224 input, 16x16 patches (196 tokens + [CLS] = 197), width 768, depth 12,
12 heads, MLP 3072, pre-LayerNorm, learned position embeddings, 1000-way
head: 86.6 M parameters in 152 tensors — large gradient buckets, which is the
point of this config for the DDP layer (bucketing + backward/comm overlap).

Attention runs our HIP kernels (``csrc/kernels/attention.hip``: MFMA, whole key range per
workgroup) on the packed QKV projection, output written in the projection's layout and the
three input gradients straight into one packed gradient (``packed_attention``); the patch embedding is a GEMM on the
unfolded patches; LayerNorms are the fused HIP kernels with the residual adds
folded in (``fluxmpi_amd.ops.layernorm``); every token-major Linear takes its weight
gradient from the split-K HIP GEMM and its bias gradient from the ``colsum`` kernel
(``fluxmpi_amd.ops.linear``).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.gelu import GeluLink, gelu, linear_gelu
from ..ops.layernorm import linear_add_layer_norm
from ..ops.linear import Linear

# False: autograd's GELU backward + separate bias reduction (A/B runs)
_FUSED_GELU = True
_FUSED_PROJ_LN = True
# False: the last block's MLP over every token (A/B runs; same result)
_CLS_ONLY = True


class PatchEmbed(nn.Module):
    def __init__(self, img=224, patch=16, cin=3, dim=768):
        super().__init__()
        self.patch = patch
        self.n = (img // patch) ** 2
        self.proj = Linear(cin * patch * patch, dim)

    def forward(self, x):
        n, c, h, w = x.shape
        p = self.patch
        x = x.reshape(n, c, h // p, p, w // p, p).permute(0, 2, 4, 1, 3, 5).reshape(n, (h // p) * (w // p), c * p * p)
        return self.proj(x)


def _attn_native(qkv, heads) -> bool:
    """Our HIP attention kernels (``csrc/kernels/attention.hip``) for bf16, head dim 64;
    ``FLUXMPI_ATTN=aten`` selects PyTorch's flash kernels (AOTriton) instead (A/B runs)."""
    import os
    if os.environ.get("FLUXMPI_ATTN", "native") == "aten":
        return False
    from ..ops.attention import supported
    return supported(qkv, heads)


class _PackedAttention(torch.autograd.Function):
    """Multi-head self-attention on the packed QKV projection ``[B, T, 3*D]``, returning
    ``[B, T, D]``. bf16 with head dim 64 runs our HIP kernels (``fluxmpi_amd.ops.attention``):
    the output is written in the projection's layout and the backward writes dQ/dK/dV straight
    into one packed gradient. Otherwise AOTriton's flash kernels + one interleaving copy.
    Through plain autograd, ``view(..).permute(2, 0, 3, 1, 4)`` + SDPA backward stacks the three
    gradients head-major and copies them back to the projection layout: 271 + 151 us per ViT-B
    block per step on MI355X (s48 trace); AOTriton's backward alone is ~740 us per block (s49)."""

    @staticmethod
    def forward(ctx, qkv, heads):
        b, t, d3 = qkv.shape
        d = d3 // 3
        if _attn_native(qkv, heads):
            from ..ops.attention import attn_fwd_packed
            out, stats = attn_fwd_packed(qkv, heads)
            ctx.save_for_backward(qkv, out, stats)
            ctx.meta = (heads, True)
            return out
        q, k, v = qkv.view(b, t, 3, heads, d // heads).unbind(2)
        q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        out, lse, cq, ck, mq, mk, seed, off, _ = torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.0, False)
        ctx.save_for_backward(qkv, out, lse, cq, ck, seed, off)
        ctx.meta = (heads, False, mq, mk)
        return out.transpose(1, 2).reshape(b, t, d)

    @staticmethod
    def backward(ctx, dy):
        if ctx.meta[1]:
            from ..ops.attention import attn_bwd_packed
            qkv, out, stats = ctx.saved_tensors
            return attn_bwd_packed(qkv, out, dy, ctx.meta[0], stats), None
        qkv, out, lse, cq, ck, seed, off = ctx.saved_tensors
        heads, _, mq, mk = ctx.meta
        b, t, d3 = qkv.shape
        d = d3 // 3
        dh = d // heads
        q, k, v = (u.transpose(1, 2) for u in qkv.view(b, t, 3, heads, dh).unbind(2))
        dout = dy.reshape(b, t, heads, dh).transpose(1, 2)
        dq, dk, dv = torch.ops.aten._scaled_dot_product_flash_attention_backward(
            dout, q, k, v, out, lse, cq, ck, mq, mk, 0.0, False, seed, off)
        dqkv = torch.empty((b, t, 3, heads, dh), device=qkv.device, dtype=qkv.dtype)
        torch.stack([dq.transpose(1, 2), dk.transpose(1, 2), dv.transpose(1, 2)], dim=2, out=dqkv)
        return dqkv.view(b, t, d3), None


def packed_attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    """``[B, T, 3*D]`` packed q|k|v -> ``[B, T, D]`` softmax attention (no mask, no dropout)."""
    b, t, d3 = qkv.shape
    d = d3 // 3
    if qkv.is_cuda and qkv.dtype in (torch.bfloat16, torch.float16) and (d // heads) % 8 == 0 and (d // heads) <= 256:
        return _PackedAttention.apply(qkv, heads)
    q, k, v = qkv.view(b, t, 3, heads, d // heads).permute(2, 0, 3, 1, 4)
    return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, t, d)


class Block(nn.Module):
    """Pre-LN transformer block. ``forward(x, pend)`` takes the residual stream ``x`` and the
    previous block's pending MLP branch ``pend = (g, fc2)`` (its GELU activations and its fc2)
    and returns ``(x + fc2(g) + attn, (g', self.fc2))``: each residual add is fused into the
    LayerNorm that reads its result, and the Linear producing the added branch (proj here, the
    previous block's fc2 at ln1) joins that LayerNorm in one autograd node
    (``ops/layernorm.linear_add_layer_norm``) whose backward also yields the Linear's bias
    gradient — no standalone add or bias-gradient kernels in either direction."""

    def __init__(self, dim, heads, mlp):
        super().__init__()
        from ..ops.layernorm import FusedLayerNorm
        self.heads = heads
        self.ln1 = FusedLayerNorm(dim, eps=1e-6)
        self.qkv = Linear(dim, 3 * dim)
        self.proj = Linear(dim, dim)
        self.ln2 = FusedLayerNorm(dim, eps=1e-6)
        self.fc1 = nn.Linear(dim, mlp)
        self.fc2 = Linear(mlp, dim)

    @staticmethod
    def _add_ln(ln, x, a, lin, link=None):
        """``(x + lin(a), ln(x + lin(a)))``."""
        if _FUSED_PROJ_LN:
            return linear_add_layer_norm(a, lin.weight, lin.bias, x, ln.weight, ln.bias, ln.eps, gelu_link=link)
        return ln.add_forward(x, lin(a))

    def forward(self, x, pend=None, cls_only=False):
        """``cls_only`` (the last block): only the [CLS] token's residual stream reaches the head,
        so after attention (which needs every token's keys / values) proj, ln2, fc1, GELU and fc2
        run on that token alone — exact, and ~1/13 of the step's GEMM FLOPs saved."""
        h = self.heads
        if pend is None:
            y = self.ln1(x)
        else:
            x, y = self._add_ln(self.ln1, x, *pend)  # x <- x + fc2(g) (previous block's MLP branch)
        a = packed_attention(self.qkv(y), h)
        if cls_only:
            x, a = x[:, 0], a[:, 0].contiguous()
        x, y = self._add_ln(self.ln2, x, a, self.proj)
        # fc1 + GELU: the GELU derivative and fc1's bias gradient come out of the consumer's
        # (the next ln1 node's fc2) input-gradient GEMM through the link (ops/gelu.py)
        link = GeluLink() if (_FUSED_GELU and not cls_only) else None
        g = linear_gelu(y, self.fc1.weight, self.fc1.bias, link=link) if _FUSED_GELU else gelu(self.fc1(y))
        return x, (g, self.fc2, link)


def cls_pos(x, cls, pos):
    """``cat([cls, x], 1) + pos`` in one elementwise pass: the patch tokens' sum is written straight
    into rows 1.. of the token buffer (no concatenated copy followed by a second add pass), the
    [CLS] row is the broadcast ``cls + pos[0]``; bit-identical to the composition (same bf16 adds).
    Not differentiable (``out=``): the forward of :class:`_ClsPos`, whose backward is explicit."""
    b, n, d = x.shape
    out = torch.empty(b, n + 1, d, device=x.device, dtype=x.dtype)
    torch.add(x, pos[:, 1:].to(x.dtype), out=out[:, 1:])
    out[:, 0] = cls[:, 0].to(x.dtype) + pos[:, 0].to(x.dtype)
    return out


class _ClsPos(torch.autograd.Function):
    """``cat([cls, x], 1) + pos``; the backward writes d(cls) and d(pos) — sums over the batch —
    into their DDP bucket slices when a communicating engine is attached (``ops/graddst.py``)."""

    @staticmethod
    def forward(ctx, x, cls, pos):
        ctx.params = (cls, pos)
        return cls_pos(x, cls, pos)

    @staticmethod
    def backward(ctx, dy):
        from ..ops import graddst
        cls, pos = ctx.params
        need = ctx.needs_input_grad
        dcls = dpos = None
        if need[2]:
            with graddst.into(pos):
                out = graddst.empty(tuple(pos.shape[1:]), pos.dtype, dy.device) if dy.dtype == pos.dtype else None
            # mismatched dtypes (fp32 parameter, bf16 activations): sum in fp32, round once
            dpos = (torch.sum(dy, 0, out=out) if out is not None
                    else dy.float().sum(0).to(pos.dtype)).view(pos.shape)
        if need[1]:
            with graddst.into(cls):
                out = graddst.empty((cls.shape[-1],), cls.dtype, dy.device) if dy.dtype == cls.dtype else None
            d0 = dy[:, 0]
            dcls = (torch.sum(d0, 0, out=out) if out is not None
                    else d0.float().sum(0).to(cls.dtype)).view(cls.shape)
        return (dy[:, 1:] if need[0] else None), dcls, dpos


class ViT(nn.Module):
    def __init__(self, img=224, patch=16, dim=768, depth=12, heads=12, mlp=3072, num_classes=1000):
        super().__init__()
        self.embed = PatchEmbed(img, patch, 3, dim)
        self.cls = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos = nn.Parameter(torch.randn(1, self.embed.n + 1, dim) * 0.02)
        self.blocks = nn.ModuleList([Block(dim, heads, mlp) for _ in range(depth)])
        from ..ops.layernorm import FusedLayerNorm
        self.ln = FusedLayerNorm(dim, eps=1e-6)
        self.head = Linear(dim, num_classes)  # ops.linear.Linear: dW / db into their bucket slices
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.embed(x)
        if x.is_cuda and torch.is_grad_enabled():
            x = _ClsPos.apply(x, self.cls, self.pos)
        else:
            # the differentiable composition (cls_pos writes through out=, which autograd does not trace)
            x = torch.cat([self.cls.expand(x.shape[0], -1, -1).to(x.dtype), x], 1) + self.pos.to(x.dtype)
        pend = None
        last = len(self.blocks) - 1
        for i, blk in enumerate(self.blocks):
            x, pend = blk(x, pend, cls_only=_CLS_ONLY and i == last)
        # only the [CLS] token reaches the head: finish its residual stream and normalise it alone
        if pend is None:
            c = x[:, 0]
        else:
            g, fc2, _ = pend
            c = x + fc2(g) if x.dim() == 2 else x[:, 0] + fc2(g)[:, 0]
        return self.head(self.ln(c))


def vit_b16(num_classes=1000, img=224, **kw) -> ViT:
    return ViT(img=img, num_classes=num_classes, **kw)


def vit_tiny(num_classes=10, img=32) -> ViT:
    return ViT(img=img, patch=8, dim=64, depth=2, heads=4, mlp=128, num_classes=num_classes)
