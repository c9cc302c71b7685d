"""``gelu(linear(x, W, b))`` with the GELU backward and the bias gradient in one HIP pass
(``csrc/kernels/gelu.hip``).

Autograd would run the GELU backward (read dy, h; write dh) and then reduce dh again for
the Linear's bias gradient. ``linear_gelu`` owns both ops: its backward writes ``dh`` and
per-workgroup column sums in one pass, then issues the same two GEMMs as ``nn.Linear``'s
backward (``dh @ W``, ``dh^T @ x``). CPU tensors and unsupported widths use the PyTorch
composition.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from .multi_tensor import DTYPE_CODE


def _native(h: torch.Tensor) -> bool:
    n = h.shape[-1]
    return (h.is_cuda and h.dtype in (torch.bfloat16, torch.float16) and n % 8 == 0 and (n // 8) % 64 == 0
            and n // 8 <= 1024 and h.numel() > 0)


def gelu_bwd_bias(dy: torch.Tensor, h: torch.Tensor, bias_dtype=torch.float32):
    """``(dh, db)``: ``dh = dy * gelu'(h)`` (erf form), ``db = dh.sum(rows)`` in ``bias_dtype``."""
    if not _native(h):
        hf = h.float()
        cdf = 0.5 * (1 + torch.erf(hf * 0.7071067811865476))
        pdf = torch.exp(-0.5 * hf * hf) * 0.3989422804014327
        dh = (dy.float() * (cdf + hf * pdf)).to(h.dtype)
        return dh, dh.float().reshape(-1, h.shape[-1]).sum(0).to(bias_dtype)
    C = _ext.get(required=True)
    n = h.shape[-1]
    rows = h.numel() // n
    h = h.contiguous()
    dy = dy.contiguous()
    dh = torch.empty_like(h)
    blocks = C.gelu_bwd_bias_blocks(rows)
    part = torch.empty(blocks, n, device=h.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(h.device).cuda_stream
    C.gelu_bwd_bias(dy.data_ptr(), h.data_ptr(), dh.data_ptr(), part.data_ptr(), blocks, rows, n,
                    DTYPE_CODE[h.dtype], stream)
    out_dt = bias_dtype if bias_dtype in (torch.float32, torch.bfloat16) else torch.float32
    db = torch.empty(n, device=h.device, dtype=out_dt)
    C.gemm_splitk_reduce(part.data_ptr(), blocks, n, db.data_ptr(), DTYPE_CODE[out_dt], stream)
    return dh, db.to(bias_dtype)


class GeluLink:
    """Hand-off between ``linear_gelu`` (fc1 + GELU) and the Linear that consumes its output
    (fc2, inside ``linear_add_layer_norm``): the consumer's input-gradient GEMM applies the
    GELU derivative and reduces fc1's bias gradient in its epilogue (gemm256.hip EPI 2) and
    deposits ``(dh, db)`` here; fc1's backward then skips its own GELU pass. The gradient
    autograd passes between the two nodes is a zero-stride placeholder (never read)."""

    __slots__ = ("h", "bias_dtype", "dh", "db")

    def __init__(self):
        self.h = self.bias_dtype = self.dh = self.db = None

    def take(self):
        out = (self.dh, self.db)
        self.h = self.dh = self.db = None
        return out


class _LinearGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, link=None):
        from . import gemm256
        n_out, n_in = weight.shape
        rows = x.numel() // n_in
        if x.is_contiguous() and gemm256.supported(rows, n_out, n_in, x, weight):
            # bias + GELU in the GEMM epilogue: h and gelu(h) from the same registers
            h2, g2 = gemm256.linear_fwd(x.view(rows, n_in), weight, bias, gelu=True)
            h, g = h2.view(*x.shape[:-1], n_out), g2.view(*x.shape[:-1], n_out)
        else:
            h = F.linear(x, weight, bias)
            g = F.gelu(h)
        ctx.save_for_backward(x, weight, h)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.link = link
        if link is not None:
            link.h, link.bias_dtype = h, ctx.bias_dtype or torch.float32
        return g

    @staticmethod
    def backward(ctx, dy):
        x, w, h = ctx.saved_tensors
        dh, db = ctx.link.take() if ctx.link is not None else (None, None)
        if dh is None:  # the consumer did not fuse the GELU derivative: own pass
            dh, db = gelu_bwd_bias(dy, h, ctx.bias_dtype or torch.float32)
        else:
            dh = dh.view(h.shape)
        n = h.shape[-1]
        dh2 = dh.reshape(-1, n)
        x2 = x.reshape(-1, x.shape[-1])
        from .linear import _wgrad_mode, dgrad, native_ok, weight_grad
        dx = dgrad(dh2, w).reshape(x.shape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            # long-K weight gradient on the split-K HIP kernel (ops/linear.py)
            dw = weight_grad(dh2, x2, w.dtype) if _wgrad_mode() == "ours" and native_ok(x2, dh2) else dh2.t() @ x2
        return dx, dw, (db if ctx.has_bias and ctx.needs_input_grad[2] else None), None


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
                link: GeluLink | None = None) -> torch.Tensor:
    """``F.gelu(F.linear(x, weight, bias))`` (exact GELU) with the fused backward on the GPU.
    ``link``: pass the same :class:`GeluLink` to the consuming ``linear_add_layer_norm``."""
    if x.is_cuda and _native_width(weight.shape[0], x.dtype):
        return _LinearGeluFn.apply(x, weight, bias, link)
    return F.gelu(F.linear(x, weight, bias))


def _native_width(n: int, dtype) -> bool:
    return dtype in (torch.bfloat16, torch.float16) and n % 8 == 0 and (n // 8) % 64 == 0 and n // 8 <= 1024
