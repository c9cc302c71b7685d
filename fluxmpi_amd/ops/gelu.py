"""``gelu(linear(x, W, b))`` with the GELU backward and the bias gradient in one HIP pass
(``csrc/kernels/gelu.hip``).

GELU form (``FLUXMPI_GELU`` / :func:`set_form`): ``tanh`` (default) — NNlib's ``gelu``, the
activation of the reference's Lux / Metalhead ViT (``x/2 (1 + tanh(sqrt(2/pi)(x + 0.044715
x^3)))``) — or ``erf`` (exact). Both run the same kernels (``gelu.hip``, gemm_nt's epilogues)
at the same speed (ViT-B/16 7.04k / 7.06k tanh vs 7.04k / 7.05k erf, same box). A hipBLASLt
bias + GELU epilogue that also writes the pre-activation (``GELU_AUX_BIAS``, which would drop
the forward's elementwise GELU pass) has no gfx950 solution in either hipBLASLt of the image
(``scripts/probe/blaslt_epi_probe.cpp``, ``profiles/rd3y_blaslt_epilogue_probe.txt``).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _ext
from .multi_tensor import DTYPE_CODE

FORM = os.environ.get("FLUXMPI_GELU", "tanh").lower()
if FORM not in ("tanh", "erf"):
    raise ValueError(f"FLUXMPI_GELU must be 'tanh' or 'erf' (got {FORM!r})")
_synced = [None]  # form last pushed to the extension
_FWD_NATIVE = True  # False: F.gelu (the pre-round-3 path; tests)


def set_form(form: str) -> None:
    """Select the GELU form of every fused GELU path (``"tanh"`` or ``"erf"``)."""
    global FORM
    if form not in ("tanh", "erf"):
        raise ValueError(f"GELU form must be 'tanh' or 'erf' (got {form!r})")
    FORM = form


def _approx() -> str:
    return "tanh" if FORM == "tanh" else "none"


def gelu(h: torch.Tensor) -> torch.Tensor:
    """GELU of the selected form (PyTorch composition)."""
    return F.gelu(h, approximate=_approx())


def _gelu_fwd(h: torch.Tensor) -> torch.Tensor:
    """``gelu(h)`` without autograd: the HIP kernel (``gelu.hip`` gelu_fwd) for contiguous bf16 /
    fp16 CUDA tensors, else PyTorch."""
    if (_FWD_NATIVE and h.is_cuda and h.dtype in (torch.bfloat16, torch.float16) and h.is_contiguous()
            and h.numel() % 8 == 0):
        C = _ext.get(required=True)
        _sync(C)
        g = torch.empty_like(h)
        C.gelu_fwd(h.data_ptr(), g.data_ptr(), h.numel(), DTYPE_CODE[h.dtype],
                   torch.cuda.current_stream(h.device).cuda_stream)
        return g
    return gelu(h)


def _sync(C) -> None:
    if _synced[0] != FORM:
        C.gelu_set_form(1 if FORM == "tanh" else 0)
        _synced[0] = FORM


def _gelu_grad_ref(hf: torch.Tensor) -> torch.Tensor:
    if FORM == "tanh":
        k0 = 0.7978845608028654
        t = torch.tanh(k0 * (hf + 0.044715 * hf ** 3))
        return 0.5 * (1 + t) + 0.5 * hf * (1 - t * t) * k0 * (1 + 3 * 0.044715 * hf * hf)
    cdf = 0.5 * (1 + torch.erf(hf * 0.7071067811865476))
    pdf = torch.exp(-0.5 * hf * hf) * 0.3989422804014327
    return cdf + hf * pdf


def _native(h: torch.Tensor) -> bool:
    n = h.shape[-1]
    return (h.is_cuda and h.dtype in (torch.bfloat16, torch.float16) and n % 8 == 0 and (n // 8) % 64 == 0
            and n // 8 <= 1024 and h.numel() > 0)


def gelu_bwd_bias(dy: torch.Tensor, h: torch.Tensor, bias_dtype=torch.float32, bias_param=None):
    """``(dh, db)``: ``dh = dy * gelu'(h)`` (the selected form), ``db = dh.sum(rows)`` in ``bias_dtype``
    (written into ``bias_param``'s DDP bucket slice when one is attached, ``ops/graddst.py``)."""
    if not _native(h):
        dh = (dy.float() * _gelu_grad_ref(h.float())).to(h.dtype)
        return dh, dh.float().reshape(-1, h.shape[-1]).sum(0).to(bias_dtype)
    C = _ext.get(required=True)
    _sync(C)
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
    from . import graddst
    with graddst.into(bias_param):
        db = graddst.empty((n,), out_dt, h.device)
    C.gemm_splitk_reduce(part.data_ptr(), blocks, n, db.data_ptr(), DTYPE_CODE[out_dt], stream)
    return dh, db.to(bias_dtype)


class GeluLink:
    """Hand-off between ``linear_gelu`` (fc1 + GELU) and the Linear that consumes its output
    (fc2, inside ``linear_add_layer_norm``): the consumer's input-gradient GEMM applies the
    GELU derivative and reduces fc1's bias gradient in its epilogue (gemm_nt.hip EPI 2) and
    deposits ``(dh, db)`` here; fc1's backward then skips its own GELU pass. The gradient
    autograd passes between the two nodes is a zero-stride placeholder (never read). ``h``: what
    fc1's forward saved — ``gelu'(pre-activation)`` when its GEMM epilogue produced it
    (``deriv`` True, gemm_nt.hip EPI 1; the only form the consumer's EPI 2 takes), else the
    pre-activation. ``bias``: fc1's bias parameter (its gradient's DDP bucket slice,
    ``ops/graddst.py``)."""

    __slots__ = ("h", "deriv", "bias_dtype", "bias", "dh", "db")

    def __init__(self):
        self.h = self.bias_dtype = self.bias = self.dh = self.db = None
        self.deriv = False

    def take(self):
        out = (self.dh, self.db)
        self.h = self.bias = self.dh = self.db = None
        return out


class _LinearGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, link=None):
        from . import gemm_nt
        _sync(_ext.get(required=True))  # the backward kernels (gelu.hip, gemm_nt EPI 2) read the form
        n_out, n_in = weight.shape
        rows = x.numel() // n_in
        deriv = x.is_contiguous() and gemm_nt.supported(rows, n_out, n_in, x, weight, fused="fwd")
        if deriv:
            # bias + GELU in the GEMM epilogue: gelu(h) and gelu'(h) from the same registers; the
            # derivative (not h) is what the backward needs, so it is what is saved
            d2, g2 = gemm_nt.linear_fwd(x.view(rows, n_in), weight, bias, gelu=True)
            h, g = d2.view(*x.shape[:-1], n_out), g2.view(*x.shape[:-1], n_out)
        else:
            h = F.linear(x, weight, bias)
            g = _gelu_fwd(h)
        ctx.save_for_backward(x, weight, h)
        ctx.deriv = deriv
        ctx.weight = weight  # the leaf itself: its gradient's bucket slice (ops/graddst.py)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.bias = bias  # the leaf: its gradient's bucket slice
        ctx.link = link
        if link is not None:
            link.h, link.deriv, link.bias_dtype, link.bias = h, deriv, ctx.bias_dtype or torch.float32, bias
        return g

    @staticmethod
    def backward(ctx, dy):
        x, w, h = ctx.saved_tensors
        dh, db = ctx.link.take() if ctx.link is not None else (None, None)
        if dh is None and ctx.deriv:  # unfused consumer, saved derivative: dh = dy * gelu'(h)
            dh = (dy.float() * h.float()).to(h.dtype)
            db = None
            if ctx.has_bias and ctx.needs_input_grad[2]:
                from . import graddst
                from .linear import bias_grad
                with graddst.into(ctx.bias):
                    db = bias_grad(dh.reshape(-1, h.shape[-1]), ctx.bias_dtype)
        elif dh is None:  # the consumer did not fuse the GELU derivative: own pass
            dh, db = gelu_bwd_bias(dy, h, ctx.bias_dtype or torch.float32, bias_param=ctx.bias)
        else:
            dh = dh.view(h.shape)
        n = h.shape[-1]
        dh2 = dh.reshape(-1, n)
        x2 = x.reshape(-1, x.shape[-1])
        from .linear import _wgrad_mode, dgrad, dgrad_wgrad, linbwd_ok, native_ok, weight_grad
        dx = dw = None
        if (ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and _wgrad_mode() == "ours" and native_ok(x2, dh2)
                and linbwd_ok(dh2, x2, w)):
            # input and weight gradient in one launch (linbwd.hip)
            from . import graddst
            with graddst.into(ctx.weight):
                dx, dw = dgrad_wgrad(dh2, x2, w, w.dtype)
            dx = dx.reshape(x.shape)
        elif ctx.needs_input_grad[0]:
            dx = dgrad(dh2, w).reshape(x.shape)
        if ctx.needs_input_grad[1] and dw is None:
            # long-K weight gradient on the split-K HIP kernel (ops/linear.py)
            from . import graddst
            with graddst.into(ctx.weight):  # the DDP bucket slice when one is attached
                if _wgrad_mode() == "ours" and native_ok(x2, dh2):
                    dw = weight_grad(dh2, x2, w.dtype)
                elif dh2.dtype == x2.dtype == w.dtype:  # short K ([CLS]-only last block): hipBLASLt, into the slice
                    dw = torch.mm(dh2.t(), x2, out=graddst.empty(tuple(w.shape), w.dtype, dh2.device))
                else:
                    dw = (dh2.t() @ x2).to(w.dtype)
        return dx, dw, (db if ctx.has_bias and ctx.needs_input_grad[2] else None), None


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
                link: GeluLink | None = None) -> torch.Tensor:
    """``gelu(F.linear(x, weight, bias))`` (the selected GELU form) with the fused backward on
    the GPU. ``link``: pass the same :class:`GeluLink` to the consuming ``linear_add_layer_norm``."""
    if x.is_cuda and _native_width(weight.shape[0], x.dtype):
        return _LinearGeluFn.apply(x, weight, bias, link)
    return gelu(F.linear(x, weight, bias))


def _native_width(n: int, dtype) -> bool:
    return dtype in (torch.bfloat16, torch.float16) and n % 8 == 0 and (n // 8) % 64 == 0 and n // 8 <= 1024
