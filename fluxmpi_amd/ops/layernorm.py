"""Fused LayerNorm (+ residual add) for transformer blocks (``csrc/kernels/layernorm.hip``).

``FusedLayerNorm`` is an ``nn.LayerNorm`` (same parameters / state dict) whose GPU path
runs one wavefront per row with the row held in registers. Its ``add_forward(x, r)``
returns ``(h, ln(h))`` with ``h = x + r`` — the residual add of a pre-LN block fused into
the normalisation pass — and the backward adds the gradient ``h`` receives from the
rest of the residual stream in the same pass, so a ViT block has no separate residual
add kernels in either direction. dw/db are reduced from per-workgroup partials (no
atomics). CPU tensors (and unsupported shapes) use the PyTorch composition.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext
from . import graddst
from .multi_tensor import DTYPE_CODE

_MAX_BLOCKS = 4096


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t):
    return t.data_ptr() if t is not None else 0


def supported(x: torch.Tensor) -> bool:
    d = x.shape[-1]
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and d % 8 == 0
            and 8 <= d <= 8192 and x.numel() > 0)


_AFFINE: dict = {}


def _const(d: int, device, value: float) -> torch.Tensor:
    """Cached fp32 ones / zeros standing in for an absent LayerNorm weight / bias (the kernels
    load the affine unconditionally)."""
    key = (d, str(device), value)
    t = _AFFINE.get(key)
    if t is None:
        t = torch.full((d,), value, device=device, dtype=torch.float32)
        _AFFINE[key] = t
    return t


def _zero(device, dtype) -> torch.Tensor:
    """A cached 0-d zero (expanded into the never-read placeholder gradient of a linked GELU output:
    a fresh ``torch.zeros(())`` launched one fill kernel per block per step)."""
    key = ("zero", str(device), dtype)
    t = _AFFINE.get(key)
    if t is None:
        t = torch.zeros((), device=device, dtype=dtype)
        _AFFINE[key] = t
    return t


def _affine(x, weight, bias):
    """The (w, b) the kernels read: the parameters themselves when both are present in the
    activation dtype (the kernels convert on load), else fp32 copies / cached ones-zeros."""
    if (weight is not None and bias is not None and weight.dtype == x.dtype == bias.dtype
            and weight.is_contiguous() and bias.is_contiguous()
            and (weight.data_ptr() | bias.data_ptr()) % 16 == 0):
        return weight, bias
    d = x.shape[-1]
    w32 = weight.float().contiguous() if weight is not None else _const(d, x.device, 1.0)
    b32 = bias.float().contiguous() if bias is not None else _const(d, x.device, 0.0)
    return w32, b32


def _fwd(x, r, w, b, eps):
    C = _ext.get(required=True)
    d = x.shape[-1]
    rows = x.numel() // d
    y = torch.empty_like(x)
    h = torch.empty_like(x) if r is not None else None
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    C.layernorm_fwd(x.data_ptr(), _p(r), _p(h), y.data_ptr(), w.data_ptr(), b.data_ptr(), mean.data_ptr(),
                    rstd.data_ptr(), rows, d, float(eps), DTYPE_CODE[x.dtype], DTYPE_CODE[w.dtype], _stream(x))
    return h, y, mean, rstd


def _bwd(dy, x, dh_ext, mean, rstd, w, dtypes, colsum_dtype=None, params=(None, None, None)):
    """``(dx, dw, db)``; dw / db reduced straight into the parameter dtype when it is fp32 or bf16
    and both share it (no cast kernels), else reduced in fp32 and cast. ``colsum_dtype`` (needs
    ``dh_ext``): also the column sums of dx, returned fourth in that dtype. ``params``: the leaves
    (LN weight, LN bias, the producer's bias for the column sums) whose DDP bucket slices the
    one reduce launch writes when a communicating engine is attached (``ops/graddst.py``)."""
    C = _ext.get(required=True)
    d = x.shape[-1]
    rows = x.numel() // d
    dx = torch.empty_like(x)
    cs = colsum_dtype is not None
    npart = 3 if cs else 2
    part = torch.empty(_MAX_BLOCKS, npart * d, device=x.device, dtype=torch.float32)
    nb = C.layernorm_bwd(dy.data_ptr(), x.data_ptr(), _p(dh_ext), mean.data_ptr(), rstd.data_ptr(), w.data_ptr(),
                         dx.data_ptr(), part.data_ptr(), _MAX_BLOCKS, rows, d, DTYPE_CODE[x.dtype],
                         DTYPE_CODE[w.dtype], _stream(x), cs)
    wd, bd = dtypes
    want = [wd, bd] + ([colsum_dtype] if cs else [])
    if not cs and wd is None and bd is None:
        return dx, None, None
    present = {t for t in want if t is not None}
    rdt = present.pop() if len(present) == 1 else torch.float32
    if rdt not in (torch.float32, torch.bfloat16):
        rdt = torch.float32
    # one reduce launch; each d-column segment lands in its own tensor (a bucket slice when the
    # dtype matches the parameter's, else a piece cast afterwards)
    outs = []
    for dt, p in zip(want, params):
        t = graddst.take(p, (d,), rdt) if (dt == rdt and p is not None) else None
        outs.append(t if t is not None else torch.empty(d, device=x.device, dtype=rdt))
    ptrs = [o.data_ptr() for o in outs] + [0] * (3 - len(outs))
    C.gemm_splitk_reduce_seg(part.data_ptr(), nb, npart * d, d, ptrs[0], ptrs[1], ptrs[2], DTYPE_CODE[rdt], _stream(x))
    dw = outs[0].to(wd) if wd is not None else None
    db = outs[1].to(bd) if bd is not None else None
    if cs:
        return dx, dw, db, outs[2].to(colsum_dtype)
    return dx, dw, db


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x = x.contiguous()
        w, b = _affine(x, weight, bias)
        _, y, mean, rstd = _fwd(x, None, w, b, eps)
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.dtypes = (weight.dtype if weight is not None else None, bias.dtype if bias is not None else None)
        ctx.params = (weight if ctx.needs_input_grad[1] else None, bias if ctx.needs_input_grad[2] else None, None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = _bwd(dy.contiguous(), x, None, mean, rstd, w, ctx.dtypes, params=ctx.params)
        return dx, dw, db, None


class _AddLayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, weight, bias, eps):
        x, r = x.contiguous(), r.contiguous()
        w, b = _affine(x, weight, bias)
        h, y, mean, rstd = _fwd(x, r, w, b, eps)
        ctx.save_for_backward(h, w, mean, rstd)
        ctx.dtypes = (weight.dtype if weight is not None else None, bias.dtype if bias is not None else None)
        ctx.params = (weight if ctx.needs_input_grad[2] else None, bias if ctx.needs_input_grad[3] else None, None)
        return h, y

    @staticmethod
    def backward(ctx, dh, dy):
        h, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(h)
        dh = dh.contiguous() if dh is not None else None
        dx, dw, db = _bwd(dy.contiguous(), h, dh, mean, rstd, w, ctx.dtypes, params=ctx.params)
        return dx, dx, dw, db, None  # h = x + r: both inputs get the same gradient


class _LinearAddLayerNormFn(torch.autograd.Function):
    """``(h, LN(h))`` with ``h = x + a W^T + b``: a pre-LN block's output projection and the next
    LayerNorm's residual add. The LayerNorm backward's dx IS the projection output's gradient,
    so its column sums (the projection's bias gradient) come out of the same pass — no colsum
    kernel over dx; the weight gradient runs on the split-K HIP kernel (ops/linear.py)."""

    @staticmethod
    def forward(ctx, a, weight, bias, x, ln_w, ln_b, eps, gelu_link=None):
        from .linear import fwd
        p = fwd(a, weight, bias)
        ctx.gelu_link = gelu_link
        x = x.contiguous()
        w, b = _affine(x, ln_w, ln_b)
        h, y, mean, rstd = _fwd(x, p.contiguous(), w, b, eps)
        ctx.save_for_backward(a, weight, h, w, mean, rstd)
        ctx.weight = weight  # the leaf itself: its gradient's bucket slice (ops/graddst.py)
        ctx.dtypes = (ln_w.dtype if ln_w is not None else None, ln_b.dtype if ln_b is not None else None)
        ctx.bias_dtype = bias.dtype
        need = ctx.needs_input_grad
        ctx.params = (ln_w if need[4] else None, ln_b if need[5] else None, bias if need[2] else None)
        return h, y

    @staticmethod
    def backward(ctx, dh, dy):
        from .linear import native_ok, weight_grad
        a, weight, h, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(h)
        if dh is None:
            dh = torch.zeros_like(h)
        dx, dlw, dlb, dbias = _bwd(dy.contiguous(), h, dh.contiguous(), mean, rstd, w, ctx.dtypes, ctx.bias_dtype,
                                   params=ctx.params)
        n_out, n_in = weight.shape
        g2 = dx.reshape(-1, n_out)
        a2 = a.reshape(-1, n_in)
        da = dw = None
        if ctx.needs_input_grad[0]:
            from . import gemm_nt
            from .linear import dgrad, dgrad_wgrad, linbwd_ok
            link = ctx.gelu_link
            if (link is not None and link.h is not None and link.deriv and link.h.shape == a.shape
                    and gemm_nt.supported(g2.shape[0], n_in, n_out, g2, weight, link.h, fused="dgrad")):
                # `a` = gelu(h) of the linear_gelu node upstream: its GELU derivative and its bias
                # gradient come out of this input-gradient GEMM's epilogue (gemm_nt.hip EPI 2)
                link.dh, link.db = gemm_nt.linear_dgrad(g2, weight, gelu_d=link.h, bias_dtype=link.bias_dtype,
                                                        bias_param=link.bias)
                da = _zero(a.device, a.dtype).expand(a.shape)  # placeholder, never read
            elif ctx.needs_input_grad[1] and native_ok(a2, g2) and linbwd_ok(g2, a2, weight):
                # input and weight gradient in one launch (linbwd.hip)
                with graddst.into(ctx.weight):
                    da, dw = dgrad_wgrad(g2, a2, weight, weight.dtype)
                da = da.reshape(a.shape)
            else:
                da = dgrad(g2, weight).reshape(a.shape)
        if ctx.needs_input_grad[1] and dw is None:
            with graddst.into(ctx.weight):  # the DDP bucket slice when one is attached
                if native_ok(a2, g2):
                    dw = weight_grad(g2, a2, weight.dtype)
                elif g2.dtype == a2.dtype == weight.dtype:  # short K ([CLS]-only last block): into the slice
                    dw = torch.mm(g2.t(), a2, out=graddst.empty(tuple(weight.shape), weight.dtype, g2.device))
                else:
                    dw = (g2.t() @ a2).to(weight.dtype)
        return da, dw, (dbias if ctx.needs_input_grad[2] else None), dx, dlw, dlb, None, None


def linear_add_layer_norm(a, weight, bias, x, ln_w, ln_b, eps=1e-5, gelu_link=None):
    """``(h, layer_norm(h))`` with ``h = x + F.linear(a, weight, bias)`` (see
    :class:`_LinearAddLayerNormFn`); the PyTorch composition off the fused path. ``gelu_link``
    (:class:`ops.gelu.GeluLink`): ``a`` is ``linear_gelu(..., link=gelu_link)``'s output, whose
    GELU backward this node's input-gradient GEMM then performs."""
    if (supported(x) and bias is not None and a.is_contiguous() and a.shape[:-1] == x.shape[:-1]
            and weight.shape[0] == x.shape[-1] and a.dtype == x.dtype == weight.dtype and torch.is_grad_enabled()
            and (ln_w is None or ln_w.shape[-1] == x.shape[-1])):
        return _LinearAddLayerNormFn.apply(a, weight, bias, x, ln_w, ln_b, eps, gelu_link)
    from .linear import linear
    return add_layer_norm(x, linear(a, weight, bias), ln_w, ln_b, eps)


def layer_norm(x, weight, bias, eps=1e-5):
    if supported(x) and (weight is None or weight.shape[-1] == x.shape[-1]):
        return _LayerNormFn.apply(x, weight, bias, eps)
    return F.layer_norm(x, x.shape[-1:], weight, bias, eps)


def add_layer_norm(x, r, weight, bias, eps=1e-5):
    """``(h, layer_norm(h))`` with ``h = x + r``."""
    if supported(x) and x.shape == r.shape and x.dtype == r.dtype:
        return _AddLayerNormFn.apply(x, r, weight, bias, eps)
    h = x + r
    return h, F.layer_norm(h, h.shape[-1:], weight, bias, eps)


class FusedLayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` over the last dimension with the fused HIP kernels on the GPU."""

    def forward(self, x):
        if len(self.normalized_shape) != 1:
            return super().forward(x)
        return layer_norm(x, self.weight, self.bias, self.eps)

    def add_forward(self, x, r):
        return add_layer_norm(x, r, self.weight, self.bias, self.eps)


__all__ = ["FusedLayerNorm", "layer_norm", "add_layer_norm", "linear_add_layer_norm"]
