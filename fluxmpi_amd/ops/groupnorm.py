"""Fused NHWC GroupNorm (+ residual add, + ReLU on its input) (``csrc/kernels/groupnorm.hip``).

``FusedGroupNorm`` is an ``nn.GroupNorm`` (same parameters / state dict) whose
``forward(x, add=None, relu=False)`` computes ``GN(relu(x + add))``. On channels_last GPU
tensors one workgroup per sample does statistics and apply (no NCHW layout copies, no
separate add / ReLU kernels) and the backward writes the gradient of the GroupNorm input
(times the ReLU mask) once — it is the gradient of both ``x`` and ``add``. Other tensors
use the PyTorch composition, which is also the test oracle.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext
from . import graddst
from .multi_tensor import DTYPE_CODE


_SKIP_PARAM_GRADS = False


class skip_param_grads:
    """Within this context the GroupNorm backward returns no weight / bias gradients.

    For vector-Jacobian products taken w.r.t. activations only (the DEQ adjoint solve:
    ``autograd.grad(f(z), z, u)``), where ``ctx.needs_input_grad`` still reports the
    parameters and their (discarded) reductions would run every iteration."""

    def __enter__(self):
        global _SKIP_PARAM_GRADS
        self._prev, _SKIP_PARAM_GRADS = _SKIP_PARAM_GRADS, True

    def __exit__(self, *exc):
        global _SKIP_PARAM_GRADS
        _SKIP_PARAM_GRADS = self._prev


_AFFINE32: dict = {}


class fp32_affine_cache:
    """Within this context the fused GroupNorms of ``module`` read fp32 copies of their
    low-precision (bf16) weight / bias made ONCE at entry, instead of casting them on every call.

    The DEQ solver calls its cell ~30 times per forward with unchanged parameters: two cast
    kernels per GroupNorm per call were ~190 launches per step. The copies are only valid while
    the parameters do not change, i.e. within one forward pass.

    ``buffers`` (a dict the caller keeps): the copies are written into the same fp32 tensors on
    every entry instead of fresh ones, so a HIP graph captured inside the context keeps reading
    the current values (models/deq.py's solver graphs)."""

    def __init__(self, module: nn.Module, buffers: dict | None = None):
        self.module = module
        self.buffers = buffers

    def __enter__(self):
        global _AFFINE32
        cache = dict(_AFFINE32)
        for mod in self.module.modules():
            if isinstance(mod, FusedGroupNorm):
                for p in (mod.weight, mod.bias):
                    if p is not None and p.dtype != torch.float32:
                        if self.buffers is None:
                            cache[id(p)] = (p, p.detach().float().contiguous())
                            continue
                        buf = self.buffers.get(id(p))
                        if buf is None or buf[0] is not p:
                            buf = self.buffers[id(p)] = (p, torch.empty(p.shape, device=p.device,
                                                                         dtype=torch.float32))
                        buf[1].copy_(p.detach())
                        cache[id(p)] = buf
        self._prev, _AFFINE32 = _AFFINE32, cache
        return self

    def __exit__(self, *exc):
        global _AFFINE32
        _AFFINE32 = self._prev


def _f32(p):
    if p is None:
        return None
    hit = _AFFINE32.get(id(p))
    if hit is not None and hit[0] is p:
        return hit[1]
    return p.float().contiguous()


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def supported(x: torch.Tensor, groups: int) -> bool:
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16, torch.float32)):
        return False
    C = x.shape[1]
    return (C % 8 == 0 and C <= 2048 and C % groups == 0 and groups <= 64 and x.numel() > 0
            and x.is_contiguous(memory_format=torch.channels_last))


def gn_fwd_raw(x, add, weight, bias, groups, eps, relu, out=None):
    """``GN(relu(x + add))`` on the fused kernel, no autograd: returns ``(y, saved, mean, rstd, w32)``
    where ``saved`` is what the backward reads (the GroupNorm input ``relu(x + add)``, or ``x``).
    ``out`` ([N, H*W*C] rows of x's dtype, any row stride, e.g. an Anderson history slot): y is
    written there (and returned as that tensor)."""
    C = _ext.get(required=True)
    N, Ch, H, W = x.shape
    if add is not None:
        add = add.contiguous(memory_format=torch.channels_last)
    w32, b32 = _f32(weight), _f32(bias)
    if out is not None:
        assert out.dtype == x.dtype and out.shape == (N, Ch * H * W) and out.stride(1) == 1
        y, ys = out, out.stride(0)
    else:
        y, ys = torch.empty_like(x, memory_format=torch.channels_last), 0
    h = torch.empty_like(y) if (add is not None or relu) else None
    mean = torch.empty(N, groups, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    C.groupnorm_nhwc_fwd(x.data_ptr(), add.data_ptr() if add is not None else 0, h.data_ptr() if h is not None else 0,
                         y.data_ptr(), w32.data_ptr() if w32 is not None else 0,
                         b32.data_ptr() if b32 is not None else 0, mean.data_ptr(), rstd.data_ptr(), N, H * W, Ch,
                         groups, bool(relu), float(eps), DTYPE_CODE[x.dtype], _stream(x), ys)
    return y, (h if h is not None else x), mean, rstd, w32


def gn_bwd_raw(dy, h, mean, rstd, w32, groups, relu, part=None):
    """Gradient of the GroupNorm input (times the ReLU mask) from the saved state of
    :func:`gn_fwd_raw`; ``part`` ([N, 2, C] fp32) receives the per-sample weight / bias sums."""
    C = _ext.get(required=True)
    N, Ch, H, W = h.shape
    dy = dy.contiguous(memory_format=torch.channels_last)
    dh = torch.empty_like(h, memory_format=torch.channels_last)
    if part is None:
        part = torch.empty(N, 2, Ch, device=h.device, dtype=torch.float32)
    C.groupnorm_nhwc_bwd(dy.data_ptr(), h.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                         w32.data_ptr() if w32 is not None else 0, dh.data_ptr(), part.data_ptr(), N, H * W, Ch,
                         groups, relu, DTYPE_CODE[h.dtype], _stream(h))
    return dh, part


class _GroupNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, add, weight, bias, groups, eps, relu, link=None):
        y, saved, mean, rstd, w32 = gn_fwd_raw(x, add, weight, bias, groups, eps, relu)
        ctx.save_for_backward(saved, mean, rstd, w32)
        ctx.cfg = (groups, bool(relu), add is not None,
                   weight.dtype if weight is not None else None, bias.dtype if bias is not None else None)
        ctx.params = (weight, bias)  # the leaves: their gradients' DDP bucket slices (graddst)
        ctx.link = link
        return y

    @staticmethod
    def backward(ctx, dy):
        h, mean, rstd, w32 = ctx.saved_tensors
        groups, relu, has_add, wd, bd = ctx.cfg
        dh, part = gn_bwd_raw(dy, h, mean, rstd, w32, groups, relu)
        want = not _SKIP_PARAM_GRADS
        # the per-sample sums reduced and cast straight into the parameters' DDP bucket slices
        wp, bp = ctx.params
        dw = graddst.deliver(wp, part[:, 0].sum(0), wd) if want and wd is not None and ctx.needs_input_grad[2] else None
        db = graddst.deliver(bp, part[:, 1].sum(0), bd) if want and bd is not None and ctx.needs_input_grad[3] else None
        dx = dh
        if ctx.link is not None and ctx.needs_input_grad[0]:
            # x's other consumer (a convolution holding the same link) adds dh in its dgrad epilogue
            ctx.link.grad = dh
            dx = None
        return dx, (dh if has_add else None), dw, db, None, None, None, None


def native_ok(x, groups, add=None) -> bool:
    """This call takes the fused kernels (and so honours a ``link``)."""
    return supported(x, groups) and (add is None or (add.shape == x.shape and add.dtype == x.dtype))


def group_norm(x, groups, weight=None, bias=None, eps=1e-5, add=None, relu=False, link=None):
    """``F.group_norm(relu(x + add), groups, weight, bias, eps)`` with the add / ReLU optional.

    ``link`` (:class:`~fluxmpi_amd.ops.batchnorm.GradLink`, fused path only — check
    :func:`native_ok`): x's gradient is deposited there for x's other consumer instead of being
    returned to autograd (which would add the two gradients with a separate kernel)."""
    if native_ok(x, groups, add):
        return _GroupNormFn.apply(x, add, weight, bias, groups, eps, relu, link)
    assert link is None, "group_norm: a GradLink needs the fused path (native_ok)"
    h = x + add if add is not None else x
    if relu:
        h = F.relu(h)
    return F.group_norm(h, groups, weight, bias, eps)


class FusedGroupNorm(nn.GroupNorm):
    def forward(self, x, add=None, relu=False, link=None):  # noqa: D102
        return group_norm(x, self.num_groups, self.weight, self.bias, self.eps, add, relu, link)
