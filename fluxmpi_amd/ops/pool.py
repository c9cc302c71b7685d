"""Fused ResNet stem tail: BatchNorm (batch statistics) + ReLU + max-pool, NHWC.

``bn_relu_maxpool(x, bn, k=3, s=2, p=1)`` == ``max_pool2d(relu(bn(x)), k, s, p)`` in
training mode, with the normalised full-resolution activation never written:
one statistics pass over the conv output, then one kernel that normalises,
rectifies and pools (``csrc/kernels/pool.hip``) and records a 1-byte window
index per pooled element. The backward gathers the pooled gradient back to full
resolution (no zero fill, no atomics) and runs the fused BatchNorm backward.

Compared with conv -> BN -> ReLU -> MaxPool2d this removes a write and a read of
the 112x112x64 activation and the pool's int64 index tensor (8 B per pooled
element vs 1 B here).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from .batchnorm import _workspace
from .fused_block import _bn_bwd, _empty_nhwc, _p, _stream
from .multi_tensor import DTYPE_CODE


def _out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


class _BNReluMaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, k, s, p, nbt=None):
        C = _ext.get(required=True)
        if not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        n, ch, h, w = x.shape
        rows = n * h * w
        w32 = weight.float() if weight is not None else torch.ones(ch, device=x.device)
        b32 = bias.float() if bias is not None else torch.zeros(ch, device=x.device)
        mean = torch.empty(ch, device=x.device, dtype=torch.float32)
        inv, scale, shift = torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean)
        ws = _workspace(x)
        C.bn_stats_finalize(x.data_ptr(), w32.data_ptr(), b32.data_ptr(), _p(running_mean), _p(running_var),
                            mean.data_ptr(), inv.data_ptr(), scale.data_ptr(), shift.data_ptr(), ws.data_ptr(), rows,
                            ch, float(momentum), float(eps), 0, DTYPE_CODE[x.dtype], _stream(x), _p(nbt))
        oh, ow = _out(h, k, s, p), _out(w, k, s, p)
        y = _empty_nhwc(n, ch, oh, ow, x)
        idx = torch.empty(n * oh * ow * ch, device=x.device, dtype=torch.uint8)
        C.bn_relu_maxpool_fwd(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), y.data_ptr(), idx.data_ptr(), n, h, w,
                              ch, k, s, p, DTYPE_CODE[x.dtype], _stream(x))
        ctx.geo = (k, s, p)
        ctx.wdtype = weight.dtype if weight is not None else None
        ctx.has_affine = (weight is not None, bias is not None)
        ctx.save_for_backward(x, idx, w32, b32, mean, inv)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.get(required=True)
        x, idx, w32, b32, mean, inv = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        n, ch, h, w = x.shape
        k, s, p = ctx.geo
        dz = torch.empty_like(x)  # gradient of the pre-ReLU normalised activation
        C.maxpool_bwd(dy.data_ptr(), idx.data_ptr(), dz.data_ptr(), n, h, w, ch, k, s, p, DTYPE_CODE[x.dtype],
                      _stream(x))
        dx, _, dw, db = _bn_bwd(dz, x, None, w32, b32, mean, inv, False, False)
        has_w, has_b = ctx.has_affine
        return (dx, dw.to(ctx.wdtype) if has_w else None, db.to(ctx.wdtype) if has_b else None,
                None, None, None, None, None, None, None, None)


def pad_c3_to_c4(x: torch.Tensor) -> torch.Tensor:
    """NHWC ``[N, H, W, 3]`` -> ``[N, H, W, 4]`` with a zero 4th channel (16-bit dtypes), one HIP
    pass (``csrc/kernels/pool.hip``); returned as the NCHW-shaped channels_last view."""
    C = _ext.get(required=True)
    n, c, h, w = x.shape
    xp = x.permute(0, 2, 3, 1)
    if c != 3 or not xp.is_contiguous() or x.dtype not in (torch.bfloat16, torch.float16):
        raise ValueError("pad_c3_to_c4: needs a channels_last bf16/fp16 [N, 3, H, W] tensor")
    y = torch.empty(n, h, w, 4, device=x.device, dtype=x.dtype)
    C.pad_c3_to_c4(xp.data_ptr(), y.data_ptr(), n * h * w, DTYPE_CODE[x.dtype], _stream(x))
    return y.permute(0, 3, 1, 2)


def supported(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.shape[1] % 8 == 0 and 8 <= x.shape[1] <= 2048)


def bn_relu_maxpool(x: torch.Tensor, bn, k: int = 3, s: int = 2, p: int = 1) -> torch.Tensor:
    """``max_pool2d(relu(bn(x)), k, s, p)`` for a training-mode BatchNorm module ``bn``."""
    from .batchnorm import bn_counter
    mom, nbt = bn_counter(bn)
    if not (bn.training and supported(x)):
        if nbt is not None:
            nbt.add_(1)
        y = F.batch_norm(x.float(), bn.running_mean, bn.running_var,
                         bn.weight.float() if bn.weight is not None else None,
                         bn.bias.float() if bn.bias is not None else None,
                         bn.training or not bn.track_running_stats, mom, bn.eps)
        return F.max_pool2d(F.relu(y), k, s, p).to(x.dtype)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return _BNReluMaxPool.apply(x, bn.weight, bn.bias, rm, rv, mom, bn.eps, k, s, p, nbt)


__all__ = ["bn_relu_maxpool", "pad_c3_to_c4"]
