"""A small-channel 3x3 convolution whose filter gradient is born in its DDP bucket slice.

The CIFAR DEQ's stem takes the 3-channel image (``models/deq.py: DEQCifar.stem1``): below the
implicit-GEMM kernels' channel granularity, so the forward and the input gradient stay on MIOpen.
MIOpen's weight gradient returns a tensor of its own, which the DDP bucket pack then copies
(10 pack copies per DEQ-CIFAR step, the stems among them). Here the filter gradient
is ONE GEMM ``dW[co, (kh, kw, ci)] = dy^T @ im2col(x)`` (NHWC im2col in the filter's
channels_last memory order, hipBLASLt accumulating in fp32) written with ``out=`` straight into the
filter's bucket slice (``ops/graddst.py``) — no copy anywhere.

Reference context: /root/reference/src/optimizer.jl:45-65 reduces every gradient leaf where it
lies; here every leaf is produced where it is reduced.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import graddst


def _im2col_nhwc(x: torch.Tensor, stride: int, pad: int) -> tuple[torch.Tensor, int, int]:
    """``[N * Ho * Wo, 9 * C]`` rows of the 3x3 windows of the NHWC image ``x`` (an NCHW tensor in
    channels_last memory), columns in (kh, kw, ci) order."""
    n, c, h, w = x.shape
    xp = F.pad(x.permute(0, 2, 3, 1), (0, 0, pad, pad, pad, pad))  # [N, H+2p, W+2p, C]
    ho, wo = (h + 2 * pad - 3) // stride + 1, (w + 2 * pad - 3) // stride + 1
    sn, sh, sw, sc = xp.stride()
    win = xp.as_strided((n, ho, wo, 3, 3, c), (sn, sh * stride, sw * stride, sh, sw, sc))
    return win.reshape(n * ho * wo, 9 * c), ho, wo


class _SmallConv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, pad):
        ctx.save_for_backward(x, weight)
        ctx.cfg = (stride, pad)
        return F.conv2d(x, weight, None, stride, pad)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, pad = ctx.cfg
        dx = dw = None
        if ctx.needs_input_grad[1]:
            co, ci = weight.shape[0], weight.shape[1]
            cols, _, _ = _im2col_nhwc(x.contiguous(memory_format=torch.channels_last), stride, pad)
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, co)  # a view for a channels_last dy
            flat = graddst.take(weight, (weight.numel(),), weight.dtype)
            if flat is None:
                flat = torch.empty(weight.numel(), dtype=weight.dtype, device=weight.device)
            torch.mm(dy2.t(), cols, out=flat.view(co, 9 * ci))
            dw = flat.view(co, 3, 3, ci).permute(0, 3, 1, 2)  # channels_last strides over (co, kh, kw, ci)
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(dy, x, weight, None, [stride] * 2, [pad] * 2, [1, 1], False,
                                                     [0, 0], 1, [True, False, False])[0]
        return dx, dw, None, None


def supported(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    return (x.dim() == 4 and conv.kernel_size == (3, 3) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.bias is None and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
            and x.dtype == conv.weight.dtype)


def conv3x3_small(x: torch.Tensor, conv: torch.nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` (3x3, no bias) with the filter gradient delivered into its DDP bucket slice."""
    if not supported(x, conv):
        return conv(x)
    return _SmallConv3x3.apply(x, conv.weight, conv.stride[0], conv.padding[0])


__all__ = ["conv3x3_small", "supported"]
