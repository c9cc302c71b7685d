"""Fused multi-tensor optimiser steps (wrappers of ``csrc/kernels/optim.hip``).

Each function updates many (param, grad, state...) tuples in one launch per
dtype group. CPU tensors use the PyTorch reference math, which mirrors the
Optimisers.jl formulas term by term (and is the GPU kernels' test oracle).
"""
from __future__ import annotations

import torch

from . import _ext
from .multi_tensor import DTYPE_CODE

_SUPPORTED = {
    (torch.float32, torch.float32, torch.float32, False),
    (torch.float32, torch.bfloat16, torch.float32, False),  # fp32 parameters, bf16 gradients (mixed precision)
    (torch.bfloat16, torch.bfloat16, torch.bfloat16, False),
    (torch.bfloat16, torch.bfloat16, torch.float32, False),
    (torch.bfloat16, torch.bfloat16, torch.float32, True),
    (torch.bfloat16, torch.float32, torch.float32, True),
    (torch.float16, torch.float16, torch.float16, False),
    (torch.float16, torch.float16, torch.float32, False),
    (torch.float16, torch.float16, torch.float32, True),
    (torch.float16, torch.float32, torch.float32, True),
    (torch.float64, torch.float64, torch.float64, False),
}


def supported(p_dtype, g_dtype, s_dtype, master: bool) -> bool:
    return (p_dtype, g_dtype, s_dtype, master) in _SUPPORTED


def adam_(params, grads, exp_avgs, exp_avg_sqs, *, lr: float, beta1: float, beta2: float, eps: float,
          bc1: float, bc2: float, weight_decay: float = 0.0, grad_scale: float = 1.0, masters=None,
          dev_hyper: torch.Tensor | None = None, dev_gscale: torch.Tensor | None = None) -> None:
    """In-place fused Adam over lists of tensors.

    ``bc1``/``bc2`` are ``1 - beta^t`` (Optimisers.jl keeps ``beta^t`` in the
    state and starts it at ``beta``). ``dev_hyper`` (fp32 ``[lr, beta1^t,
    beta2^t]`` on device) overrides ``lr``/``bc1``/``bc2`` for HIP-graph replay.
    """
    if not params:
        return
    if params[0].is_cuda:
        C = _ext.get(required=True)
        stream = torch.cuda.current_stream(params[0].device).cuda_stream
        m_list = masters if masters is not None else None
        groups: dict = {}
        for i, p in enumerate(params):
            key = (p.dtype, grads[i].dtype, exp_avgs[i].dtype, m_list is not None)
            groups.setdefault(key, []).append(i)
        for (pd, gd, sd, hm), idx in groups.items():
            if not supported(pd, gd, sd, hm):
                raise TypeError(f"fused Adam: unsupported dtypes param={pd} grad={gd} state={sd} master={hm}")
            C.mt_adam([params[i].data_ptr() for i in idx], [grads[i].data_ptr() for i in idx],
                      [exp_avgs[i].data_ptr() for i in idx], [exp_avg_sqs[i].data_ptr() for i in idx],
                      [m_list[i].data_ptr() for i in idx] if hm else [],
                      [params[i].numel() for i in idx], DTYPE_CODE[pd], DTYPE_CODE[gd], DTYPE_CODE[sd],
                      float(lr), float(beta1), float(beta2), float(eps), float(bc1), float(bc2),
                      float(weight_decay), float(grad_scale),
                      dev_hyper.data_ptr() if dev_hyper is not None else 0,
                      dev_gscale.data_ptr() if dev_gscale is not None else 0, stream)
        return
    if dev_hyper is not None:
        h = dev_hyper.tolist()
        lr, bc1, bc2 = h[0], 1.0 - float(torch.tensor(h[1])), 1.0 - float(torch.tensor(h[2]))
    if dev_gscale is not None:
        grad_scale = grad_scale * float(dev_gscale)
    adam_reference_(params, grads, exp_avgs, exp_avg_sqs, lr=lr, beta1=beta1, beta2=beta2, eps=eps, bc1=bc1,
                    bc2=bc2, weight_decay=weight_decay, grad_scale=grad_scale, masters=masters)


def adam_reference_(params, grads, exp_avgs, exp_avg_sqs, *, lr, beta1, beta2, eps, bc1, bc2,
                    weight_decay=0.0, grad_scale=1.0, masters=None):
    """PyTorch reference of the fused kernel (compute in fp32, or fp64 for fp64 params)."""
    for i, p in enumerate(params):
        ct = torch.float64 if p.dtype == torch.float64 else torch.float32
        g = grads[i].to(ct) * grad_scale if grad_scale != 1.0 else grads[i].to(ct)
        m = exp_avgs[i].to(ct) * beta1 + (1 - beta1) * g
        v = exp_avg_sqs[i].to(ct) * beta2 + (1 - beta2) * (g * g)
        x = masters[i].to(ct) if masters is not None else p.to(ct)
        dx = m / bc1 / (torch.sqrt(v / bc2) + eps) * lr
        if weight_decay != 0.0:
            dx = dx + weight_decay * x
        x = x - dx
        exp_avgs[i].copy_(m)
        exp_avg_sqs[i].copy_(v)
        if masters is not None:
            masters[i].copy_(x)
        p.copy_(x)


def adam_advance_(dev_hyper: torch.Tensor, beta1: float, beta2: float) -> None:
    """``beta^t *= beta`` on the device hyper block (after the step's Adam launches)."""
    if dev_hyper.is_cuda:
        C = _ext.get(required=True)
        C.adam_advance(dev_hyper.data_ptr(), float(beta1), float(beta2),
                       torch.cuda.current_stream(dev_hyper.device).cuda_stream)
    else:
        dev_hyper[1] *= beta1
        dev_hyper[2] *= beta2


def sgd_(params, grads, bufs, *, lr: float, momentum: float = 0.0, nesterov: bool = False,
         weight_decay: float = 0.0, grad_scale: float = 1.0, masters=None,
         dev_lr: torch.Tensor | None = None) -> None:
    """Fused Descent / Momentum / Nesterov (Optimisers.jl semantics)."""
    if not params:
        return
    if params[0].is_cuda:
        C = _ext.get(required=True)
        stream = torch.cuda.current_stream(params[0].device).cuda_stream
        groups: dict = {}
        for i, p in enumerate(params):
            sd = bufs[i].dtype if (bufs is not None and momentum != 0.0) else p.dtype
            key = (p.dtype, grads[i].dtype, sd, masters is not None)
            groups.setdefault(key, []).append(i)
        for (pd, gd, sd, hm), idx in groups.items():
            if not supported(pd, gd, sd, hm):
                raise TypeError(f"fused SGD: unsupported dtypes param={pd} grad={gd} state={sd} master={hm}")
            C.mt_sgd([params[i].data_ptr() for i in idx], [grads[i].data_ptr() for i in idx],
                     [bufs[i].data_ptr() for i in idx] if momentum != 0.0 else [],
                     [masters[i].data_ptr() for i in idx] if hm else [],
                     [params[i].numel() for i in idx], DTYPE_CODE[pd], DTYPE_CODE[gd], DTYPE_CODE[sd],
                     float(lr), float(momentum), float(weight_decay), float(grad_scale), int(bool(nesterov)),
                     dev_lr.data_ptr() if dev_lr is not None else 0, stream)
        return
    if dev_lr is not None:
        lr = float(dev_lr.reshape(-1)[0])
    sgd_reference_(params, grads, bufs, lr=lr, momentum=momentum, nesterov=nesterov, weight_decay=weight_decay,
                   grad_scale=grad_scale, masters=masters)


def sgd_reference_(params, grads, bufs, *, lr, momentum=0.0, nesterov=False, weight_decay=0.0, grad_scale=1.0,
                   masters=None):
    for i, p in enumerate(params):
        ct = torch.float64 if p.dtype == torch.float64 else torch.float32
        x = masters[i].to(ct) if masters is not None else p.to(ct)
        g = grads[i].to(ct) * grad_scale
        if weight_decay:
            g = g + weight_decay * x
        if momentum == 0.0:
            dx = g * lr
        elif not nesterov:
            vel = momentum * bufs[i].to(ct) + lr * g
            bufs[i].copy_(vel)
            dx = vel
        else:
            vel0 = bufs[i].to(ct)
            dx = -(momentum * momentum) * vel0 + (1 + momentum) * lr * g
            bufs[i].copy_(momentum * vel0 - lr * g)
        x = x - dx
        if masters is not None:
            masters[i].copy_(x)
        p.copy_(x)


def bias_corrections(beta1_t: float, beta2_t: float) -> tuple[float, float]:
    return 1.0 - beta1_t, 1.0 - beta2_t


__all__ = ["adam_", "adam_reference_", "adam_advance_", "sgd_", "sgd_reference_", "supported", "bias_corrections"]
