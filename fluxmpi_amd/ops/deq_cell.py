"""The DEQ cell ``f(z, x) = GN3(relu(z + GN2(x + conv2(GN1(relu(conv1 z))))))`` and its adjoint VJP
as ONE kernel each (``csrc/kernels/deq_cell.hip``): one workgroup per sample with the sample's
activations and the 3x3 filter resident in LDS, the convolutions on MFMA tiles straight out of
the halo image, every GroupNorm reduction inside the workgroup.

The unfused path (``ResidualCell.forward_state`` / ``vjp`` on ``conv3x3_*_raw`` + ``gn_*_raw``)
is 5 launches and ~5 full-tensor HBM round trips per evaluation; the DEQ solver makes ~60 such
evaluations per training step. Same state format, same numerics (bf16 activations, fp32
statistics); the reference example this serves is the FastDEQ model of the reference README.

``ENABLED = False`` keeps the unfused path (A/B runs).
"""
from __future__ import annotations

import os

import torch

from . import _ext

ENABLED = True  # False: the unfused 5-launch cell (A/B, scripts/diag_deq_graphs.py)


def _ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _cl(t: torch.Tensor) -> bool:
    return t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)


def supported(cell, z: torch.Tensor) -> bool:
    """Whether the fused kernels take this cell at ``z``'s shape (bf16 channels_last, 48 channels,
    H*W a multiple of 16 that fits LDS, equal group counts and eps in the three GroupNorms)."""
    if not (ENABLED and z.is_cuda and z.dtype == torch.bfloat16 and _cl(z)):
        return False
    norms = (cell.n1, cell.n2, cell.n3)
    if len({n.num_groups for n in norms}) != 1 or len({float(n.eps) for n in norms}) != 1:
        return False
    for conv in (cell.conv1, cell.conv2):
        w = conv.weight
        if (w.dtype != torch.bfloat16 or w.shape[2:] != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1)
                or conv.bias is not None or conv.groups != 1 or w.shape[0] != w.shape[1]):
            return False
    C = _ext.get(required=False)
    if C is None or not hasattr(C, "deq_cell_fwd"):
        return False
    n, ch, h, wd = z.shape
    return bool(C.deq_cell_supported(h, wd, ch, cell.n1.num_groups))


def _filter_k(w: torch.Tensor) -> torch.Tensor:
    """[co][ci][3][3] -> [co][tap][ci] (a view for a channels_last filter, else one copy)."""
    return w.permute(0, 2, 3, 1).contiguous()


def cell_forward(cell, z: torch.Tensor, x: torch.Tensor, keep: bool = False, out32: torch.Tensor | None = None,
                 want_out: bool = True, out_slot: torch.Tensor | None = None):
    """``f(z, x)`` in one launch. ``keep``: also return the VJP state of ``ResidualCell.forward_state``
    (``(shape, (h1, mean1, rstd1, w1), (h2, ...), (h3, ...))``). ``out32`` ([N, H*W*C] fp32 rows,
    any row stride): the output is also written there in fp32 (an Anderson history slot).
    ``out_slot`` ([N, H*W*C] bf16 rows, any row stride): the bf16 output goes there instead of a
    fresh tensor (an Anderson bf16 history slot; returned)."""
    from .gemm import note_filter
    from .groupnorm import _f32
    C = _ext.get(required=True)
    n, ch, h, wd = z.shape
    G = cell.n1.num_groups
    if not _cl(x) or x.dtype != z.dtype or x.shape != z.shape:
        x = x.to(z.dtype).contiguous(memory_format=torch.channels_last)
    # as the unfused forward: the cached transposed filters are stale once the weights move
    note_filter(cell.conv1.weight)
    note_filter(cell.conv2.weight)
    w1, w2 = _filter_k(cell.conv1.weight), _filter_k(cell.conv2.weight)
    norms = (cell.n1, cell.n2, cell.n3)
    gw = [_f32(m.weight) for m in norms]
    gb = [_f32(m.bias) for m in norms]
    out_stride = 0
    if out_slot is not None:
        assert out_slot.dtype == torch.bfloat16 and out_slot.shape == (n, ch * h * wd) and out_slot.stride(1) == 1
        out, out_stride = out_slot, out_slot.stride(0)
    else:
        out = torch.empty_like(z, memory_format=torch.channels_last) if want_out or out32 is None else None
    hs = [torch.empty_like(z, memory_format=torch.channels_last) for _ in range(3)] if keep else [None] * 3
    st = [torch.empty(n, G, device=z.device, dtype=torch.float32) for _ in range(6)] if keep else [None] * 6
    if out32 is not None:
        assert out32.dtype == torch.float32 and out32.shape == (n, ch * h * wd) and out32.stride(1) == 1
    C.deq_cell_fwd(z.data_ptr(), x.data_ptr(), w1.data_ptr(), w2.data_ptr(), [_ptr(t) for t in gw],
                   [_ptr(t) for t in gb], _ptr(out), _ptr(out32), out32.stride(0) if out32 is not None else 0,
                   [_ptr(t) for t in hs], [_ptr(t) for t in st[0::2]], [_ptr(t) for t in st[1::2]],
                   n, h, wd, ch, G, float(cell.n1.eps), _stream(z), out_stride)
    if not keep:
        return out
    state = (tuple(z.shape), (hs[0], st[0], st[1], gw[0]), (hs[1], st[2], st[3], gw[1]), (hs[2], st[4], st[5], gw[2]))
    return out, state


def cell_vjp(cell, state, u: torch.Tensor, grad: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """``J_f(z)^T u`` in one launch from a ``forward_state`` state (fused or unfused producer).

    ``grad``: the adjoint iteration's update is fused in — returns ``(u_new, part)`` with
    ``u_new = bf16(J^T u + grad)`` and ``part[n]`` the per-sample ``sum (u_new - u)^2`` (sum them
    with :func:`adjoint_check`): one launch instead of the VJP + ``adjoint_step`` pair. ``out``
    (channels_last bf16 like ``u``, not ``u`` itself): written instead of a new tensor."""
    from .gemm import filter_t
    C = _ext.get(required=True)
    zs, (h1, m1, r1, w1), (h2, m2, r2, w2), (h3, m3, r3, w3) = state
    n, ch, h, wd = zs
    if not _cl(u) or u.dtype != torch.bfloat16:
        u = u.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    hs = [t if _cl(t) else t.contiguous(memory_format=torch.channels_last) for t in (h1, h2, h3)]
    G = cell.n1.num_groups
    if tuple(u.shape) != tuple(zs) or any(t.shape != u.shape or t.dtype != torch.bfloat16 for t in hs) or any(
            t.shape != (n, G) or t.dtype != torch.float32 for t in (m1, r1, m2, r2, m3, r3)):
        raise ValueError("deq_cell.cell_vjp: state does not match the gradient's shape")
    w2t, w1t = filter_t(cell.conv2.weight), filter_t(cell.conv1.weight)  # [ci][tap * co], taps flipped
    if out is None or out.shape != u.shape or out.dtype != torch.bfloat16 or not _cl(out) or \
            out.data_ptr() == u.data_ptr():
        out = torch.empty_like(u, memory_format=torch.channels_last)
    part = None
    if grad is not None:
        if not _cl(grad) or grad.dtype != torch.bfloat16:
            grad = grad.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if grad.shape != u.shape:
            raise ValueError("deq_cell.cell_vjp: grad does not match u")
        part = torch.empty(n, device=u.device, dtype=torch.float32)
    C.deq_cell_vjp(u.data_ptr(), [t.data_ptr() for t in hs], w2t.data_ptr(), w1t.data_ptr(),
                   [_ptr(w1), _ptr(w2), _ptr(w3)], [m1.data_ptr(), m2.data_ptr(), m3.data_ptr()],
                   [r1.data_ptr(), r2.data_ptr(), r3.data_ptr()], out.data_ptr(), _ptr(grad), _ptr(part),
                   n, h, wd, ch, G, _stream(u))
    return out if grad is None else (out, part)


def adjoint_check(part: torch.Tensor, thresh2: torch.Tensor | None = None, flag: torch.Tensor | None = None):
    """``ss = part.sum()`` (0-d fp32, returned) and, with ``flag`` (1 fp32 element) and ``thresh2``
    (fp32 device scalar), ``flag = ss <= thresh2`` — one launch."""
    C = _ext.get(required=True)
    ss = torch.empty((), device=part.device, dtype=torch.float32)
    if flag is not None:
        assert thresh2 is not None and thresh2.dtype == torch.float32 and flag.dtype == torch.float32
    C.deq_adjoint_check(part.data_ptr(), part.numel(), _ptr(thresh2), ss.data_ptr(), _ptr(flag), _stream(part))
    return ss


__all__ = ["ENABLED", "supported", "cell_forward", "cell_vjp", "adjoint_check"]
