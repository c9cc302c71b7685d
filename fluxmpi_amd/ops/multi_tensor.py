"""Multi-tensor pack / unpack / scale / fill / sum-of-squares.

GPU tensors go through the gfx950 kernels in ``csrc/kernels/multi_tensor.hip``
(one launch per <=40 tensors, 16 B vector accesses); CPU tensors use the
PyTorch reference implementation below, which is also the numerics oracle of
the GPU tests.
"""
from __future__ import annotations

import torch

from . import _ext

DTYPE_CODE = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6, torch.float64: 8}

# Leaves inside a flat buffer start on 64-byte boundaries (16 B-aligned vector
# path for every dtype, whole cache-line segments per leaf).
ALIGN_BYTES = 64


def align_elems(dtype: torch.dtype) -> int:
    return max(1, ALIGN_BYTES // torch.empty((), dtype=dtype).element_size())


def aligned_offsets(numels, dtype: torch.dtype):
    """Start offset of each leaf in a flat buffer (64 B aligned) and the total length."""
    a = align_elems(dtype)
    offs, cur = [], 0
    for n in numels:
        offs.append(cur)
        cur += (n + a - 1) // a * a
    return offs, cur


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _code(dt: torch.dtype) -> int:
    try:
        return DTYPE_CODE[dt]
    except KeyError:
        raise TypeError(f"dtype {dt} not supported by the multi-tensor kernels") from None


def pack(tensors, flat: torch.Tensor, offsets, scale: float = 1.0) -> torch.Tensor:
    """Gather ``tensors`` into ``flat`` at element ``offsets`` (cast to ``flat.dtype``, times ``scale``)."""
    if not tensors:
        return flat
    if flat.is_cuda:
        C = _ext.get(required=True)
        groups: dict = {}
        for t, o in zip(tensors, offsets):
            if not t.is_contiguous():
                raise ValueError("pack: tensors must be contiguous")
            groups.setdefault(t.dtype, []).append((t, o))
        es = flat.element_size()
        base = flat.data_ptr()
        for dt, items in groups.items():
            C.mt_copy([t.data_ptr() for t, _ in items], [base + o * es for _, o in items],
                      [t.numel() for t, _ in items], _code(dt), _code(flat.dtype), float(scale), _stream(flat))
        return flat
    for t, o in zip(tensors, offsets):
        seg = flat[o:o + t.numel()]
        if scale == 1.0:
            seg.copy_(t.reshape(-1))
        else:
            seg.copy_(t.reshape(-1).to(torch.promote_types(t.dtype, torch.float32)) * scale)
    return flat


def unpack(flat: torch.Tensor, tensors, offsets, scale: float = 1.0):
    """Scatter ``flat`` back into ``tensors`` (cast to each tensor's dtype, times ``scale``)."""
    if not tensors:
        return tensors
    if flat.is_cuda:
        C = _ext.get(required=True)
        groups: dict = {}
        for t, o in zip(tensors, offsets):
            if not t.is_contiguous():
                raise ValueError("unpack: tensors must be contiguous")
            groups.setdefault(t.dtype, []).append((t, o))
        es = flat.element_size()
        base = flat.data_ptr()
        for dt, items in groups.items():
            C.mt_copy([base + o * es for _, o in items], [t.data_ptr() for t, _ in items],
                      [t.numel() for t, _ in items], _code(flat.dtype), _code(dt), float(scale), _stream(flat))
        return tensors
    for t, o in zip(tensors, offsets):
        seg = flat[o:o + t.numel()].reshape(t.shape)
        if scale == 1.0:
            t.copy_(seg)
        else:
            t.copy_(seg.to(torch.promote_types(seg.dtype, torch.float32)) * scale)
    return tensors


def scale_(tensors, scale: float):
    """In-place ``t *= scale`` over many tensors in one launch per dtype."""
    gpu = [t for t in tensors if t.is_cuda]
    cpu = [t for t in tensors if not t.is_cuda]
    for t in cpu:
        t.mul_(scale)
    if gpu:
        C = _ext.get(required=True)
        groups: dict = {}
        for t in gpu:
            groups.setdefault(t.dtype, []).append(t)
        for dt, ts in groups.items():
            ptrs = [t.data_ptr() for t in ts]
            C.mt_copy(ptrs, ptrs, [t.numel() for t in ts], _code(dt), _code(dt), float(scale), _stream(ts[0]))
    return tensors


def fill_(tensors, value: float = 0.0):
    gpu = [t for t in tensors if t.is_cuda]
    for t in tensors:
        if not t.is_cuda:
            t.fill_(value)
    if gpu:
        C = _ext.get(required=True)
        groups: dict = {}
        for t in gpu:
            groups.setdefault(t.dtype, []).append(t)
        for dt, ts in groups.items():
            C.mt_fill([t.data_ptr() for t in ts], [t.numel() for t in ts], _code(dt), float(value), _stream(ts[0]))
    return tensors


def sumsq(tensors) -> torch.Tensor:
    """Sum of squares over all tensors (fp32 scalar tensor on the tensors' device)."""
    if not tensors:
        return torch.zeros(())
    dev = tensors[0].device
    if dev.type == "cuda":
        C = _ext.get(required=True)
        out = torch.zeros(1, device=dev, dtype=torch.float32)
        groups: dict = {}
        for t in tensors:
            groups.setdefault(t.dtype, []).append(t)
        for dt, ts in groups.items():
            C.mt_sumsq([t.data_ptr() for t in ts], [t.numel() for t in ts], _code(dt), out.data_ptr(),
                       _stream(out))
        return out[0]
    acc = torch.zeros((), dtype=torch.float64)
    for t in tensors:
        acc += t.double().pow(2).sum()
    return acc.float()
