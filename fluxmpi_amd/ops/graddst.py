"""Direct gradient delivery: kernels write a parameter's gradient straight into its DDP bucket.

In "steal" mode the data-parallel engine (``parallel/ddp.py``) packs every freshly produced
gradient into its flat bucket with one multi-tensor copy per bucket before the bucket's
allreduce. The weight-gradient kernels of this package can skip that copy: while a DDP engine
that communicates is attached, each of its parameters carries a destination (its bucket slice),
and the op that produces the parameter's gradient allocates its output there
(:func:`empty`) instead of in a fresh tensor. Autograd then steals that tensor as ``p.grad``
(it has the parameter's strides), the bucket's pack finds ``p.grad`` already in place and moves
nothing.

Rules that keep it exact:

* a destination is handed out at most once per backward (:func:`take`), and only while
  ``p.grad`` is None: a parameter used twice in one graph (its second gradient is summed with the
  first by autograd) or a gradient accumulation (``no_sync``) gets fresh tensors, which the pack
  copies as before;
* the destination is only the MEMORY: whatever the op returns (even if autograd clones it for a
  layout mismatch) is still what ``p.grad`` becomes, and the pack copies anything that is not
  already in the slice;
* ops bind the parameter (:func:`into`) only around the call whose result they return (never
  around an autotuning measurement).

Reference behaviour this replaces: ``/root/reference/src/optimizer.jl:45-65`` reduces every
leaf's gradient where it lies (one MPI call per leaf); here the gradient is born in the
communication buffer.
"""
from __future__ import annotations

import threading
from contextlib import contextmanager

import torch

_ATTR = "_fluxmpi_gdst"
_cur = threading.local()


class _Dest:
    __slots__ = ("flat", "offset", "armed")

    def __init__(self, flat: torch.Tensor, offset: int):
        self.flat = flat
        self.offset = offset
        self.armed = True


def attach(p: torch.Tensor, flat: torch.Tensor, offset: int) -> None:
    """Give parameter ``p`` the destination ``flat[offset:offset + p.numel()]`` (DDP setup)."""
    setattr(p, _ATTR, _Dest(flat, offset))


def detach(p: torch.Tensor) -> None:
    if hasattr(p, _ATTR):
        delattr(p, _ATTR)


def rearm(p: torch.Tensor) -> None:
    """Allow one more delivery (DDP re-arms every parameter for each backward)."""
    d = getattr(p, _ATTR, None)
    if d is not None:
        d.armed = True


def take(p: torch.Tensor | None, shape, dtype: torch.dtype) -> torch.Tensor | None:
    """A contiguous ``shape`` tensor over ``p``'s bucket slice, or None (no destination, already
    delivered this backward, ``p.grad`` holds a gradient, or size / dtype differ)."""
    if p is None:
        return None
    d = getattr(p, _ATTR, None)
    if d is None or not d.armed or p.grad is not None or dtype != p.dtype:
        return None
    n = 1
    for s in shape:
        n *= int(s)
    if n != p.numel():
        return None
    d.armed = False
    return d.flat[d.offset:d.offset + n].view(*shape)


@contextmanager
def into(param: torch.Tensor | None):
    """Within the block, the next :func:`empty` of the parameter's size and dtype is its slice."""
    prev = getattr(_cur, "p", None)
    _cur.p = param
    try:
        yield
    finally:
        _cur.p = prev


def empty(shape, dtype: torch.dtype, device) -> torch.Tensor:
    """``torch.empty(shape)``, or the bound parameter's bucket slice when it fits (see module)."""
    p = getattr(_cur, "p", None)
    if p is not None:
        t = take(p, shape, dtype)
        if t is not None:
            _cur.p = None
            return t
    return torch.empty(*shape, dtype=dtype, device=device)


def _dense(p: torch.Tensor) -> bool:
    """``p``'s elements fill ``p.numel()`` consecutive slots in some dimension order (contiguous,
    channels_last, ...): its strides are a permutation of a contiguous layout's."""
    expect = 1
    for size, stride in sorted(zip(p.shape, p.stride()), key=lambda t: (t[1], t[0])):
        if size == 1:
            continue
        if stride != expect:
            return False
        expect *= size
    return True


def empty_like(p: torch.Tensor, dtype: torch.dtype | None = None) -> torch.Tensor:
    """A gradient buffer for ``p`` with ``p``'s strides (``p.shape``, ``p.stride()``, e.g. a
    channels_last filter) over its bucket slice when one is available (see :func:`take`), else
    ``torch.empty_like(p)`` (``memory_format`` preserved)."""
    dt = dtype or p.dtype
    t = take(p, (p.numel(),), dt) if p.is_contiguous() or _dense(p) else None
    if t is not None:
        return t.as_strided(p.shape, p.stride())
    return torch.empty_like(p, dtype=dt)


def deliver(p: torch.Tensor | None, value: torch.Tensor, dtype: torch.dtype | None = None) -> torch.Tensor:
    """``value.to(dtype or p.dtype)`` written straight into ``p``'s bucket slice when one is
    available (the cast a reduction result needs anyway becomes the delivery: no separate pack
    copy later), else the plain cast."""
    dt = dtype or (p.dtype if p is not None else value.dtype)
    t = take(p, tuple(value.shape), dt) if p is not None else None
    if t is None:
        return value.to(dt)
    t.copy_(value)
    return t


def delivered(p: torch.Tensor) -> bool:
    """True if ``p.grad`` lies in ``p``'s destination slice (diagnostics / tests)."""
    d = getattr(p, _ATTR, None)
    if d is None or p.grad is None:
        return False
    es = d.flat.element_size()
    return p.grad.data_ptr() == d.flat.data_ptr() + d.offset * es
