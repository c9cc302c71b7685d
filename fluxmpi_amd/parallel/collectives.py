"""Public comm primitives (reference ``src/mpi_extensions.jl``).

=====================================  ==========================================
reference                              here
=====================================  ==========================================
``Iallreduce!(send, recv, op, comm)``  ``Iallreduce(send, recv, op)`` -> ``(recv, req)``
``Iallreduce!(buf, op, comm)``         ``Iallreduce(buf, op)`` -> ``(buf, req)`` (in place)
``Ibcast!(buf, root, comm)``           ``Ibcast(buf, root)`` -> ``(buf, req)``
``allreduce!(v, op, comm)``            ``allreduce(v, op)`` -> reduced ``v``
``bcast!(v, root, comm)``              ``bcast(v, root)`` -> broadcast ``v``
``reduce!(v, op, root, comm)``         ``reduce(v, op, root)``; non-root ranks keep ``v``
``MPI.Wait!`` / ``MPI.Waitall!``       ``Wait(req)`` / ``Waitall(reqs)``
=====================================  ==========================================

A trailing communicator argument is accepted and ignored when it is
:data:`COMM_WORLD` (so Julia-shaped calls ``allreduce(x, "+", COMM_WORLD)``
read the same). Inputs may be ``torch.Tensor`` (CPU or GPU), contiguous
``numpy`` arrays (reduced in place through a zero-copy tensor view) or Python
scalars / lists of scalars (a new value is returned).

Unlike the reference, GPU tensors are reduced **in place**,
device-direct over RCCL; as in the reference, callers should still use the
return value.
"""
from __future__ import annotations

import numbers
from typing import Any

import numpy as np
import torch

from . import runtime
from .comm import ReduceOp, Work, to_op


class _CommWorld:
    """Stand-in for ``MPI.COMM_WORLD`` (the only communicator the reference uses)."""

    def __repr__(self):
        return "COMM_WORLD"


COMM_WORLD = _CommWorld()


def _strip_comm(args):
    if args and (args[-1] is COMM_WORLD or args[-1] is None):
        return args[:-1]
    return args


class _Buf:
    """Normalises a user buffer to a contiguous tensor and writes results back."""

    def __init__(self, x: Any):
        self.orig = x
        self.kind = "tensor"
        if isinstance(x, torch.Tensor):
            self.t = x if x.is_contiguous() else x.contiguous()
        elif isinstance(x, np.ndarray):
            if x.flags.c_contiguous and x.flags.writeable:
                self.t = torch.from_numpy(x)
                self.kind = "numpy"
            else:
                self.t = torch.from_numpy(np.ascontiguousarray(x).copy())
                self.kind = "numpy-copy"
        elif isinstance(x, numbers.Number):
            self.t = torch.tensor([x])
            self.kind = "scalar"
        elif isinstance(x, (list, tuple)) and all(isinstance(v, numbers.Number) for v in x):
            self.t = torch.tensor(list(x))
            self.kind = "list"
        else:
            raise TypeError(f"unsupported buffer type {type(x)}")

    def result(self):
        if self.kind == "tensor":
            if self.t is not self.orig:
                self.orig.copy_(self.t)
            return self.orig
        if self.kind == "numpy":
            return self.orig
        if self.kind == "numpy-copy":
            return self.t.numpy()
        if self.kind == "scalar":
            return self.t.item()
        return type(self.orig)(self.t.tolist())


class Request(Work):
    """Result of :func:`Iallreduce` / :func:`Ibcast` (``MPI.Request`` analogue)."""

    def __init__(self, work: Work, buf: _Buf):
        super().__init__(None)
        self._work = work
        self._buf = buf
        self._value = None
        self._done = False

    def wait(self):
        if not self._done:
            self._work.wait()
            self._value = self._buf.result()
            self._done = True
        return self._value

    def is_completed(self):
        return self._done or self._work.is_completed()

    def synchronize(self):
        v = self.wait()
        self._work.synchronize()
        return v


def Wait(req: Request):
    """``MPI.Wait!``: complete ``req`` and return its buffer."""
    return req.wait()


def Waitall(reqs) -> list:
    """``MPI.Waitall!``."""
    return [r.wait() for r in reqs]


# ------------------------------------------------------------------ non-blocking
def Iallreduce(*args):
    """Non-blocking allreduce (reference ``src/mpi_extensions.jl:26-60``).

    ``Iallreduce(sendbuf, recvbuf, op)`` or in place ``Iallreduce(buf, op)``.
    Returns ``(recvbuf, request)``; ``recvbuf`` is valid after ``Wait(request)``.
    """
    args = _strip_comm(args)
    if len(args) == 3:
        send, recv, op = args
        src = _Buf(send)
        dst = _Buf(recv)
        c = runtime.comm_for(dst.t)
        if hasattr(c, "allreduce_out") and src.t.is_cuda and dst.t.is_cuda:
            w = c.allreduce_out(src.t, dst.t, to_op(op), async_op=True)
        else:
            dst.t.copy_(src.t.reshape(dst.t.shape).to(dst.t.dtype))
            w = c.allreduce(dst.t, to_op(op), async_op=True)
        req = Request(w, dst)
        return dst.orig if dst.kind in ("tensor", "numpy") else None, req
    if len(args) == 2:
        buf, op = args
        b = _Buf(buf)
        w = runtime.comm_for(b.t).allreduce(b.t, to_op(op), async_op=True)
        return b.orig if b.kind in ("tensor", "numpy") else None, Request(w, b)
    raise TypeError("Iallreduce(sendbuf, recvbuf, op) or Iallreduce(buf, op)")


def Ibcast(buf, root: int = 0, *rest):
    """Non-blocking broadcast from ``root`` (reference ``src/mpi_extensions.jl:70-88``)."""
    b = _Buf(buf)
    w = runtime.comm_for(b.t).broadcast(b.t, int(root), async_op=True)
    return b.orig if b.kind in ("tensor", "numpy") else None, Request(w, b)


# ------------------------------------------------------------------ blocking
def allreduce(v, op=ReduceOp.SUM, *rest):
    """Blocking allreduce (reference ``src/mpi_extensions.jl:97-111``)."""
    b = _Buf(v)
    runtime.comm_for(b.t).allreduce(b.t, to_op(op))
    return b.result()


def bcast(v, root: int = 0, *rest):
    """Blocking broadcast from ``root`` (reference ``src/mpi_extensions.jl:119-133``)."""
    b = _Buf(v)
    runtime.comm_for(b.t).broadcast(b.t, int(root))
    return b.result()


def reduce(v, op=ReduceOp.SUM, root: int = 0, *rest):
    """Blocking reduce to ``root`` (reference ``src/mpi_extensions.jl:141-155``).

    Non-root ranks get their input back unchanged.
    """
    b = _Buf(v)
    runtime.comm_for(b.t).reduce(b.t, to_op(op), int(root))
    return b.result()


def allgather(v, *rest):
    """Concatenate ``v`` from every rank along a new leading dim (extension)."""
    b = _Buf(v)
    c = runtime.comm_for(b.t)
    out = torch.empty((c.size,) + tuple(b.t.shape), dtype=b.t.dtype, device=b.t.device)
    c.allgather(out.reshape(-1), b.t.reshape(-1))
    return out


def reduce_scatter(v, op=ReduceOp.SUM, *rest):
    """Reduce ``v`` (leading dim divisible by world size) and keep this rank's shard (extension)."""
    b = _Buf(v)
    c = runtime.comm_for(b.t)
    n = b.t.numel()
    if n % c.size:
        raise ValueError("reduce_scatter: numel must be divisible by the world size")
    out = torch.empty(n // c.size, dtype=b.t.dtype, device=b.t.device)
    c.reduce_scatter(out, b.t.reshape(-1), to_op(op))
    return out.reshape((b.t.shape[0] // c.size,) + tuple(b.t.shape[1:])) if b.t.dim() and b.t.shape[0] % c.size == 0 else out


def Barrier(*rest) -> None:
    runtime.barrier()
