"""Communicator layer (L3 of SURVEY §1).

The reference talks to MPI through MPI.jl plus two raw ``ccall``s
(``MPI_Iallreduce`` / ``MPI_Ibcast``, ``src/mpi_extensions.jl:26-88``) and
always stages GPU buffers through host memory (``:97-155``).

Here every collective is *device-direct* and *stream-ordered*:

* :class:`RcclComm` — the native MI355X path. A C++ communicator
  (``csrc/comm/rccl_comm.cpp``) owns an ``ncclComm_t`` (RCCL over xGMI) that
  is bootstrapped from a unique id exchanged through the process-group store.
  Collectives run on a dedicated HIP stream (normal priority: measured); the caller's
  stream is fenced with HIP events on both sides, so a blocking call never
  blocks the host and an ``async_op`` call returns a :class:`Work` that can
  be waited on later (the ``MPI_Request`` analogue).
* :class:`TorchComm` — a ``torch.distributed`` ProcessGroup (``gloo`` for
  CPU tensors, the RCCL-backed ``nccl`` group as an alternative GPU path).
* :class:`SelfComm` — world of one: every reduction is the identity.

``host_staged=True`` (the ``disable_cudampi_support`` preference) re-creates
the reference's D2H -> collective -> H2D path for A/B comparisons.
"""
from __future__ import annotations

import enum
import operator
import os
from typing import Any

import numpy as np
import torch
import torch.distributed as dist

from ..ops import _ext

# RcclComm's stream priority: 0 normal (default), -1 high (FLUXMPI_COMM_PRIORITY=-1). Measured
# (rd3zh / rd3zi, ResNet-50 --force-comm, same boxes): the high-priority queue cost 1.0-2.9 % of
# the step at N=1 against 0.25-0.5 % at normal priority, and with an emulated RCCL CU footprint
# (--emulate-comm 64:300) normal priority exposed LESS comm time (0.010 vs 0.037 ms per step)
_COMM_PRIORITY = int(os.environ.get("FLUXMPI_COMM_PRIORITY", "0"))


class ReduceOp(enum.IntEnum):
    """Built-in reductions; values are RCCL's ``ncclRedOp_t``."""

    SUM = 0
    PROD = 1
    MAX = 2
    MIN = 3
    AVG = 4


_OP_ALIASES = {
    operator.add: ReduceOp.SUM, "+": ReduceOp.SUM, "sum": ReduceOp.SUM, sum: ReduceOp.SUM,
    np.add: ReduceOp.SUM, torch.add: ReduceOp.SUM,
    operator.mul: ReduceOp.PROD, "*": ReduceOp.PROD, "prod": ReduceOp.PROD, np.multiply: ReduceOp.PROD,
    torch.mul: ReduceOp.PROD,
    max: ReduceOp.MAX, "max": ReduceOp.MAX, np.maximum: ReduceOp.MAX, torch.maximum: ReduceOp.MAX,
    min: ReduceOp.MIN, "min": ReduceOp.MIN, np.minimum: ReduceOp.MIN, torch.minimum: ReduceOp.MIN,
    "avg": ReduceOp.AVG, "mean": ReduceOp.AVG,
}


def to_op(op: Any) -> ReduceOp:
    """Coerce a Julia-style operator (``+``, ``*``, ``max``, ``min``) to a :class:`ReduceOp`.

    Mirrors ``Iallreduce!(rbuf, op, comm) = Iallreduce!(rbuf, MPI.Op(op, eltype(rbuf)), comm)``
    (reference ``src/mpi_extensions.jl:52-54``).
    """
    if isinstance(op, ReduceOp):
        return op
    if isinstance(op, dist.ReduceOp.RedOpType) or isinstance(op, dist.ReduceOp):
        m = {dist.ReduceOp.SUM: ReduceOp.SUM, dist.ReduceOp.PRODUCT: ReduceOp.PROD,
             dist.ReduceOp.MAX: ReduceOp.MAX, dist.ReduceOp.MIN: ReduceOp.MIN,
             dist.ReduceOp.AVG: ReduceOp.AVG}
        return m[op]
    key = op.lower() if isinstance(op, str) else op
    try:
        return _OP_ALIASES[key]
    except (KeyError, TypeError):
        raise ValueError(f"unsupported reduction operator {op!r}; use +, *, max, min or 'avg'") from None


_TORCH_OP = {
    ReduceOp.SUM: dist.ReduceOp.SUM,
    ReduceOp.PROD: dist.ReduceOp.PRODUCT,
    ReduceOp.MAX: dist.ReduceOp.MAX,
    ReduceOp.MIN: dist.ReduceOp.MIN,
}

# Reductions over bool buffers run on a uint8 copy with the logical equivalent of the
# requested op (SUM/MAX = OR, PROD/MIN = AND), so no rank count can overflow or wrap
# the byte, and the result is renormalised to {0, 1} when it is copied back.
_BOOL_OP = {ReduceOp.SUM: ReduceOp.MAX, ReduceOp.MAX: ReduceOp.MAX, ReduceOp.PROD: ReduceOp.MIN,
            ReduceOp.MIN: ReduceOp.MIN}


def bool_op(op: ReduceOp) -> ReduceOp:
    try:
        return _BOOL_OP[op]
    except KeyError:
        raise ValueError(f"reduction {op.name} is not defined for bool buffers") from None


class CommAbortedError(RuntimeError):
    """The communicator was aborted (by the watchdog or :meth:`RcclComm.abort`)."""


# torch dtype -> ncclDataType_t
NCCL_DTYPE = {
    torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4,
    torch.float16: 6, torch.float32: 7, torch.float64: 8, torch.bfloat16: 9,
    torch.bool: 1,
}
if hasattr(torch, "float8_e4m3fn"):
    NCCL_DTYPE[torch.float8_e4m3fn] = 10
    NCCL_DTYPE[torch.float8_e5m2] = 11


class Work:
    """Handle of an in-flight collective (the ``MPI.Request`` analogue)."""

    def __init__(self, result: Any = None):
        self.result = result
        self._done = True

    def wait(self) -> Any:
        return self.result

    def is_completed(self) -> bool:
        return True

    def synchronize(self) -> Any:
        """Block the *host* until the collective finished (``MPI.Wait!`` on host data)."""
        return self.wait()


class _TorchWork(Work):
    def __init__(self, work, result, post=None):
        super().__init__(result)
        self._work = work
        self._post = post
        self._finished = False

    def wait(self):
        if not self._finished:
            if self._work is not None:
                self._work.wait()
            if self._post is not None:
                self._post()
            self._finished = True
        return self.result

    def is_completed(self) -> bool:
        return self._finished or (self._work is None or self._work.is_completed())


class _StreamWork(Work):
    """A collective enqueued on the comm stream; ``wait`` fences the caller's stream."""

    def __init__(self, event: torch.cuda.Event, result, device, post=None):
        super().__init__(result)
        self.event = event
        self.device = device
        self._post = post
        self._waited = False

    def wait(self):
        if not self._waited:
            torch.cuda.current_stream(self.device).wait_event(self.event)
            if self._post is not None:
                self._post()
            self._waited = True
        return self.result

    def is_completed(self) -> bool:
        return self.event.query()

    def covered(self):
        """The caller's stream already waits on a LATER collective of the same (in-order) comm
        stream: this one is complete by then, so skip its own fence (post-processing still runs)."""
        if not self._waited:
            if self._post is not None:
                self._post()
            self._waited = True
        return self.result

    def synchronize(self):
        self.wait()
        self.event.synchronize()
        return self.result


class _MultiWork(Work):
    def __init__(self, works, result):
        super().__init__(result)
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return self.result

    def is_completed(self):
        return all(w.is_completed() for w in self.works)

    def synchronize(self):
        for w in self.works:
            w.synchronize()
        return self.result


class Communicator:
    """Abstract communicator over one group of ranks."""

    name = "abstract"

    def __init__(self, rank: int, size: int):
        self.rank = rank
        self.size = size

    # all tensor arguments are modified in place; the tensor is also returned
    def allreduce(self, t: torch.Tensor, op=ReduceOp.SUM, async_op: bool = False):
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, root: int = 0, async_op: bool = False):
        raise NotImplementedError

    def reduce(self, t: torch.Tensor, op=ReduceOp.SUM, root: int = 0, async_op: bool = False):
        raise NotImplementedError

    def allgather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """``out`` (size*n) <- concat over ranks of ``inp`` (n)."""
        raise NotImplementedError

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op=ReduceOp.SUM, async_op: bool = False):
        """``out`` (n) <- this rank's slice of the reduction of ``inp`` (size*n)."""
        raise NotImplementedError

    def alltoall(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        raise NotImplementedError

    def self_report(self) -> dict:
        """What the backend itself reports about the group (RCCL: rank count, rank, device);
        empty for backends without such a query."""
        return {}

    def barrier(self) -> None:
        raise NotImplementedError

    def allreduce_coalesced(self, tensors, op=ReduceOp.SUM, async_op: bool = False):
        """Allreduce several buffers as one batched operation (in place)."""
        works = [self.allreduce(t, op, async_op=True) for t in tensors]
        if async_op:
            return _MultiWork(works, list(tensors))
        for w in works:
            w.wait()
        return list(tensors)

    def destroy(self) -> None:
        pass

    def check_async_error(self) -> None:
        pass


class SelfComm(Communicator):
    """World of size one: reductions are the identity, broadcasts are no-ops."""

    name = "self"

    def __init__(self):
        super().__init__(0, 1)

    def allreduce(self, t, op=ReduceOp.SUM, async_op=False):
        w = Work(t)
        return w if async_op else t

    def broadcast(self, t, root=0, async_op=False):
        if root != 0:
            raise ValueError(f"root {root} out of range for a world of size 1")
        w = Work(t)
        return w if async_op else t

    def reduce(self, t, op=ReduceOp.SUM, root=0, async_op=False):
        return self.broadcast(t, root, async_op)

    def allgather(self, out, inp, async_op=False):
        out.copy_(inp.reshape(out.shape))
        return Work(out) if async_op else out

    def reduce_scatter(self, out, inp, op=ReduceOp.SUM, async_op=False):
        out.copy_(inp.reshape(out.shape))
        return Work(out) if async_op else out

    def alltoall(self, out, inp, async_op=False):
        out.copy_(inp)
        return Work(out) if async_op else out

    def barrier(self):
        return None


class TorchComm(Communicator):
    """``torch.distributed`` ProcessGroup (gloo on CPU; RCCL-backed nccl on GPU)."""

    name = "torch"

    def __init__(self, group, rank: int, size: int, backend: str):
        super().__init__(rank, size)
        self.group = group
        self.backend = backend
        self.name = f"torch-{backend}"

    def _global(self, r: int) -> int:
        if self.group is None or self.group is dist.GroupMember.WORLD:
            return r
        return dist.get_global_rank(self.group, r)

    def allreduce(self, t, op=ReduceOp.SUM, async_op=False):
        op = to_op(op)
        post = None
        if op == ReduceOp.AVG and self.backend == "gloo":
            # gloo has no AVG: SUM then scale
            tdop = dist.ReduceOp.SUM
            post = (lambda: t.div_(self.size)) if t.is_floating_point() else (
                lambda: t.copy_(torch.div(t, self.size, rounding_mode="floor")))
        else:
            tdop = _TORCH_OP.get(op, dist.ReduceOp.AVG)
        if t.dtype == torch.bool:
            # reductions over bool are not supported by every backend
            tmp = t.to(torch.uint8)
            w = dist.all_reduce(tmp, op=_TORCH_OP[bool_op(op)], group=self.group, async_op=True)
            work = _TorchWork(w, t, post=lambda: t.copy_(tmp.bool()))
        else:
            w = dist.all_reduce(t, op=tdop, group=self.group, async_op=True)
            work = _TorchWork(w, t, post=post)
        if async_op:
            return work
        return work.wait()

    def broadcast(self, t, root=0, async_op=False):
        w = dist.broadcast(t, src=self._global(root), group=self.group, async_op=True)
        work = _TorchWork(w, t)
        return work if async_op else work.wait()

    def reduce(self, t, op=ReduceOp.SUM, root=0, async_op=False):
        op = to_op(op)
        if op == ReduceOp.AVG:
            raise ValueError("reduce with AVG is not supported; use SUM and scale")
        if self.backend == "gloo" and self.rank != root:
            # gloo's reduce may scribble on non-root buffers; the reference contract is
            # "non-root ranks keep their input" (test/test_mpi_extensions.jl:55-60).
            tmp = t.clone()
            w = dist.reduce(tmp, dst=self._global(root), op=_TORCH_OP[op], group=self.group, async_op=True)
            work = _TorchWork(w, t)
        else:
            w = dist.reduce(t, dst=self._global(root), op=_TORCH_OP[op], group=self.group, async_op=True)
            work = _TorchWork(w, t)
        return work if async_op else work.wait()

    def allgather(self, out, inp, async_op=False):
        w = dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)
        work = _TorchWork(w, out)
        return work if async_op else work.wait()

    def reduce_scatter(self, out, inp, op=ReduceOp.SUM, async_op=False):
        op = to_op(op)
        if self.backend == "gloo":
            # gloo lacks reduce_scatter_tensor: allreduce a copy and slice
            tmp = inp.clone()
            w = dist.all_reduce(tmp, op=_TORCH_OP.get(op, dist.ReduceOp.SUM), group=self.group, async_op=True)
            n = out.numel()

            def post():
                sl = tmp.reshape(-1)[self.rank * n:(self.rank + 1) * n].reshape(out.shape)
                if op == ReduceOp.AVG:
                    sl = sl / self.size
                out.copy_(sl)
            work = _TorchWork(w, out, post=post)
        else:
            w = dist.reduce_scatter_tensor(out, inp, op=_TORCH_OP.get(op, dist.ReduceOp.AVG),
                                           group=self.group, async_op=True)
            work = _TorchWork(w, out)
        return work if async_op else work.wait()

    def alltoall(self, out, inp, async_op=False):
        w = dist.all_to_all_single(out, inp, group=self.group, async_op=True)
        work = _TorchWork(w, out)
        return work if async_op else work.wait()

    def barrier(self):
        dist.barrier(group=self.group)


class GlooDeviceComm(TorchComm):
    """gloo collectives on *device* tensors (backend ``gloo-device``).

    RCCL refuses two ranks on one GPU (``ncclCommInitRank`` -> invalid usage,
    ``profiles/r2_probe_rccl_two_ranks_one_gpu.json``), so this is how several
    ranks sharing one MI355X run the device-side engine: DDP's hook-driven
    overlap, packing and stream fencing over CUDA tensors, with gloo's own
    device<->host staging. allreduce and broadcast go to gloo directly (its CUDA
    work makes the caller's stream wait on completion); the rarer collectives
    stage through host memory explicitly. A test/rehearsal backend, not a fast one.
    """

    name = "gloo-device"

    def __init__(self, group, rank: int, size: int):
        super().__init__(group, rank, size, "gloo")
        self.name = "gloo-device"

    def self_report(self) -> dict:
        """The process group's own answer (``dist.get_world_size`` / ``get_rank`` on this
        communicator's group) and the device the ranks share, so the bench self-check runs on the
        ``--same-device`` rehearsal path too (keys as RcclComm's, prefixed ``comm_``)."""
        import torch.distributed as dist

        dev = torch.cuda.current_device() if torch.cuda.is_available() else None
        return {"comm_backend": self.name, "comm_nranks": int(dist.get_world_size(self.group)),
                "comm_rank": int(dist.get_rank(self.group)), "comm_device": dev}

    def _host(self, fn, out, *inputs):
        hs = [t.detach().cpu() for t in inputs]
        ho = out.detach().cpu()
        fn(ho, *hs)
        out.copy_(ho)
        return out

    def reduce(self, t, op=ReduceOp.SUM, root=0, async_op=False):
        if not t.is_cuda:
            return super().reduce(t, op, root, async_op)
        h = t.detach().cpu()
        TorchComm.reduce(self, h, op, root)
        if self.rank == root:
            t.copy_(h)
        return Work(t) if async_op else t

    def allgather(self, out, inp, async_op=False):
        if not out.is_cuda:
            return super().allgather(out, inp, async_op)
        r = self._host(lambda ho, hi: TorchComm.allgather(self, ho, hi), out, inp)
        return Work(r) if async_op else r

    def reduce_scatter(self, out, inp, op=ReduceOp.SUM, async_op=False):
        if not out.is_cuda:
            return super().reduce_scatter(out, inp, op, async_op)
        r = self._host(lambda ho, hi: TorchComm.reduce_scatter(self, ho, hi, op), out, inp)
        return Work(r) if async_op else r

    def alltoall(self, out, inp, async_op=False):
        if not out.is_cuda:
            return super().alltoall(out, inp, async_op)
        r = self._host(lambda ho, hi: TorchComm.alltoall(self, ho, hi), out, inp)
        return Work(r) if async_op else r


def bootstrap_unique_id(make_uid, store, rank: int, size: int, tag: str = "world") -> bytes:
    """The RCCL unique id of this communicator generation, shared through the host store.

    Rank 0 creates it (``make_uid()`` = ``ncclGetUniqueId``) and publishes it; the others
    block in ``store.get`` until it is there. One key per Init generation: every rank bumps the
    counter once per bootstrap, and all adds of generation k precede any add of k+1
    (``ncclCommInitRank`` is collective), so Init -> Finalize -> Init on a surviving store can
    never read the previous generation's id. (The reference's analogue is ``MPI.Init``'s PMI
    wire-up, ``/root/reference/src/common.jl:22``.)
    """
    if size == 1:
        return bytes(make_uid())
    gen = (int(store.add(f"fluxmpi_amd/rccl_gen/{tag}", 1)) - 1) // size
    key = f"fluxmpi_amd/rccl_uid/{tag}/{gen}"
    if rank == 0:
        uid = bytes(make_uid())
        store.set(key, uid)
        return uid
    return bytes(store.get(key))


class RcclComm(Communicator):
    """Native RCCL communicator (C++ ``fluxmpi::RcclComm``) on a dedicated HIP stream.

    Every call: record "inputs ready" on the caller's stream -> the comm stream
    waits -> ``ncclAllReduce``/``ncclBroadcast``/... -> record "done". A
    blocking call makes the caller's *stream* (not the host) wait on "done",
    which is exactly the ordering a subsequent kernel needs. The
    caching allocator is told about the cross-stream use (``record_stream``).
    """

    name = "rccl"
    # every collective runs on ONE stream, in issue order: a wait on the newest covers the rest
    in_order = True

    def __init__(self, rank: int, size: int, device: torch.device, store=None, tag: str = "world"):
        super().__init__(rank, size)
        C = _ext.get(required=True)
        if C is None or not hasattr(C, "RcclComm"):
            raise RuntimeError("native RCCL communicator not available in fluxmpi_amd._C")
        self.device = torch.device(device)
        self.abort_reason: str | None = None
        uid = bootstrap_unique_id(C.rccl_unique_id, store, rank, size, tag)
        with torch.cuda.device(self.device):
            self._h = C.RcclComm(bytes(uid), rank, size, self.device.index)
            # normal priority by default: a high-priority queue slowed the overlapped
            # backward more than it sped up the comm (see _COMM_PRIORITY)
            self.stream = torch.cuda.Stream(self.device, priority=_COMM_PRIORITY)
        self.version = C.rccl_version()
        self.priority = _COMM_PRIORITY

    def self_report(self) -> dict:
        """``ncclCommCount`` / ``ncclCommUserRank`` / ``ncclCommCuDevice`` of the live
        communicator, the stream priority and the RCCL version (bench.py records and checks them)."""
        h = self._handle()
        return {"rccl_nranks": int(h.comm_count()), "rccl_rank": int(h.comm_user_rank()),
                "rccl_device": int(h.comm_device()), "comm_priority": getattr(self, "priority", _COMM_PRIORITY),
                "rccl_version": getattr(self, "version", None)}

    # --- helpers ---------------------------------------------------------------
    def _enter(self, *tensors):
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        return cur

    def _exit(self, tensors, result, async_op, post=None):
        for t in tensors:
            t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        work = _StreamWork(ev, result, self.device, post)
        if async_op:
            return work
        return work.wait()

    @property
    def aborted(self) -> bool:
        return self.abort_reason is not None

    def _handle(self):
        if self.abort_reason is not None:
            raise CommAbortedError(f"RCCL communicator was aborted ({self.abort_reason}); "
                                   "re-run Init in a new process to continue")
        if self._h is None:
            raise RuntimeError("RCCL communicator has been destroyed (Finalize)")
        return self._h

    def abort(self, reason: str = "abort() called") -> None:
        """``ncclCommAbort``: unblock every pending collective; later calls raise
        :class:`CommAbortedError`. Safe to call from the watchdog thread."""
        if self.abort_reason is None:
            self.abort_reason = reason
        h = self._h
        if h is not None:
            h.abort()

    @staticmethod
    def _check(t: torch.Tensor):
        if not t.is_cuda:
            raise ValueError("RcclComm handles device tensors only")
        if not t.is_contiguous():
            raise ValueError("collective buffers must be contiguous")
        if t.dtype not in NCCL_DTYPE:
            raise TypeError(f"dtype {t.dtype} not supported by RCCL")

    # --- collectives ---------------------------------------------------------
    def allreduce(self, t, op=ReduceOp.SUM, async_op=False):
        self._check(t)
        op = to_op(op)
        h = self._handle()
        if t.dtype == torch.bool:
            # RCCL has no bool type: reduce a uint8 copy with the logical op, renormalise back
            tmp = t.to(torch.uint8)
            self._enter()
            h.allreduce(tmp.data_ptr(), tmp.data_ptr(), tmp.numel(), NCCL_DTYPE[torch.uint8], int(bool_op(op)),
                        self.stream.cuda_stream)
            return self._exit([tmp], t, async_op, post=lambda: t.copy_(tmp.bool()))
        self._enter(t)
        h.allreduce(t.data_ptr(), t.data_ptr(), t.numel(), NCCL_DTYPE[t.dtype], int(op), self.stream.cuda_stream)
        return self._exit([t], t, async_op)

    def allreduce_out(self, send, recv, op=ReduceOp.SUM, async_op=False):
        self._check(send)
        self._check(recv)
        op = to_op(op)
        self._enter()
        self._handle().allreduce(send.data_ptr(), recv.data_ptr(), send.numel(), NCCL_DTYPE[send.dtype], int(op),
                          self.stream.cuda_stream)
        return self._exit([send, recv], recv, async_op)

    def broadcast(self, t, root=0, async_op=False):
        self._check(t)
        self._enter()
        self._handle().broadcast(t.data_ptr(), t.data_ptr(), t.numel(), NCCL_DTYPE[t.dtype], int(root),
                          self.stream.cuda_stream)
        return self._exit([t], t, async_op)

    def reduce(self, t, op=ReduceOp.SUM, root=0, async_op=False):
        self._check(t)
        op = to_op(op)
        self._enter()
        if self.rank == root:
            self._handle().reduce(t.data_ptr(), t.data_ptr(), t.numel(), NCCL_DTYPE[t.dtype], int(op), int(root),
                           self.stream.cuda_stream)
            return self._exit([t], t, async_op)
        # non-root keeps its input (reference contract): send from t, receive nowhere useful
        scratch = torch.empty_like(t)
        self._handle().reduce(t.data_ptr(), scratch.data_ptr(), t.numel(), NCCL_DTYPE[t.dtype], int(op), int(root),
                       self.stream.cuda_stream)
        return self._exit([t, scratch], t, async_op)

    def allgather(self, out, inp, async_op=False):
        self._check(out)
        self._check(inp)
        self._enter()
        self._handle().allgather(inp.data_ptr(), out.data_ptr(), inp.numel(), NCCL_DTYPE[inp.dtype],
                          self.stream.cuda_stream)
        return self._exit([out, inp], out, async_op)

    def reduce_scatter(self, out, inp, op=ReduceOp.SUM, async_op=False):
        self._check(out)
        self._check(inp)
        op = to_op(op)
        self._enter()
        self._handle().reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(), NCCL_DTYPE[inp.dtype], int(op),
                               self.stream.cuda_stream)
        return self._exit([out, inp], out, async_op)

    def alltoall(self, out, inp, async_op=False):
        self._check(out)
        self._check(inp)
        self._enter()
        self._handle().alltoall(inp.data_ptr(), out.data_ptr(), inp.numel() // self.size, NCCL_DTYPE[inp.dtype],
                         self.stream.cuda_stream)
        return self._exit([out, inp], out, async_op)

    def barrier(self):
        flag = torch.zeros(1, device=self.device, dtype=torch.int32)
        self.allreduce(flag)
        torch.cuda.current_stream(self.device).synchronize()

    def allreduce_coalesced(self, tensors, op=ReduceOp.SUM, async_op=False):
        """One ``ncclGroupStart/End`` over many buffers: a single fused launch."""
        for t in tensors:
            self._check(t)
        op = to_op(op)
        self._enter()
        self._handle().allreduce_many([t.data_ptr() for t in tensors], [t.numel() for t in tensors],
                               [NCCL_DTYPE[t.dtype] for t in tensors], int(op), self.stream.cuda_stream)
        return self._exit(list(tensors), list(tensors), async_op)

    def check_async_error(self):
        h = self._h
        if h is None or self.abort_reason is not None:  # destroyed (Finalize) or aborted
            return
        code = h.async_error()
        if code != 0:
            raise RuntimeError(f"RCCL asynchronous error {code}: {h.error_string(code)}")

    def destroy(self):
        h = getattr(self, "_h", None)
        if h is not None:
            if self.abort_reason is None:
                torch.cuda.synchronize(self.device)
                h.destroy()
            self._h = None


class HostStagedComm(Communicator):
    """Reference-faithful GPU path: D2H copy -> CPU collective -> H2D copy.

    Enabled only by the ``disable_cudampi_support`` preference; exists for A/B
    measurements of what device-direct RCCL buys.
    """

    name = "host-staged"

    def __init__(self, cpu_comm: Communicator):
        super().__init__(cpu_comm.rank, cpu_comm.size)
        self.cpu = cpu_comm

    def _staged(self, t, fn):
        h = t.detach().cpu()
        fn(h)
        t.copy_(h)
        return t

    def allreduce(self, t, op=ReduceOp.SUM, async_op=False):
        r = self._staged(t, lambda h: self.cpu.allreduce(h, op))
        return Work(r) if async_op else r

    def broadcast(self, t, root=0, async_op=False):
        r = self._staged(t, lambda h: self.cpu.broadcast(h, root))
        return Work(r) if async_op else r

    def reduce(self, t, op=ReduceOp.SUM, root=0, async_op=False):
        r = self._staged(t, lambda h: self.cpu.reduce(h, op, root))
        return Work(r) if async_op else r

    def allgather(self, out, inp, async_op=False):
        ho = out.cpu()
        self.cpu.allgather(ho, inp.cpu())
        out.copy_(ho)
        return Work(out) if async_op else out

    def reduce_scatter(self, out, inp, op=ReduceOp.SUM, async_op=False):
        ho = out.cpu()
        self.cpu.reduce_scatter(ho, inp.cpu(), op)
        out.copy_(ho)
        return Work(out) if async_op else out

    def alltoall(self, out, inp, async_op=False):
        ho = out.cpu()
        self.cpu.alltoall(ho, inp.cpu())
        out.copy_(ho)
        return Work(out) if async_op else out

    def barrier(self):
        self.cpu.barrier()
