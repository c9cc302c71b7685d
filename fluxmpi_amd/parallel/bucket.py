"""Bucketed collectives over many tensors (the functional API's fast path).

The reference issues one collective per leaf (``src/optimizer.jl:21,53``,
``src/synchronize.jl:16``), each staged through host memory. For ResNet-50
that is ~161 allreduces of 1 element .. 2.4 M elements per step. Here leaves
are grouped by (device, dtype), packed by one multi-tensor HIP launch into
64 B-aligned flat buckets (``FLUXMPI_BUCKET_MB``, default 16 MiB: on xGMI a
ring allreduce is per-link bandwidth bound, so messages of MBs amortise the
~10-30 µs per-collective latency; the DDP engine's overlap wants them no
larger, see ``ddp.py``), reduced on the comm stream
while the next bucket is packed, and unpacked after the stream-side wait.

Leaves larger than half a bucket that are already contiguous skip the
pack/unpack copies and are reduced in place.

In a world of one the collectives are the identity and are skipped, unless
``force_comm`` (``FLUXMPI_FORCE_COMM=1``) asks for the real path: pack, RCCL
on the comm stream, event fence, unpack, exactly as with N ranks.
"""
from __future__ import annotations

import torch

from ..ops import multi_tensor as mt
from ..utils.config import get_config
from . import runtime
from .comm import Communicator, ReduceOp, to_op

_WORKSPACE: dict = {}


def _workspace(device: torch.device, dtype: torch.dtype, numel: int, slot: str) -> torch.Tensor:
    key = (str(device), dtype, slot)
    buf = _WORKSPACE.get(key)
    if buf is None or buf.numel() < numel:
        buf = torch.empty(max(numel, 1), dtype=dtype, device=device)
        _WORKSPACE[key] = buf
    return buf[:numel]


def clear_workspace() -> None:
    _WORKSPACE.clear()


def _bucket_bytes() -> int:
    return int(get_config().bucket_mb * (1 << 20))


def plan_buckets(tensors: list, bucket_bytes: int | None = None):
    """Group tensors by (device, dtype) and split each group into buckets.

    Returns a list of ``(kind, device, dtype, [indices], offsets, total)`` where
    kind is ``"direct"`` (one big contiguous tensor, reduced in place) or
    ``"packed"``.
    """
    bb = bucket_bytes or _bucket_bytes()
    groups: dict = {}
    for i, t in enumerate(tensors):
        groups.setdefault((t.device, t.dtype), []).append(i)
    plan = []
    for (dev, dt), idx in groups.items():
        esz = torch.empty((), dtype=dt).element_size()
        cur: list = []
        cur_bytes = 0
        packable = dt in mt.DTYPE_CODE or dev.type != "cuda"  # the HIP pack kernels' dtypes
        for i in idx:
            t = tensors[i]
            nb = t.numel() * esz
            if (nb >= bb // 2 or not packable) and t.is_contiguous():
                # big leaves, and leaves the pack kernels cannot move (int64 step counters,
                # bool masks ...), are reduced in place, one collective each
                plan.append(("direct", dev, dt, [i], [0], t.numel()))
                continue
            if cur and cur_bytes + nb > bb:
                offs, total = mt.aligned_offsets([tensors[j].numel() for j in cur], dt)
                plan.append(("packed", dev, dt, cur, offs, total))
                cur, cur_bytes = [], 0
            cur.append(i)
            cur_bytes += nb
        if cur:
            offs, total = mt.aligned_offsets([tensors[j].numel() for j in cur], dt)
            plan.append(("packed", dev, dt, cur, offs, total))
    return plan


def _contig(tensors):
    """Contiguous views/copies and a list of (orig, copy) pairs to write back."""
    out, back = [], []
    for t in tensors:
        if t.is_contiguous():
            out.append(t)
        else:
            c = t.contiguous()
            out.append(c)
            back.append((t, c))
    return out, back


def _comm_for(dev: torch.device, comm: Communicator | None) -> Communicator:
    if comm is not None:
        return comm
    return runtime.comm_for(torch.empty(0, device=dev))


def _forced(force_comm: bool | None) -> bool:
    return get_config().force_comm if force_comm is None else bool(force_comm)


def _bump_versions(tensors) -> None:
    """The multi-tensor kernels write through raw pointers; tell autograd's version
    counters (and the DDP engine's stale-master check) that the tensors changed."""
    for t in tensors:
        torch.autograd.graph.increment_version(t)


def allreduce_tensors(tensors: list, op=ReduceOp.SUM, comm: Communicator | None = None,
                      bucket_bytes: int | None = None, force_comm: bool | None = None) -> list:
    """In-place allreduce of many tensors with bucketing. Returns ``tensors``."""
    tensors = [t for t in tensors if t is not None]
    if not tensors:
        return tensors
    op = to_op(op)
    forced = _forced(force_comm)
    work_t, back = _contig(tensors)
    plan = plan_buckets(work_t, bucket_bytes)
    pending = []
    ws_off: dict = {}
    for kind, dev, dt, idx, offs, total in plan:
        c = _comm_for(dev, comm)
        if c.size == 1 and not forced:
            continue  # every reduction is the identity for a world of one
        if kind == "direct":
            pending.append((c.allreduce(work_t[idx[0]], op, async_op=True), None, idx, offs))
            continue
        key = (str(dev), dt)
        start = ws_off.get(key, 0)
        ws_off[key] = start + total
        pending.append((None, (dev, dt, start, total), idx, offs))
    # allocate one workspace per (device, dtype) big enough for every in-flight bucket
    flats = {}
    for key, n in ws_off.items():
        dev = torch.device(key[0])
        flats[key] = _workspace(dev, key[1], n, "allreduce")
    launched = []
    for w, ws, idx, offs in pending:
        if ws is None:
            launched.append((w, None, idx, offs))
            continue
        dev, dt, start, total = ws
        flat = flats[(str(dev), dt)][start:start + total]
        mt.pack([work_t[i] for i in idx], flat, offs)
        c = _comm_for(dev, comm)
        launched.append((c.allreduce(flat, op, async_op=True), flat, idx, offs))
    written = []
    for w, flat, idx, offs in launched:
        w.wait()
        if flat is not None:
            mt.unpack(flat, [work_t[i] for i in idx], offs)
        # packed leaves are written by the unpack kernel, "direct" ones by the collective
        # itself through their raw pointer: both bypass autograd's version counters
        written.extend(work_t[i] for i in idx)
    for orig, c in back:
        orig.copy_(c)
    _bump_versions(written)
    return tensors


def broadcast_tensors(tensors: list, root: int = 0, comm: Communicator | None = None,
                      bucket_bytes: int | None = None, force_comm: bool | None = None) -> list:
    """In-place broadcast of many tensors from ``root`` with bucketing."""
    tensors = [t for t in tensors if t is not None]
    if not tensors:
        return tensors
    forced = _forced(force_comm)
    work_t, back = _contig(tensors)
    plan = plan_buckets(work_t, bucket_bytes)
    launched = []
    for kind, dev, dt, idx, offs, total in plan:
        c = _comm_for(dev, comm)
        if c.size == 1:
            if root != 0:
                raise ValueError(f"root {root} out of range for a world of size 1")
            if not forced:
                continue
        if kind == "direct":
            launched.append((c.broadcast(work_t[idx[0]], root, async_op=True), None, idx, offs, c))
            continue
        flat = torch.empty(total, dtype=dt, device=dev)
        if c.rank == root:
            mt.pack([work_t[i] for i in idx], flat, offs)
        launched.append((c.broadcast(flat, root, async_op=True), flat, idx, offs, c))
    written = []
    for w, flat, idx, offs, c in launched:
        w.wait()
        if flat is not None and c.rank != root:  # root already holds the data
            mt.unpack(flat, [work_t[i] for i in idx], offs)
        # every rank, root included, bumps every leaf the broadcast covered (packed or direct):
        # a DDP engine's fp32 master of a synchronised parameter is then re-read from the
        # parameter on ALL ranks, so the masters stay identical across ranks
        written.extend(work_t[i] for i in idx)
    for orig, cc in back:
        orig.copy_(cc)
    _bump_versions(written)
    return tensors
