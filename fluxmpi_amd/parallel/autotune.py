"""Rank-consistent per-shape kernel selection for N > 1.

The per-shape choices of ``ops/fused_block.py`` (ours vs MIOpen, tile configurations, split-K
variants — the analogue of ``cudnn.benchmark``) are timed on first use. Left alone in a
multi-rank job that would happen:

* on every rank separately, so ranks can pick different kernels (different rounding, and the
  slowest rank's choice gates every step), and
* inside the first backward, while earlier buckets' allreduces are already running on the
  comm stream — RCCL's spinning kernels and the inter-rank skew perturb the timings.

:func:`calibrate` fixes the table once, before any gradient collective: the root rank runs one
forward + backward under ``ddp.no_sync()`` (hooks launch nothing), its table travels to every
rank through the host (gloo) group, every rank loads it, and the table is frozen — a shape
first seen later takes the deterministic default instead of a measurement. This mirrors the
reference's pattern for shared state: the root's copy is broadcast to everyone
(``/root/reference/src/synchronize.jl:10-35``).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from . import runtime


def broadcast_lines(lines: list[str] | None, root: int = 0) -> list[str]:
    """Broadcast a list of strings from ``root`` over the host group (identity at world 1)."""
    comm = runtime.cpu_comm()
    if comm.size == 1:
        return list(lines or [])
    group = getattr(comm, "group", None)
    src = dist.get_global_rank(group, root) if group not in (None, dist.GroupMember.WORLD) else root
    box = [lines if comm.rank == root else None]
    dist.broadcast_object_list(box, src=src, group=group)
    return list(box[0] or [])


def calibrate(ddp, fwd_bwd: Callable[[], object], root: int = 0) -> list[str]:
    """Measure the per-shape kernel choices on ``root`` only, share them, freeze them.

    ``fwd_bwd()`` runs one forward + backward of the training step (no optimiser step). On the
    root it runs under ``ddp.no_sync()``, so no bucket collective is in flight while kernels are
    timed; the other ranks wait in the broadcast. Gradients are discarded afterwards
    (``ddp.zero_grad()``). Returns the choice records every rank now holds.
    """
    from ..ops import fused_block

    comm = runtime.cpu_comm()
    recs = None
    if comm.rank == root:
        with ddp.no_sync():
            fwd_bwd()
        if ddp.device.type == "cuda":
            torch.cuda.synchronize(ddp.device)
        recs = fused_block.dump_choices()
    recs = broadcast_lines(recs, root)
    if comm.rank != root:
        fused_block.load_choice_lines(recs)
    fused_block.freeze_choices()
    ddp.zero_grad()
    if comm.size > 1:
        # the root's extra forward moved its BatchNorm running statistics / batch counters: put
        # every rank's buffers back in step (parameters are untouched: no optimiser step ran)
        bufs = [t.detach() for t in ddp.module.buffers() if t.numel() > 0]
        if bufs:
            from .bucket import broadcast_tensors
            broadcast_tensors(bufs, root, comm=ddp.comm if ddp.comm is not None else None)
    return recs


__all__ = ["broadcast_lines", "calibrate"]
