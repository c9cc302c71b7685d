"""Weight gradients on a side HIP stream, concurrent with the rest of the backward.

In a backward pass every layer's weight gradient ``dW = dY^T X`` is independent of the
input-gradient chain that carries on to the previous layer: nothing in the backward reads
``dW`` again, only the gradient collective and the optimiser do. On one in-order stream each
``dW`` kernel still sits between two links of that chain, so the chip drains and refills at
every boundary, a persistent GEMM's partial last round leaves CUs idle, and a memory-bound
BatchNorm / LayerNorm backward leaves the matrix cores idle. Here the weight-gradient kernels
run on a second stream of the same device: they start as soon as their operands exist (the side
stream waits for the compute stream at each launch) and fill whatever CUs the chain leaves free
(CDNA4 runs workgroups of two kernels on one CU side by side when registers and LDS allow:
an MFMA-bound wave beside a memory-bound one, MI355X_MICROARCH.md "Wave scheduling").

Joins (what makes the results safe to read):

* **end of backward**: a final autograd callback makes every compute stream that issued side
  work wait for the side stream, so after ``loss.backward()`` returns, ``p.grad`` is ordered
  like any other gradient (user code, the optimiser in ``DDP.step``);
* **collectives during backward**: :func:`fence` makes the communicator's stream wait for the
  side work issued so far before a bucket's allreduce (``parallel/ddp.py``);
* **accumulation**: a tensor hook on every enabled parameter makes the compute stream wait
  before autograd ADDS a side-produced gradient into an existing ``p.grad`` (a parameter used
  twice, ``no_sync`` accumulation, a gradient that is cloned for its layout); the first
  gradient of a parameter is stolen by autograd (no kernel reads it).

Operands are marked with ``record_stream`` so the caching allocator does not hand their memory
to the compute stream while the side stream still reads them.

Scope: parameters registered by a data-parallel engine in "steal" gradient mode
(:func:`enable`); everything else computes its weight gradient in place, on the current stream.

OFF by default (``FLUXMPI_WGRAD_STREAM=1`` turns it on): measured slower. ViT-B/16's Linear weight
gradients on the side stream ran 7229 / 7219 img/s against 7293 / 7278 on one stream, same box,
alternating (``profiles/rd6a_wgrad_stream_ab.jsonl``); round 3 measured the same on ResNet-50
(-4 %). The persistent GEMMs size their grids to one workgroup per CU and assume the chip is
theirs: a concurrent kernel takes CUs from their first round instead of filling their last one,
so the input-gradient chain — the critical path — gets longer by more than the weight gradients
save.

Reference: ``/root/reference/src/optimizer.jl:45-65`` issues every leaf's reduction at once and
waits for all of them; this is the same "all independent work in flight" idea one level down,
for the gradient producers themselves.
"""
from __future__ import annotations

import os
import weakref

import torch

ENABLED = os.environ.get("FLUXMPI_WGRAD_STREAM", "0") == "1"

_ATTR = "_fluxmpi_wgs"
_side: dict = {}          # device index -> side stream
_mains: dict = {}         # device index -> {stream id: stream} that issued side work this backward
_queued = False           # the end-of-backward join is queued for the current backward
launches = 0              # side-stream launches so far (diagnostics / tests)


def enable(params, on: bool = True) -> None:
    """Let the weight gradients of ``params`` run on the side stream (DDP "steal" engines)."""
    for p in params:
        if on and ENABLED and p.is_cuda and not hasattr(p, _ATTR):
            ref = weakref.ref(p)
            h = p.register_hook(lambda g, ref=ref: _before_accumulate(ref, g))
            setattr(p, _ATTR, h)
        elif not on and hasattr(p, _ATTR):
            getattr(p, _ATTR).remove()
            delattr(p, _ATTR)


def active(param) -> bool:
    return ENABLED and param is not None and hasattr(param, _ATTR)


def side_stream(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = torch.cuda.Stream(torch.device("cuda", idx))
        _side[idx] = s
    return s


def pending(device: torch.device) -> bool:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return bool(_mains.get(idx))


def run(fn, param, *inputs: torch.Tensor):
    """``fn()`` (a weight-gradient computation over ``inputs``) on the side stream when ``param``
    is enabled and capture is not active; else on the current stream."""
    if not active(param) or not inputs or not inputs[0].is_cuda or torch.cuda.is_current_stream_capturing():
        return fn()
    global _queued, launches
    dev = inputs[0].device
    main = torch.cuda.current_stream(dev)
    side = side_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in inputs:
        if t is not None and t.is_cuda:
            t.record_stream(side)
    _mains.setdefault(dev.index, {})[main.cuda_stream] = main
    launches += 1
    if not _queued:
        torch.autograd.Variable._execution_engine.queue_callback(join)
        _queued = True
    return out


def fence(stream, device: torch.device) -> None:
    """Make ``stream`` wait for the side work issued so far on ``device`` (before a collective)."""
    if pending(device):
        stream.wait_stream(side_stream(device))


def join() -> None:
    """Every compute stream that issued side work waits for the side stream (end of backward)."""
    global _queued
    _queued = False
    for idx, mains in list(_mains.items()):
        side = _side[idx]
        for s in mains.values():
            s.wait_stream(side)
    _mains.clear()


def _before_accumulate(ref, grad):
    p = ref()
    if p is None or not grad.is_cuda:
        return None
    idx = grad.device.index
    if _mains.get(idx) and (p.grad is not None or grad.stride() != p.stride()):
        # autograd is about to read this (possibly side-produced) gradient on the compute stream
        torch.cuda.current_stream(grad.device).wait_stream(_side[idx])
    return None


__all__ = ["ENABLED", "enable", "active", "run", "fence", "join", "pending", "side_stream"]
