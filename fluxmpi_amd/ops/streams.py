"""A side HIP stream for weight gradients, overlapped with the input-gradient chain.

In a backward pass the input gradient (dgrad) of layer L feeds layer L-1 — the critical path —
while the weight gradient (wgrad) of layer L feeds nothing but the optimizer (and the gradient
allreduce). On one stream the two serialize; here the wgrad GEMMs (and their split-K reductions)
run on a second stream of the same device, so a memory-bound BatchNorm pass or a dgrad GEMM of
the chain shares the CUs with an MFMA-bound wgrad instead of waiting for it.

Ordering, all with stream waits (no host sync):

* :func:`run` makes the side stream wait for the current stream's work so far (the wgrad's
  inputs: the output gradient and the saved activation), launches on the side stream, and marks
  the inputs/outputs with ``record_stream`` so the caching allocator does not hand their memory
  to either stream early;
* the current stream joins the side stream at the end of the backward pass (an autograd engine
  callback, queued once per backward), so the optimizer step sees every gradient;
* :class:`~fluxmpi_amd.parallel.ddp.DistributedDataParallel` packs and launches a bucket's
  allreduce from the side stream (after it waited for the main stream), so a bucket's collective
  orders after the weight gradients it carries (:func:`pending`).

Opt-in (``FLUXMPI_WGRAD_STREAM=1``): measured on one MI355X it costs more than it overlaps —
ResNet-50 bs256 11746 -> 11247 img/s (also with 2 or 4 rounds of persistent grids: 11212 / 11177),
ViT-B/16 6283 -> 6099 img/s (profiles/r3_wgrad_stream_ab.jsonl): the main stream's kernels lose CUs
and L2 to the concurrent weight-gradient GEMMs for longer than the overlap saves. Gradients are
bit-identical either way (tests/test_wgrad_stream_gpu.py). Under HIP graph capture the side
stream is not used.
"""
from __future__ import annotations

import os

import torch

ENABLED = os.environ.get("FLUXMPI_WGRAD_STREAM", "0") == "1"

_SIDE: dict = {}    # device index -> torch.cuda.Stream
_ARMED: dict = {}   # device index -> side stream, while a join is queued for the current backward


def side_stream(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _SIDE[idx] = s
    return s


def active(device: torch.device) -> bool:
    return (ENABLED and device.type == "cuda" and torch.cuda.is_available()
            and not torch.cuda.is_current_stream_capturing())


def _tensors(obj):
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, (tuple, list)):
        for o in obj:
            yield from _tensors(o)


def run(fn, *inputs, param=None):
    """``fn()`` on the weight-gradient stream of ``inputs[0]``'s device (see the module docstring);
    returns its result. Falls back to a plain call when the side stream is off or capturing, and
    when ``param`` (the weight whose gradient ``fn`` computes) already holds a gradient: autograd
    would then accumulate into it with a kernel on the current stream, which must not race the
    side stream ("steal"-mode DDP and ``zero_grad(set_to_none=True)`` leave it None). ``param``
    may be a list when ``fn`` produces several parameters' gradients (weight and bias): every
    one of them must be gradient-free."""
    dev = inputs[0].device
    params = param if isinstance(param, (list, tuple)) else (param,)
    if not active(dev) or any(p is not None and p.grad is not None for p in params):
        return fn()
    main = torch.cuda.current_stream(dev)
    side = side_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in _tensors(inputs):
        if t.is_cuda:
            t.record_stream(side)
    for t in _tensors(out):
        if t.is_cuda:
            t.record_stream(main)
    _arm_join(dev, main, side)
    return out


def _arm_join(dev: torch.device, main: torch.cuda.Stream, side: torch.cuda.Stream) -> None:
    idx = dev.index
    if idx in _ARMED:
        return
    _ARMED[idx] = side

    def join():
        main.wait_stream(side)
        _ARMED.pop(idx, None)

    torch.autograd.Variable._execution_engine.queue_callback(join)


def pending(device: torch.device):
    """The side stream if weight gradients were launched on it in the running backward, else None."""
    if device.type != "cuda":
        return None
    return _ARMED.get(device.index if device.index is not None else torch.cuda.current_device())


__all__ = ["run", "pending", "side_stream", "active", "ENABLED"]
