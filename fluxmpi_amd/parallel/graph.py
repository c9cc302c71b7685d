"""HIP-graph capture of a whole data-parallel training step.

A ResNet-50 step is ~600 kernel launches; at small per-GPU batches the host
launch rate (~3-4 µs per launch) becomes the limit. ``GraphedStep`` captures
forward + loss + backward (including the hook-driven bucket allreduces on the
communicator's stream) + the fused optimiser + gradient zeroing into one HIP
graph and replays it with a single launch per step.

Requirements (as for any HIP graph): static shapes, inputs copied into the
captured input tensors (``step(x, y)`` does that), no host synchronisation
inside the step. The optimiser's step-dependent scalars already live on the
device (``DDP.hyper``), so replays advance Adam's bias correction correctly.
"""
from __future__ import annotations

import torch

from .ddp import DDP


class GraphedStep:
    """``step = GraphedStep(ddp, loss_fn, x, y); loss = step(x, y)``.

    ``loss_fn(ddp, x, y) -> loss`` must only do tensor work. ``warmup`` eager
    iterations run on a side stream before capture (allocator / autotune
    warm-up); they are real optimisation steps.
    """

    def __init__(self, ddp: DDP, loss_fn, *example_inputs, warmup: int = 3):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a GPU")
        self.ddp = ddp
        self.loss_fn = loss_fn
        self.static_inputs = [t.clone() for t in example_inputs]
        dev = self.static_inputs[0].device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        wd = ddp.watchdog
        if wd is not None:
            wd.pause()  # event queries from the watchdog thread are illegal during capture
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph):
                self.static_loss = self._eager()
        finally:
            if wd is not None:
                wd.resume()
        ddp.step_count -= 1  # capture records the step but executes nothing
        self.replays = 0

    def _eager(self):
        loss = self.loss_fn(self.ddp, *self.static_inputs)
        loss.backward()
        self.ddp.step()
        return loss.detach()

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        self.ddp.step_count += 1
        return self.static_loss
