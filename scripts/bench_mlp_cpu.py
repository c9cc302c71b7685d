#!/usr/bin/env python
"""BASELINE.json config #1: the reference README's 4-layer Dense MLP on CPU ranks.

The reference (``README.md:32-72``) trains Dense(1=>256,tanh)->Dense(256=>512,tanh)->
Dense(512=>256,tanh)->Dense(256=>1) on 16 samples per rank with
``DistributedOptimizer(Adam(0.001))`` for 100 epochs and prints the elapsed time; it
publishes no value. Here the same loop runs through the reference-shaped functional API
(``synchronize``, ``DistributedOptimizer``, ``Optimisers.update_``) over gloo, and rank 0
prints one JSON line with the step time (max over ranks): the per-epoch ``fluxmpi_println``
of the README (a rank-ordered, barrier-per-rank collective) is timed separately, since it
dominates a step this small.

Run: ``python -m fluxmpi_amd.launch -n 2 scripts/bench_mlp_cpu.py``
"""
import json
import os
import sys
import time

import torch
from torch.func import functional_call

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fluxmpi_amd as FluxMPI  # noqa: E402
from fluxmpi_amd import optimisers as O  # noqa: E402
from fluxmpi_amd.models import mlp  # noqa: E402


def run(epochs: int, println: bool):
    dev = FluxMPI.device()
    model = mlp().to(dev)
    torch.manual_seed(FluxMPI.local_rank())
    ps = {n: torch.randn_like(p) * 0.1 for n, p in model.named_parameters()}
    ps = FluxMPI.synchronize(ps, root_rank=0)
    x = torch.rand(1, 16, device=dev).T.contiguous()
    y = x ** 2
    opt = FluxMPI.DistributedOptimizer(O.Adam(0.001))
    st_opt = FluxMPI.synchronize(O.setup(opt, ps), root_rank=0)

    def loss(p):
        return ((functional_call(model, p, (x,)) - y) ** 2).sum()

    FluxMPI.barrier()
    t1 = time.perf_counter()
    for epoch in range(1, epochs + 1):
        for v in ps.values():
            v.requires_grad_(True)
        l = loss(ps)
        if println:
            FluxMPI.fluxmpi_println(f"Epoch {epoch}: Loss {l.item()}", file=open(os.devnull, "w"))
        gs = dict(zip(ps.keys(), torch.autograd.grad(l, list(ps.values()))))
        ps = {k: v.detach() for k, v in ps.items()}
        st_opt, ps = O.update_(st_opt, ps, gs)
    FluxMPI.barrier()
    dt = time.perf_counter() - t1
    dt = FluxMPI.allreduce(torch.tensor([dt], dtype=torch.float64), max).item()
    return dt, float(l)


def main():
    torch.set_num_threads(1)
    FluxMPI.Init()
    epochs = int(os.environ.get("MLP_EPOCHS", "100"))
    run(5, False)  # warm-up
    dt_plain, l1 = run(epochs, False)
    dt_print, l2 = run(epochs, True)
    if FluxMPI.local_rank() == 0:
        print(json.dumps({
            "metric": "README MLP step time (reference README.md:32-72), CPU, gloo",
            "config": {"model": "Dense 1-256-512-256-1 tanh", "per_rank_batch": 16, "optimizer": "DistributedOptimizer(Adam(1e-3))",
                       "world": FluxMPI.total_workers(), "backend": FluxMPI.backend_name(), "epochs": epochs,
                       "torch_threads": 1},
            "ms_per_step": round(1000 * dt_plain / epochs, 3),
            "ms_per_step_with_println": round(1000 * dt_print / epochs, 3),
            "total_s_100_epochs_with_println": round(dt_print * 100 / epochs, 3),
            "final_loss": round(l1, 6), "data": "synthetic (rand 16 x 1, y = x^2)",
        }), flush=True)
    FluxMPI.Finalize()


if __name__ == "__main__":
    main()
