"""The reference README quick start (``README.md:32-70``), line for line in fluxmpi_amd.

Run:  python -m fluxmpi_amd.launch -n 3 examples/readme_quickstart.py
      (or torchrun --nproc-per-node 3 examples/readme_quickstart.py)

Julia                                            | here
-------------------------------------------------|--------------------------------------------
FluxMPI.Init()                                   | FluxMPI.Init()
ps, st = Lux.setup(rng, model) .|> gpu           | ps = {name: tensor} on FluxMPI.device()
ps = FluxMPI.synchronize!(ps; root_rank = 0)     | ps = FluxMPI.synchronize(ps, root_rank=0)
opt = DistributedOptimizer(Adam(0.001f0))        | opt = FluxMPI.DistributedOptimizer(O.Adam(0.001))
st_opt = Optimisers.setup(opt, ps)               | st_opt = O.setup(opt, ps)
st_opt = FluxMPI.synchronize!(st_opt; ...)       | st_opt = FluxMPI.synchronize(st_opt, root_rank=0)
l, back = Zygote.pullback(loss, ps)              | l = loss(ps); grads = torch.autograd.grad(l, ...)
st_opt, ps = Optimisers.update(st_opt, ps, gs)   | st_opt, ps = O.update_(st_opt, ps, gs)
"""
import time

import torch
from torch.func import functional_call

import fluxmpi_amd as FluxMPI
from fluxmpi_amd import optimisers as O
from fluxmpi_amd.models import mlp

FluxMPI.Init()
dev = FluxMPI.device()

model = mlp().to(dev)  # Dense(1=>256,tanh) -> Dense(256=>512,tanh) -> Dense(512=>256,tanh) -> Dense(256=>1)
torch.manual_seed(FluxMPI.local_rank())
ps = {n: torch.randn_like(p) * 0.1 for n, p in model.named_parameters()}
ps = FluxMPI.synchronize(ps, root_rank=0)

x = torch.rand(1, 16, device=dev).T.contiguous()
y = x ** 2

opt = FluxMPI.DistributedOptimizer(O.Adam(0.001))
st_opt = O.setup(opt, ps)


def loss(p):
    return ((functional_call(model, p, (x,)) - y) ** 2).sum()


st_opt = FluxMPI.synchronize(st_opt, root_rank=0)

t1 = time.time()
for epoch in range(1, 101):
    for v in ps.values():
        v.requires_grad_(True)
    l = loss(ps)
    FluxMPI.fluxmpi_println(f"Epoch {epoch}: Loss {l.item()}")
    gs = dict(zip(ps.keys(), torch.autograd.grad(l, list(ps.values()))))
    ps = {k: v.detach() for k, v in ps.items()}
    st_opt, ps = O.update_(st_opt, ps, gs)

FluxMPI.fluxmpi_println(time.time() - t1)
FluxMPI.Finalize()
