"""The v0.5.3 API (reference ``README.md:110-112``): no DistributedOptimizer, call
``allreduce_gradients(gs)`` before every plain optimiser update; data sharded
with ``DistributedDataContainer`` (guide steps 1-6, ``docs/src/guide.md``).

Run:  python -m fluxmpi_amd.launch -n 2 examples/allreduce_gradients_api.py
"""
import torch

import fluxmpi_amd as FluxMPI
from fluxmpi_amd import optimisers as O

FluxMPI.Init()                                                      # 1. initialise
dev = FluxMPI.device()
torch.manual_seed(0)
model = torch.nn.Sequential(torch.nn.Linear(8, 32), torch.nn.ReLU(), torch.nn.Linear(32, 1)).to(dev)
model = FluxMPI.synchronize(FluxMPI.FluxMPIFluxModel(model), root_rank=0)   # 2. sync parameters

X = torch.randn(1000, 8)
Y = X.sum(1, keepdim=True).sin()
data = FluxMPI.DistributedDataContainer(list(zip(X, Y)))           # 3. shard the data
loader = torch.utils.data.DataLoader(data, batch_size=50, shuffle=True)

st = O.setup(O.Adam(1e-3), model)                                   # 4. plain optimiser ...
st = FluxMPI.synchronize(st, root_rank=0)                           # 5. ... with synced state

for epoch in range(3):
    for xb, yb in loader:
        xb, yb = xb.to(dev), yb.to(dev)
        model.zero_grad()
        loss = ((model(xb) - yb) ** 2).mean() / FluxMPI.total_workers()  # SUM semantics: scale the loss
        loss.backward()
        gs = {n: p.grad for n, p in model.named_parameters()}
        gs = FluxMPI.allreduce_gradients(gs)                         # ... + explicit gradient allreduce
        st, model = O.update_(st, model, gs)
    if FluxMPI.local_rank() == 0:                                    # 6. log from rank 0 with plain print
        print(f"epoch {epoch}: loss {loss.item() * FluxMPI.total_workers():.4f}")
FluxMPI.Finalize()
