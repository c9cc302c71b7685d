"""High-performance DDP training loop (flat buckets, backward/comm overlap, fused Adam).

Run:  torchrun --nproc-per-node 8 examples/train_ddp.py --model resnet50 --batch 256 --steps 100
      python -m fluxmpi_amd.launch -n 2 examples/train_ddp.py --model resnet_tiny --batch 8 --image 32 (CPU)
"""
import argparse
import time

import torch
import torch.nn.functional as F

import fluxmpi_amd as FluxMPI
from fluxmpi_amd import optimisers as O
from fluxmpi_amd.models import build_model
from fluxmpi_amd.parallel.ddp import DDP
from fluxmpi_amd.utils.profiling import StepTimer

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet50")
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--image", type=int, default=224)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--lr", type=float, default=1e-3)
args = ap.parse_args()

FluxMPI.Init()
dev = FluxMPI.device()
kw = {"norm": "fused"} if args.model.startswith("resnet") and dev.type == "cuda" else {}
model = build_model(args.model, **kw).to(dev)
if dev.type == "cuda":
    model = model.to(memory_format=torch.channels_last)
    for m in model.modules():
        if not isinstance(m, (torch.nn.modules.batchnorm._BatchNorm, torch.nn.LayerNorm)):
            for p in m.parameters(recurse=False):
                p.data = p.data.bfloat16()
ddp = DDP(model, O.AdamW(args.lr, decay=1e-4), average=True)
if FluxMPI.local_rank() == 0:
    print("buckets:", ddp.bucket_summary())

dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
x = torch.randn(args.batch, 3, args.image, args.image, device=dev, dtype=dt)
if dev.type == "cuda":
    x = x.contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10 if args.model in ("resnet_tiny",) else 1000, (args.batch,), device=dev)
timer = StepTimer(dev)
t0 = time.time()
for step in range(args.steps):
    with timer.phase("forward"):
        loss = F.cross_entropy(ddp(x).float(), y)
    with timer.phase("backward"):
        loss.backward()
    with timer.phase("optimizer"):
        ddp.step()
    if step % 10 == 0:
        FluxMPI.fluxmpi_println(f"step {step} loss {loss.item():.4f}")
if FluxMPI.local_rank() == 0:
    print({k: round(v, 3) for k, v in timer.summary().items()}, "ms;",
          f"{args.steps * args.batch * FluxMPI.total_workers() / (time.time() - t0):.1f} samples/s")
FluxMPI.Finalize()
