#!/usr/bin/env python
"""Does the DEQ cell stay contractive under the bench's training? Runs the bench.py training loop
(fixed synthetic batch, Adam 1e-3, average=True) for --steps steps and prints per step: forward
solve iterations and final residual, adjoint iterations, the conv filters' largest output-channel
norm and n3's largest |gain|. FLUXMPI_DEQ_CONSTRAIN picks the constraint (models/deq.py).
    python scripts/diag_deq_contract.py --model deq --steps 40"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="deq")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--labels", default="random", choices=["random", "teacher"],
                    help="teacher: labels from a fixed random linear teacher on the 4x4-pooled input "
                         "(a learnable synthetic task) instead of independent random labels")
    ap.add_argument("--batches", type=int, default=1, help="distinct synthetic batches, cycled")
    ap.add_argument("--lr", type=float, default=1e-3, help="Adam learning rate")
    ap.add_argument("--solver", default="", help="DEQ solver overrides, k=v pairs (bench.py --deq-solver)")
    a = ap.parse_args()
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models import build_model
    from fluxmpi_amd.models import deq as D
    from fluxmpi_amd.parallel.ddp import DDP
    FluxMPI.Init()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    solver = {}
    for kv in filter(None, a.solver.split(",")):
        k, v = kv.split("=")
        solver[k.strip()] = int(v) if k.strip() in ("max_iter", "bwd_iter", "check_lag", "m", "bwd_m", "skip", "restart", "skip_detach") else float(v)
    model = build_model(a.model, **solver).to(dev, memory_format=torch.channels_last)
    for m in model.modules():
        if not (isinstance(m, torch.nn.modules.batchnorm._BatchNorm) or type(m).__name__ == "FusedBatchNorm2d"):
            for p in m.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    ddp = DDP(model, O.Adam(a.lr), average=True)
    cin, img = {"deq": (1, 28), "deq_cifar": (3, 32)}[a.model]
    g = torch.Generator(device=dev).manual_seed(0)
    data = []
    teacher = torch.randn(cin * (img // 4) ** 2, 10, device=dev, generator=g)
    for _ in range(a.batches):
        xb = torch.randn(a.batch, cin, img, img, device=dev, generator=g)
        if a.labels == "teacher":
            yb = (F.avg_pool2d(xb, 4).flatten(1) @ teacher).argmax(1)
        else:
            yb = torch.randint(0, 10, (a.batch,), device=dev, generator=g)
        data.append((xb.bfloat16().contiguous(memory_format=torch.channels_last), yb))
    cell = model.deq.f
    for s in range(a.steps):
        x, y = data[s % len(data)]
        loss = F.cross_entropy(ddp(x).float(), y)
        loss.backward()
        ddp.step()
        torch.cuda.synchronize()
        wn = max(float(c.weight.float().square().sum((1, 2, 3)).sqrt().max()) for c in (cell.conv1, cell.conv2))
        rec = {"model": a.model, "lr": a.lr, "labels": a.labels, "batches": a.batches, "constrain": D.CONSTRAIN, "step": s, "loss": round(float(loss), 4),
               "skip_res": float(model.deq.last_skip_res) if getattr(model.deq, "last_skip_res", None) is not None else None,
               "jac_reg": model.deq.jac_reg, "jr": float(model.deq.last_jr) if model.deq.last_jr is not None else None,
               "fwd_iters": model.deq.last_iters, "fwd_res": float(model.deq.last_res),
               "bwd_iters": model.deq.last_bwd_iters, "conv_norm_max": round(wn, 4), "max_norm": round(cell.max_norm, 4),
               "g3_absmax": round(float(cell.n3.weight.float().abs().max()), 4),
               "g1_absmax": round(float(cell.n1.weight.float().abs().max()), 4),
               "g2_absmax": round(float(cell.n2.weight.float().abs().max()), 4)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
