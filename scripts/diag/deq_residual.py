"""Forward fixed-point residual of the random-init DEQ models against the iteration count
(Anderson, synchronous test, no graphs): does the solve converge, and to what?

    python scripts/diag/deq_residual.py [--model deq_cifar|deq] [--batch 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="deq_cifar")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--m", type=int, default=5)
    ap.add_argument("--beta", type=float, default=1.0)
    ap.add_argument("--lam", type=float, default=1e-4)
    ap.add_argument("--iters", default="5,10,15,20,30,45,60,90")
    ap.add_argument("--picard", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    import torch
    from fluxmpi_amd.models import deq as D
    torch.manual_seed(0)
    if a.model == "deq_cifar":
        m = D.deq_cifar()
        x = torch.randn(a.batch, 3, 32, 32)
    else:
        m = D.deq_mnist()
        x = torch.randn(a.batch, 1, 28, 28)
    m = m.to(a.device, memory_format=torch.channels_last)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    for mod in m.modules():  # as bench.py: bf16 except the BatchNorms
        if not (isinstance(mod, torch.nn.modules.batchnorm._BatchNorm) or type(mod).__name__ == "FusedBatchNorm2d"):
            for p in mod.parameters(recurse=False):
                p.data = p.data.to(dt)
    x = x.to(a.device).to(dt).contiguous(memory_format=torch.channels_last)
    deq = m.deq
    captured = {}
    orig = deq._forward

    def grab(xx, gs=None):
        captured["x"] = xx.detach()
        return orig(xx, gs)

    deq._forward = grab
    with torch.no_grad():
        m(x)
    xin = captured["x"]
    raw = deq.f.manual_ok(xin)
    fz = D._CellEval(deq.f, xin, raw)
    with torch.no_grad(), D.fp32_affine_cache(deq.f):
        for it in map(int, a.iters.split(",")):
            _, k, res = D.anderson(fz, torch.zeros_like(xin), m=a.m, lam=a.lam, beta=a.beta, max_iter=it, tol=0.0,
                                   check_lag=0)
            print(json.dumps({"model": a.model, "m": a.m, "beta": a.beta, "lam": a.lam, "max_iter": it, "iters": k,
                              "rel_residual": float(res)}), flush=True)
        if not a.picard:
            return
        # plain (undamped) fixed-point iteration for comparison
        z = torch.zeros_like(xin)
        for k in range(1, 61):
            fzv = fz(z)
            if k in (5, 10, 20, 30, 60):
                r = float((fzv.float() - z.float()).norm() / (1e-5 + fzv.float().norm()))
                print(json.dumps({"model": a.model, "picard_iter": k, "rel_residual": r}), flush=True)
            z = fzv


if __name__ == "__main__":
    main()
