#!/usr/bin/env python
"""Diagnose the DEQ solver graphs: after an in-place weight change, compare the graphed and eager
solve (z*), adjoint (u) and parameter gradients, fused and unfused cell. Prints one line per check."""
import sys
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fluxmpi_amd.models.deq as D  # noqa: E402
from fluxmpi_amd.ops import deq_cell  # noqa: E402


def build():
    torch.manual_seed(3)
    m = D.deq_mnist(max_iter=13, tol=0.0, bwd_iter=12, bwd_tol=0.0).cuda().to(memory_format=torch.channels_last)
    for mod in m.modules():
        if type(mod).__name__ != "FusedBatchNorm2d":
            for p in mod.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    return m


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def run(fused, graphs, steps=3):
    deq_cell.ENABLED = fused
    m = build()
    m.deq.use_graphs = graphs
    torch.manual_seed(7)
    x = torch.randn(32, 1, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    recs = []
    caught = {}
    orig = D.DEQFixedPoint._forward

    def spy(self, xx, gs=None):
        z = orig(self, xx, gs)
        caught["z"] = z.detach().clone()
        if z.requires_grad:
            z.register_hook(lambda g: caught.__setitem__("u", g.detach().clone()))
        return z

    D.DEQFixedPoint._forward = spy
    try:
        for step in range(steps):
            out = m(x)
            F.cross_entropy(out.float(), y).backward()
            torch.cuda.synchronize()
            recs.append((caught["z"], caught.get("u"), [p.grad.float().clone() for p in m.parameters()],
                         [n for n, _ in m.named_parameters()]))
            with torch.no_grad():
                for i, p in enumerate(m.parameters()):
                    p.grad = None
                    p.mul_(1.0 + 0.03 * ((i + step) % 3 - 1))
    finally:
        D.DEQFixedPoint._forward = orig
    return recs


for fused in (False, True):
    e1 = run(fused, False)
    e2 = run(fused, False)
    g = run(fused, True)
    for s in range(len(e1)):
        zs = (rel(e2[s][0], e1[s][0]), rel(g[s][0], e1[s][0]))
        worst_e = max(rel(a, b) for a, b in zip(e2[s][2], e1[s][2]))
        gr = [(rel(a, b), n) for a, b, n in zip(g[s][2], e1[s][2], e1[s][3])]
        worst_g = max(gr)
        ue = rel(g[s][1], e1[s][1]) if g[s][1] is not None else -1
        print(f"fused={fused} step={s} z* eager2 {zs[0]:.2e} graphed {zs[1]:.2e} | u graphed {ue:.2e} | grads "
              f"eager2 worst {worst_e:.2e} graphed worst {worst_g[0]:.2e} ({worst_g[1]})", flush=True)
        print("   per-param graphed:", " ".join(f"{n}={e:.1e}" for e, n in gr), flush=True)
