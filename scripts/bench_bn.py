#!/usr/bin/env python
"""Microbenchmark of the fused NHWC BatchNorm kernels on ResNet-50 shapes (bf16, batch 256).

Reports per-shape forward / backward time and effective HBM bandwidth, next to
the eager PyTorch composition (batch_norm + add + relu).
"""
import json
import sys

import torch
import torch.nn.functional as F

from fluxmpi_amd.ops.batchnorm import fused_batch_norm


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    shapes = [(64, 112, True, False), (64, 56, True, False), (256, 56, True, True), (128, 28, True, False),
              (512, 28, True, True), (256, 14, True, False), (1024, 14, True, True), (512, 7, True, False),
              (2048, 7, True, True), (2048, 7, False, False)]
    out = []
    for C, hw, relu, res in shapes:
        x = torch.randn(B, C, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x) if res else None
        w = torch.ones(C, device="cuda", requires_grad=True)
        b = torch.zeros(C, device="cuda", requires_grad=True)
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        xg = x.clone().requires_grad_()
        y = fused_batch_norm(xg, w, b, rm, rv, True, 0.1, 1e-5, relu, r)
        dy = torch.randn_like(y)
        t_fwd = bench(lambda: fused_batch_norm(x, w, b, rm, rv, True, 0.1, 1e-5, relu, r))
        t_bwd = bench(lambda: torch.autograd.grad(y, (xg, w, b), dy, retain_graph=True))

        def eager():
            o = F.batch_norm(x, rm, rv, w, b, True, 0.1, 1e-5)
            if r is not None:
                o = o + r
            return F.relu(o) if relu else o
        xe = x.clone().requires_grad_()
        t_eager_fwd = bench(eager)
        o = F.batch_norm(xe, rm, rv, w, b, True, 0.1, 1e-5)
        o = F.relu(o + r) if res else (F.relu(o) if relu else o)
        t_eager_bwd = bench(lambda: torch.autograd.grad(o, (xe, w, b), dy, retain_graph=True))
        n = x.numel() * 2
        fwd_bytes = n * (1 + 2 + (1 if res else 0))
        bwd_bytes = n * ((3 if relu else 2) * 2 + 1 + (1 if res else 0))
        rec = {"C": C, "hw": hw, "relu": relu, "res": res, "fwd_us": round(t_fwd, 1), "bwd_us": round(t_bwd, 1),
               "fwd_TBps": round(fwd_bytes / t_fwd / 1e6, 2), "bwd_TBps": round(bwd_bytes / t_bwd / 1e6, 2),
               "eager_fwd_us": round(t_eager_fwd, 1), "eager_bwd_us": round(t_eager_bwd, 1)}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    tot = {k: round(sum(r[k] for r in out), 1) for k in ("fwd_us", "bwd_us", "eager_fwd_us", "eager_bwd_us")}
    print(json.dumps({"total": tot}))


if __name__ == "__main__":
    main()
