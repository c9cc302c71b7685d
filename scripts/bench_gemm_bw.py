#!/usr/bin/env python
"""Achieved HBM bandwidth of the memory-bound 1x1-convolution GEMMs of ResNet-50 (batch 256,
bf16 NHWC) on the LDS-DMA kernel, per epilogue: forward + BN statistics, input gradient +
masked residual (conv1 of an identity block), input gradient + BN-backward reductions (conv3).

usage: python scripts/bench_gemm_bw.py [batch] [engine ...]   (one JSON line per case)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops.gemm import SHARDS, gemm  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    engines = [int(e) for e in sys.argv[2:]] or [0]
    dev = "cuda"
    bf = dict(device=dev, dtype=torch.bfloat16)
    tot = {}
    for H, w in ((56, 64), (28, 128), (14, 256), (7, 512)):
        M = B * H * H
        c4 = 4 * w
        x4 = torch.randn(M, c4, **bf)           # block input / conv1 dgrad output
        xw = torch.randn(M, w, **bf)            # width-channel activation
        w1 = (torch.randn(w, c4, device=dev) * 0.05).to(torch.bfloat16)   # conv1 [w][4w]
        w3 = (torch.randn(c4, w, device=dev) * 0.05).to(torch.bfloat16)   # conv3 [4w][w]
        w1t, w3t = w1.t().contiguous(), w3.t().contiguous()
        stats4 = torch.zeros(SHARDS, 2, c4, device=dev)
        statsw = torch.zeros(SHARDS, 2, w, device=dev)
        mask = torch.randint(0, 256, (M * c4 // 8,), device=dev, dtype=torch.uint8)
        f32 = dict(device=dev, dtype=torch.float32)
        bnw, bnb, mean, inv = torch.ones(w, **f32), torch.zeros(w, **f32), torch.zeros(w, **f32), torch.ones(w, **f32)
        out4 = torch.empty(M, c4, **bf)
        outw = torch.empty(M, w, **bf)
        E = 2
        cases = {
            # name: (fn, bytes)
            "fwd1_stats": (lambda: gemm(x4, w1, outw, M=M, N=w, K=c4, lda=c4, ldb=c4, ldc=w, mode=1, stats=statsw,
                                        engine=E), M * (c4 + w) * 2),
            "fwd3_stats": (lambda: gemm(xw, w3, out4, M=M, N=c4, K=w, lda=w, ldb=w, ldc=c4, mode=1, stats=stats4,
                                        engine=E), M * (c4 + w) * 2),
            "dgrad1_res_mask": (lambda: gemm(xw, w1t, out4, M=M, N=c4, K=w, lda=w, ldb=w, ldc=c4, residual=x4,
                                             res_mask=mask, engine=E), M * (w + 2 * c4) * 2 + M * c4 // 8),
            "dgrad1_plain": (lambda: gemm(xw, w1t, out4, M=M, N=c4, K=w, lda=w, ldb=w, ldc=c4, engine=E),
                             M * (w + c4) * 2),
            "dgrad3_bnb": (lambda: gemm(x4, w3t, outw, M=M, N=w, K=c4, lda=c4, ldb=c4, ldc=w, mode=1, stats=statsw,
                                        bn_bwd=(xw, bnw, bnb, mean, inv, None, 2), engine=E), M * (c4 + 2 * w) * 2),
            "dgrad3_plain": (lambda: gemm(x4, w3t, outw, M=M, N=w, K=c4, lda=c4, ldb=c4, ldc=w, engine=E),
                             M * (c4 + w) * 2),
        }
        for eng in engines:
            for name, (fn, nbytes) in cases.items():
                E = eng or 2
                us = bench(fn)
                r = {"H": H, "w": w, "case": name, "engine": E, "us": round(us, 1),
                     "TBps": round(nbytes / us / 1e6, 2)}
                tot[(name, E)] = tot.get((name, E), 0) + us
                print(json.dumps(r), flush=True)
    for (name, E), us in sorted(tot.items()):
        print(json.dumps({"total": name, "engine": E, "us": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
