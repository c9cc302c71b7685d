#!/usr/bin/env python
"""conv1x1n (narrow-K 1x1 forward + statistics) vs the 128-tile LDS-DMA GEMM (+ statistics) vs
MIOpen (no statistics) at ResNet-50's stage-1 / 2 expansion shapes, batch 256; JSON lines."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import gemm as G  # noqa: E402


def t_us(fn, iters=20, repeats=3):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(repeats):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def main():
    torch.manual_seed(0)
    for (n, h, w, k, co) in [(256, 56, 56, 64, 256), (256, 28, 28, 128, 512), (256, 56, 56, 64, 64 * 4)]:
        m = n * h * w
        x = torch.randn(n, k, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(co, k, 1, 1, device="cuda") * k ** -0.5).bfloat16().contiguous(memory_format=torch.channels_last)
        x2, w2 = x.permute(0, 2, 3, 1).reshape(m, k), wt.reshape(co, k)
        y = torch.empty(m, co, device="cuda", dtype=torch.bfloat16)
        st = torch.zeros(G.SHARDS, 2, co, device="cuda")
        G.conv1x1n(x2, w2, y, st)
        ref = x2.float() @ w2.float().t()
        rel = float((y.float() - ref).norm() / ref.norm())
        yg = torch.empty(n, h, w, co, device="cuda", dtype=torch.bfloat16).permute(0, 3, 1, 2)
        ours = t_us(lambda: G.conv1x1n(x2, w2, y, st))
        ours_plain = t_us(lambda: G.conv1x1n(x2, w2, y))
        glds = t_us(lambda: G.gemm(x2, w2, yg, M=m, N=co, K=k, lda=k, ldb=k, ldc=co, a_kmajor=True, b_kmajor=True,
                                   mode=1, stats=st))
        mio = t_us(lambda: F.conv2d(x, wt))
        byts = m * (k + co) * 2
        rec = {"shape": [n, h, w, k, co], "rel": round(rel, 5), "n_stats_us": round(ours, 1),
               "n_stats_tbs": round(byts / ours / 1e6, 2), "n_plain_us": round(ours_plain, 1),
               "glds_stats_us": round(glds, 1), "miopen_us": round(mio, 1),
               "miopen_tbs": round(byts / mio / 1e6, 2)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
