#!/usr/bin/env python
"""Tile-shape sweep of the MFMA GEMM on ResNet-50's 1x1-conv shapes (batch 256): forward
(K-major x K-major) and dgrad (K-major x N-major) with the 128/64 tile choices forced,
next to MIOpen's forward. Prints one JSON line per shape and a total."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops.gemm import gemm  # noqa: E402
from fluxmpi_amd.ops import gemm as G  # noqa: E402
from fluxmpi_amd.utils.miopen import install_tuned_db  # noqa: E402


ENGINES = tuple(int(e) for e in os.environ.get("BENCH_ENGINES", "1,2,3,5,6").split(","))


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
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    install_tuned_db()
    torch.backends.cudnn.benchmark = True
    B = 256
    shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
              (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512), (7, 512, 2048), (7, 2048, 512)]
    tiles = [(0, 0)]
    tot = {}
    for H, ci, co in shapes:
        M = B * H * H
        x = torch.randn(M, ci, device="cuda").bfloat16()
        w = (torch.randn(co, ci, device="cuda") * 0.05).bfloat16()
        dy = torch.randn(M, co, device="cuda").bfloat16()
        y = torch.empty(M, co, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(M, ci, device="cuda", dtype=torch.bfloat16)
        rec = {"H": H, "Cin": ci, "Cout": co}
        for eng in ENGINES:
            G.ENGINE = eng
            rec[f"fwd_e{eng}"] = bench(lambda: gemm(x, w, y, M=M, N=co, K=ci, lda=ci, ldb=ci, ldc=co))
        G.ENGINE = 0
        for tm, tn in tiles:
            rec[f"fwd_{tm}_{tn}"] = bench(lambda: gemm(x, w, y, M=M, N=co, K=ci, lda=ci, ldb=ci, ldc=co,
                                                       tile_m=tm, tile_n=tn))
            continue
            rec[f"dgrad_{tm}_{tn}"] = bench(lambda: gemm(dy, w, dx, M=M, N=ci, K=co, lda=co, ldb=ci, ldc=ci,
                                                         a_kmajor=True, b_kmajor=False, tile_m=tm, tile_n=tn))
        x4 = x.view(B, H, H, ci).permute(0, 3, 1, 2)
        w4 = w.view(co, ci, 1, 1)
        rec["miopen_fwd"] = bench(lambda: torch.nn.functional.conv2d(x4, w4))
        for k, v in rec.items():
            if k not in ("H", "Cin", "Cout"):
                tot[k] = round(tot.get(k, 0.0) + v, 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": tot}))
    # square TN GEMMs (compare with the guide's ladder)
    for n in (4096, 8192):
        a = torch.randn(n, n, device="cuda").bfloat16()
        b = torch.randn(n, n, device="cuda").bfloat16()
        c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        rec = {"square": n}
        for eng in ENGINES:
            G.ENGINE = eng
            us = bench(lambda: gemm(a, b, c, M=n, N=n, K=n, lda=n, ldb=n, ldc=n), iters=10)
            rec[f"e{eng}_TF"] = round(2 * n ** 3 / us / 1e6, 1)
        rec["hipblaslt_TF"] = round(2 * n ** 3 / bench(lambda: torch.matmul(a, b.t(), out=c), iters=10) / 1e6, 1)
        G.ENGINE = 0
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
