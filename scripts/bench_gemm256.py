#!/usr/bin/env python
"""ViT-B/16 Linear GEMMs (batch 256: M = 50432 tokens): gemm256.hip (pipeline / schedule variants,
interleaved in one process) vs hipBLASLt (torch), TFLOP/s.

usage: python scripts/bench_gemm256.py  -> JSON lines (one per shape, op and variant)
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import _ext  # noqa: E402
from fluxmpi_amd.ops import gemm256 as G  # noqa: E402

CONFIGS = [(64, 0), (64, 2), (64, 8), (64, 10), (32, 1)]


def t_us(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    C = _ext.get(required=True)
    M = 50432
    shapes = [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]
    for name, k, n in shapes:
        x = torch.randn(M, k, device="cuda").bfloat16()
        w = (torch.randn(n, k, device="cuda") * k ** -0.5).bfloat16()
        b = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(M, n, device="cuda").bfloat16()
        fl = 2.0 * M * n * k
        best: dict = {}
        for rnd in range(3):  # interleaved rounds: min over rounds per variant
            best.setdefault("fwd_blas", []).append(t_us(lambda: torch.nn.functional.linear(x, w, b)))
            best.setdefault("dgrad_blas", []).append(t_us(lambda: dy @ w))
            for bk, var in CONFIGS:
                C.gemm256_set_bk(bk)
                C.gemm256_set_var(var)
                best.setdefault(f"fwd_{bk}_{var}", []).append(t_us(lambda: G.linear_fwd(x, w, b)))
                best.setdefault(f"dgrad_{bk}_{var}", []).append(t_us(lambda: G.linear_dgrad(dy, w)))
        C.gemm256_set_bk(64)
        C.gemm256_set_var(0)
        rec = {"shape": name, "M": M, "N": n, "K": k}
        for key, v in best.items():
            us = min(v)
            rec[key + "_us"] = round(us, 1)
            rec[key + "_tfs"] = round(fl / us / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
