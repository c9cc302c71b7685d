#!/usr/bin/env python
"""ViT-B/16 Linear GEMMs (batch 256: M = 50432 tokens): gemm256.hip vs hipBLASLt (torch), TFLOP/s.

usage: python scripts/bench_gemm256.py  -> JSON lines (one per shape and op)
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import gemm256 as G  # noqa: E402


def t_us(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def main():
    from fluxmpi_amd.ops import _ext
    C = _ext.get(required=True)
    M = 50432
    shapes = [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]
    for bk in (64, 32):
        C.gemm256_set_bk(bk)
        run(M, shapes, bk)
    C.gemm256_set_bk(64)


def run(M, shapes, bk):
    for name, k, n in shapes:
        x = torch.randn(M, k, device="cuda").bfloat16()
        w = (torch.randn(n, k, device="cuda") * k ** -0.5).bfloat16()
        b = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(M, n, device="cuda").bfloat16()
        fl = 2.0 * M * n * k
        rec = {"shape": name, "M": M, "N": n, "K": k, "bk": bk}
        rec["fwd_ours_us"] = t_us(lambda: G.linear_fwd(x, w, b, gelu=(name == "fc1")))
        rec["fwd_blas_us"] = t_us(lambda: torch.nn.functional.linear(x, w, b))
        rec["dgrad_ours_us"] = t_us(lambda: G.linear_dgrad(dy, w))
        rec["dgrad_blas_us"] = t_us(lambda: dy @ w)
        if name == "fc2":
            h = torch.randn(M, k, device="cuda").bfloat16()
            rec["dgrad_gelu_ours_us"] = t_us(lambda: G.linear_dgrad(dy, w, gelu_h=h))
        for key in [kk for kk in rec if kk.endswith("_us")]:
            rec[key.replace("_us", "_tfs")] = round(fl / rec[key] / 1e6, 1)
            rec[key] = round(rec[key], 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
