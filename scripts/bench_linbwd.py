#!/usr/bin/env python
"""ViT-B/16 Linear backward GEMMs (M = 50432 tokens): one linbwd.hip launch (input + weight gradient,
planned split / order, and a sweep) against the round-5 pair (hipBLASLt input gradient + wgrad256
weight gradient + its reduce). JSON lines.   python scripts/bench_linbwd.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t_us(fn, iters=20, reps=3):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / iters)
    return best


def main():
    from fluxmpi_amd.ops import _ext
    from fluxmpi_amd.ops.conv_choice import _LB_CHOICE
    from fluxmpi_amd.ops.linear import dgrad_wgrad, weight_grad
    from fluxmpi_amd.ops.multi_tensor import DTYPE_CODE
    C = _ext.get(required=True)
    M = 50432
    for name, N, K in (("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768)):
        dy = torch.randn(M, N, device="cuda").bfloat16()
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        flops = 2 * 2.0 * M * N * K
        old = t_us(lambda: (dy @ w, weight_grad(dy, x, torch.bfloat16)))
        new = t_us(lambda: dgrad_wgrad(dy, x, w, torch.bfloat16))
        sp, first = [v for k, v in _LB_CHOICE.items() if k[:3] == (M, N, K)][0], 0
        rec = {"shape": name, "M": M, "N": N, "K": K, "old_us": round(old, 1), "new_us": round(new, 1),
               "plan": [sp, first], "old_tfs": round(flops / old / 1e6, 1), "new_tfs": round(flops / new / 1e6, 1)}
        # the input gradient alone and the weight gradient alone on the new kernel, and a sweep
        s = torch.cuda.current_stream().cuda_stream
        dx = torch.empty(M, K, device="cuda").bfloat16()
        rec["dgrad_only_us"] = round(t_us(lambda: C.linear_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), dx.data_ptr(),
                                                                0, M, N, K, N, K, K, K, 1, 1, s)), 1)
        rec["hipblaslt_dgrad_us"] = round(t_us(lambda: dy @ w), 1)
        sweep = {}
        for spx in (4, 8, 12, 16, 24, 32):
            se = C.linear_bwd_splits(M, N, K, spx)
            ws = torch.empty(se, N, K, device="cuda")
            for fx in (0, 1):
                def run():
                    C.linear_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), dx.data_ptr(), ws.data_ptr(), M, N, K, N, K,
                                 K, K, spx, fx, s)
                    C.gemm_splitk_reduce(ws.data_ptr(), se, N * K, dx.data_ptr(), DTYPE_CODE[torch.bfloat16], s)
                sweep[f"s{se}_{'dg' if fx else 'wg'}first"] = round(t_us(run), 1)
        rec["sweep_us"] = sweep
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
