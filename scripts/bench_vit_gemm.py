#!/usr/bin/env python
"""ViT-B/16 weight-gradient GEMMs (bs 256: M = 50432 tokens, bf16): candidates per shape.

dW[N_out, N_in] = dY^T X with K = M = 50432 — a long-K, small-output GEMM: hipBLASLt's
256x256 tiles give only 36-108 workgroups for 256 CUs (the 312-431 us kernels of
profiles/r1_vit_b16_s61_steady.md). Candidates:
  torch     dy.t() @ x (hipBLASLt, bf16 out)
  torch32   torch.mm(dy.t(), x, out_dtype=fp32)
  bmmS      S-way split of K as a batched GEMM (fp32 out) + sum over the batch
  oursS     our split-K MFMA kernel (gemm_wgrad: fp32 partials + one reduce), S splits (0 = auto)
  bias      column sums of dY: torch .sum(0) vs ours (gelu_bwd_bias-style partials)
Prints one JSON line per (shape, candidate) with us and TFLOP/s.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops.gemm import conv1x1_wgrad_v2  # noqa: E402


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
    M = int(os.environ.get("VIT_TOKENS", str(256 * 197)))
    shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}
    for name, (no, ni) in shapes.items():
        dy = torch.randn(M, no, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, ni, device="cuda").to(torch.bfloat16)
        ref = torch.mm(dy.t().float(), x.float())
        flop = 2.0 * M * no * ni
        cands = {
            "torch": lambda: dy.t() @ x,
            "torch32": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32),
        }
        for s in (0, 4, 8, 16):
            cands[f"ours{s}"] = lambda s=s: conv1x1_wgrad_v2(dy, x, torch.bfloat16, splits=s or None)
        from fluxmpi_amd.ops.linear import weight_grad
        for s in (0, 4, 7, 9, 14, 28):
            cands[f"w256_{s}"] = lambda s=s: weight_grad(dy, x, torch.bfloat16, splits=s or None)
        for cname, fn in cands.items():
            try:
                out = fn()
                err = float((out.float() - ref).abs().max() / ref.abs().max())
                us = bench(fn)
                rec = {"shape": name, "M": M, "N_out": no, "N_in": ni, "cand": cname, "us": round(us, 1),
                       "tflops": round(flop / us / 1e6, 1), "rel_err": round(err, 5)}
            except Exception as e:  # noqa: BLE001
                rec = {"shape": name, "cand": cname, "error": repr(e)[:200]}
            print(json.dumps(rec), flush=True)
        bias = {"bias_torch": lambda: dy.sum(0), "bias_torch32": lambda: dy.float().sum(0)}
        for cname, fn in bias.items():
            us = bench(fn)
            print(json.dumps({"shape": name, "cand": cname, "us": round(us, 1),
                              "GBps": round(dy.numel() * 2 / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
