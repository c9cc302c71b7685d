#!/usr/bin/env python
"""wgrad256.hip variants (3: hoisted addressing, 4: ping-pong schedule) on the ViT-B/16 weight
gradients dW = dY^T X (K = 50432 tokens) vs hipBLASLt, uniform [-1, 1) bf16 operands; every
variant checked against an fp32 matmul first. usage: python scripts/bench_wgrad.py -> JSON lines"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import _ext  # noqa: E402
from fluxmpi_amd.ops.linear import weight_grad  # noqa: E402


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
    K = 50432
    for name, n_out, n_in in (("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)):
        dy = (torch.rand(K, n_out, device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand(K, n_in, device="cuda") * 2 - 1).bfloat16()
        ref = dy.float().t() @ x.float()
        rec = {"shape": name, "M": n_out, "N": n_in, "K": K}
        for v in (3, 4):
            C.wgrad256_set_variant(v)
            dw = weight_grad(dy, x, torch.float32)
            err = float((dw - ref).abs().max() / ref.abs().max())
            if err > 1e-2:
                raise SystemExit(f"{name} variant {v}: wrong (rel max err {err})")
            rec[f"v{v}_err"] = round(err, 6)
        best: dict = {}
        fl = 2.0 * K * n_out * n_in
        for _ in range(3):
            best.setdefault("blas", []).append(t_us(lambda: dy.t() @ x))
            for v in (3, 4):
                C.wgrad256_set_variant(v)
                best.setdefault(f"v{v}", []).append(t_us(lambda: weight_grad(dy, x, torch.bfloat16)))
        C.wgrad256_set_variant(4)
        for k, vals in best.items():
            rec[k + "_us"] = round(min(vals), 1)
            rec[k + "_tfs"] = round(fl / min(vals) / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
