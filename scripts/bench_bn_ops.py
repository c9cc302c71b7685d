#!/usr/bin/env python
"""Per-kernel timing of the fused BatchNorm ops on ResNet-50's bn1/bn2/bn3 shapes (batch 256,
bf16, NHWC): statistics (+finalize), normalise(+ReLU)(+residual), backward reduce+dx — with
the effective HBM bandwidth of each, to find the shapes that fall short of the streaming rate."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import _ext  # noqa: E402
from fluxmpi_amd.ops.batchnorm import _workspace  # noqa: E402


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
    C = _ext.get(required=True)
    B = 256
    st = torch.cuda.current_stream().cuda_stream
    # (channels, spatial, residual): bn1/bn2 shapes of every stage, then bn3
    shapes = [(64, 56, False), (128, 56, False), (128, 28, False), (256, 28, False), (256, 14, False),
              (512, 14, False), (512, 7, False), (256, 56, True), (512, 28, True), (1024, 14, True), (2048, 7, True)]
    tot = {}
    for ch, hw, res in shapes:
        x = torch.randn(B, hw, hw, ch, device="cuda").bfloat16()
        r = torch.randn_like(x) if res else None
        y = torch.empty_like(x)
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if res else None
        mask = torch.empty(x.numel() // 8, device="cuda", dtype=torch.uint8) if res else None
        w = torch.rand(ch, device="cuda") + 0.5
        b = torch.randn(ch, device="cuda") * 0.1
        rm, rv = torch.zeros(ch, device="cuda"), torch.ones(ch, device="cuda")
        mean, inv = torch.empty(ch, device="cuda"), torch.empty(ch, device="cuda")
        dw, db = torch.empty(ch, device="cuda"), torch.empty(ch, device="cuda")
        ws = _workspace(x)
        rows = x.numel() // ch
        p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        stats = lambda: C.bn_stats_finalize(x.data_ptr(), w.data_ptr(), b.data_ptr(), rm.data_ptr(), rv.data_ptr(),  # noqa: E731
                                            mean.data_ptr(), inv.data_ptr(), 0, 0, ws.data_ptr(), rows, ch, 0.1, 1e-5, 0,
                                            9, st, 0)
        apply = lambda: C.bn_apply(x.data_ptr(), y.data_ptr(), p(r), w.data_ptr(), b.data_ptr(), mean.data_ptr(),  # noqa: E731
                                   inv.data_ptr(), rows, ch, 1, p(mask), 9, st)
        stats()
        apply()
        bwd = lambda: C.bn_bwd(dy.data_ptr(), x.data_ptr(), 0, p(mask), w.data_ptr(), b.data_ptr(), mean.data_ptr(),  # noqa: E731
                               inv.data_ptr(), dx.data_ptr(), p(dres), dw.data_ptr(), db.data_ptr(), ws.data_ptr(),
                               rows, ch, 1, 9, st, 0)
        n = x.numel() * 2
        rec = {"C": ch, "hw": hw, "res": res, "MB": round(n / 2 ** 20, 1)}
        rec["stats_us"] = round(bench(stats), 1)
        rec["apply_us"] = round(bench(apply), 1)
        rec["bwd_us"] = round(bench(bwd), 1)
        rec["stats_TBps"] = round(n / rec["stats_us"] / 1e6, 2)
        rec["apply_TBps"] = round(n * (3 if res else 2) / rec["apply_us"] / 1e6, 2)
        # reduce pass reads dy, x (+ mask); dx pass reads dy, x (+ mask), writes dx (+ dres)
        rec["bwd_TBps"] = round(n * (6.125 if res else 5.0) / rec["bwd_us"] / 1e6, 2)
        for k in ("stats_us", "apply_us", "bwd_us"):
            tot[k] = round(tot.get(k, 0) + rec[k], 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total": tot}))


if __name__ == "__main__":
    main()
