#!/usr/bin/env python
"""Our split-K weight-gradient kernel (gemm_wgrad) on the ResNet-50 (batch 256) weight gradients it
takes in the step (profiles/rd5m_resnet50_choices.jsonl), in the (variant, target-workgroups)
configurations of the autotune: best of 3 interleaved rounds per shape, us -> one JSON line per
shape plus a total. Runs on a variant build too (FLUXMPI_C_VARIANT, scripts/diag/load_variant.py)
for a same-box A/B. Each shape is checked against an fp32 reference first."""
import json
import os
import sys

import torch

ROOT = __file__.rsplit("/scripts/", 1)[0]
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "diag"))
import load_variant  # noqa: E402

load_variant.install()
from fluxmpi_amd.ops import conv_choice as CC  # noqa: E402
from fluxmpi_amd.ops import gemm as G  # noqa: E402

# (kind, (n, ci, h, w), co, stride, calls per step)
SHAPES = [("1x1", (256, 64, 56, 56), 64, 1, 1), ("1x1", (256, 64, 56, 56), 256, 1, 4),
          ("1x1", (256, 256, 56, 56), 64, 1, 2), ("1x1", (256, 256, 56, 56), 128, 1, 1),
          ("1x1", (256, 128, 28, 28), 512, 1, 4), ("1x1", (256, 512, 28, 28), 128, 1, 3),
          ("1x1", (256, 256, 14, 14), 1024, 1, 6), ("1x1", (256, 1024, 14, 14), 256, 1, 5),
          ("1x1", (256, 1024, 14, 14), 512, 1, 1), ("1x1", (256, 512, 7, 7), 2048, 1, 3),
          ("1x1", (256, 2048, 7, 7), 512, 1, 2), ("3x3", (256, 128, 28, 28), 128, 1, 3),
          ("3x3", (256, 256, 14, 14), 256, 1, 5), ("3x3", (256, 512, 7, 7), 512, 1, 2),
          ("3x3s2", (256, 128, 56, 56), 128, 2, 1), ("3x3s2", (256, 256, 28, 28), 256, 2, 1),
          ("3x3s2", (256, 512, 14, 14), 512, 2, 1), ("ds", (256, 256, 56, 56), 512, 2, 1),
          ("ds", (256, 512, 28, 28), 1024, 2, 1), ("ds", (256, 1024, 14, 14), 2048, 2, 1)]


def t_us(fn, iters=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def make(kind, xs, co, stride):
    n, ci, h, w = xs
    ho, wo = (h + 1) // 2 if stride == 2 else h, (w + 1) // 2 if stride == 2 else w
    x = (torch.rand(n, ci, h, w, device="cuda") * 2 - 1).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = (torch.rand(n, co, ho, wo, device="cuda") * 2 - 1).bfloat16().contiguous(memory_format=torch.channels_last)
    if kind == "1x1":
        d2, x2 = dy.permute(0, 2, 3, 1).reshape(-1, co), x.permute(0, 2, 3, 1).reshape(-1, ci)
        return (lambda: G.conv1x1_wgrad_v2(d2, x2)), (lambda: d2.float().t() @ x2.float())
    if kind == "ds":
        d2 = dy.permute(0, 2, 3, 1).reshape(-1, co)
        xs2 = x[:, :, ::2, ::2].permute(0, 2, 3, 1).reshape(-1, ci)
        return (lambda: G.conv1x1_wgrad_s2(d2, x)), (lambda: d2.float().t() @ xs2.float())
    wt = torch.zeros(co, ci, 3, 3, device="cuda")
    ref = (lambda: torch.ops.aten.convolution_backward(dy.float(), x.float(), wt, None, [stride] * 2, [1, 1], [1, 1],
                                                         False, [0, 0], 1, [False, True, False])[1])
    fn = (lambda: G.conv3x3_wgrad(dy, x)) if kind == "3x3" else (lambda: G.conv3x3_wgrad_s2(dy, x))
    return fn, ref


def main():
    total = 0.0
    tag = os.environ.get("FLUXMPI_C_VARIANT", "tree")
    for kind, xs, co, stride, calls in SHAPES:
        fn, ref = make(kind, xs, co, stride)
        r = ref().float()
        d = fn().float().reshape(r.shape)
        err = float((d - r).norm() / r.norm())
        assert err < 1e-2, (kind, xs, co, err)
        best = {}
        for _ in range(3):
            for cfg in CC._WG_CONFIGS:
                best.setdefault(cfg, []).append(CC._with_cfg(cfg, lambda: t_us(fn)))
        (cfg, ts) = min(best.items(), key=lambda kv: min(kv[1]))
        us = min(ts)
        total += us * calls
        print(json.dumps({"build": tag, "kind": kind, "x": list(xs), "co": co, "calls": calls, "err": round(err, 5),
                          "best_cfg": list(cfg), "us": round(us, 1),
                          "all_us": {str(k): round(min(v), 1) for k, v in best.items()}}), flush=True)
    print(json.dumps({"build": tag, "total_us_per_step": round(total, 1)}), flush=True)


if __name__ == "__main__":
    main()
