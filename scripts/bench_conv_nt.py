#!/usr/bin/env python
"""ResNet-50 (batch 256) convolutions on the 256x256 persistent kernel (gemm_nt.hip: implicit-GEMM
3x3, 1x1 as plain NT GEMMs, BatchNorm-statistics epilogue) vs the 128-tile LDS-DMA kernel
(gemm_glds.hip) and MIOpen (F.conv2d), interleaved rounds in one process, TFLOP/s.

Every path is checked against an fp32 F.conv2d of the same bf16 operands, and the statistics
epilogue against the column sums of its own output, before it is timed.

usage: python scripts/bench_conv_nt.py  -> JSON lines
"""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import gemm as G  # noqa: E402
from fluxmpi_amd.ops import gemm_nt as NT  # noqa: E402


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


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def check(name, got, ref, tol=1e-2):
    err = rel(got, ref)
    print(json.dumps({"check": name, "rel_err": round(err, 6), "ok": err < tol}), flush=True)
    if err >= tol:
        raise SystemExit(f"{name}: wrong result ({err})")


def nhwc(n, c, h, w):
    return (torch.rand(n, c, h, w, device="cuda") * 2 - 1).bfloat16().contiguous(memory_format=torch.channels_last)


def main():
    B = 256
    # (name, H, W, Cin, Cout, kind): the stride-1 3x3 convolutions of stages 3-4 (forward and input
    # gradient have the same shape) and the 1x1 convolutions whose widths tile by 256
    shapes = [("s3_3x3", 14, 14, 256, 256, 3), ("s4_3x3", 7, 7, 512, 512, 3),
              ("s2_3x3_c128", 28, 28, 128, 128, 3),
              ("s3_1x1_expand", 14, 14, 256, 1024, 1), ("s3_1x1_reduce", 14, 14, 1024, 256, 1),
              ("s4_1x1_expand", 7, 7, 512, 2048, 1), ("s4_1x1_reduce", 7, 7, 2048, 512, 1),
              ("s2_1x1_expand", 28, 28, 128, 512, 1), ("s2_1x1_reduce", 28, 28, 512, 128, 1),
              ("s1_1x1_expand", 56, 56, 64, 256, 1), ("s1_1x1_reduce", 56, 56, 256, 64, 1)]
    for name, h, w, ci, co, k in shapes:
        x = nhwc(B, ci, h, w)
        wt = (torch.randn(co, ci, k, k, device="cuda") * (ci * k * k) ** -0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        M = B * h * w
        fl = 2.0 * M * co * ci * k * k
        ref = F.conv2d(x.float(), wt.float(), padding=k // 2)
        stats = torch.zeros(G.SHARDS, 2, co, device="cuda", dtype=torch.float32)
        rec = {"shape": name, "M": M, "N": co, "K": ci * k * k}
        x2 = x.permute(0, 2, 3, 1).reshape(M, ci)
        w2 = wt.reshape(co, ci) if k == 1 else None

        def run(nt, st=None):
            NT.CONV = nt
            if k == 3:
                return G.conv3x3_fwd(x, wt, stats=st)
            return G.conv1x1_fwd(x2, w2, stats=st)

        NT.CONV = True
        NT.MIN_TILES, NT.MIN_K = 0, 0  # measure every shape the kernel supports (routing thresholds off)
        ok_nt = NT.conv_ok(M, ci, co, x) if k == 3 else NT.gemm_ok(M, co, ci, x2)
        rec["nt_supported"] = bool(ok_nt)
        paths = [("glds", False)] + ([("nt", True)] if ok_nt else [])
        for tag, nt in paths:
            stats.zero_()
            y = run(nt, stats)
            torch.cuda.synchronize()
            y4 = y if k == 3 else y.view(B, h, w, co).permute(0, 3, 1, 2)
            check(f"{name}_{tag}", y4, ref)
            yf = y4.float().permute(0, 2, 3, 1).reshape(M, co)
            check(f"{name}_{tag}_sum", stats[:, 0].sum(0), yf.sum(0), tol=2e-3)
            check(f"{name}_{tag}_sumsq", stats[:, 1].sum(0), (yf * yf).sum(0), tol=2e-3)
        best: dict = {}
        for _ in range(3):
            best.setdefault("miopen", []).append(t_us(lambda: F.conv2d(x, wt, padding=k // 2)))
            for tag, nt in paths:
                best.setdefault(tag, []).append(t_us(lambda: run(nt, stats)))
        for key, v in best.items():
            us = min(v)
            rec[key + "_us"] = round(us, 1)
            rec[key + "_tfs"] = round(fl / us / 1e6, 1)
        print(json.dumps(rec), flush=True)
        del x, wt, ref, y, x2
        torch.cuda.empty_cache()
    NT.CONV = True
    NT.MIN_TILES, NT.MIN_K = 0, 0
    # input gradients of the 3x3 shapes (the flipped-transpose filter, same kernel)
    for name, h, w, ci, co in (("s3_3x3_dgrad", 14, 14, 256, 256), ("s4_3x3_dgrad", 7, 7, 512, 512)):
        dy = nhwc(B, co, h, w)
        wt = (torch.randn(co, ci, 3, 3, device="cuda") * (ci * 9) ** -0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        G.note_filter(wt)
        ref = torch.nn.grad.conv2d_input((B, ci, h, w), wt.float(), dy.float(), padding=1)
        rec = {"shape": name}
        for tag, nt in (("glds", False), ("nt", True)):
            NT.CONV = nt
            dx = G.conv3x3_dgrad(dy, wt)
            torch.cuda.synchronize()
            check(f"{name}_{tag}", dx, ref)
            rec[tag + "_us"] = round(min(t_us(lambda: G.conv3x3_dgrad(dy, wt)) for _ in range(3)), 1)
        print(json.dumps(rec), flush=True)
    NT.CONV = True


if __name__ == "__main__":
    main()
