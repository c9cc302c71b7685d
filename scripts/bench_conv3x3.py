#!/usr/bin/env python
"""ResNet-50's 3x3 convolutions (batch 256, stride 1): the implicit-GEMM MFMA kernel vs MIOpen
(tuned find-db), forward and input gradient. One JSON line per shape and a total."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import gemm as G  # noqa: E402
from fluxmpi_amd.ops.gemm import conv1x1_wgrad_v2, conv3x3_dgrad, conv3x3_fwd, conv3x3_wgrad  # noqa: E402
from fluxmpi_amd.utils.miopen import install_tuned_db  # noqa: E402


WG_CFGS = tuple(tuple(int(t) for t in c.split(":")) for c in
                os.environ.get("BENCH_WG_CFGS", "1:768,2:768,1:1536,2:512").split(","))
ENGINES = tuple(int(e) for e in os.environ.get("BENCH_ENGINES", "2").split(","))


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
    B = int(os.environ.get("BENCH_BATCH", "256"))
    tot = {}
    for H, C in [(56, 64), (28, 128), (14, 256), (7, 512)]:
        x = torch.randn(B, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        y = torch.empty_like(x)
        flop = 2 * B * H * H * C * C * 9
        rec = {"H": H, "C": C}
        G.HALO = True
        rec["halo_fwd"] = bench(lambda: conv3x3_fwd(x, w, out=y))
        rec["halo_dgrad"] = bench(lambda: conv3x3_dgrad(dy, w, out=y))
        G.HALO = False
        for eng in ENGINES:
            G.ENGINE = eng
            rec[f"e{eng}_fwd"] = bench(lambda: conv3x3_fwd(x, w, out=y))
            rec[f"e{eng}_dgrad"] = bench(lambda: conv3x3_dgrad(dy, w, out=y))
        G.ENGINE = 2
        rec["ours_fwd"] = rec["e2_fwd"]
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
        rec["ours_fwd_affine"] = bench(lambda: conv3x3_fwd(x, w, in_affine=(sc, sh), out=y))
        rec["miopen_fwd"] = bench(lambda: F.conv2d(x, w, padding=1))
        rec["ours_dgrad"] = rec["e2_dgrad"]
        rec["miopen_dgrad"] = bench(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
        for v, tw in WG_CFGS:
            G.WGRAD_VARIANT, G.WGRAD_TARGET_WG = v, tw
            rec[f"ours_wgrad_v{v}_{tw}"] = bench(lambda: conv3x3_wgrad(dy, x))
        rec["miopen_wgrad"] = bench(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        for k in ("halo_fwd", "halo_dgrad", "ours_fwd", "miopen_fwd", "ours_dgrad", "miopen_dgrad"):
            rec[k + "_TF"] = round(flop / rec[k] / 1e6, 1)
        for k, v in rec.items():
            if k not in ("H", "C") and not k.endswith("_TF"):
                tot[k] = round(tot.get(k, 0.0) + v, 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": tot}))
    # 1x1 forward with / without the BN+ReLU prologue (conv3 of each stage: width -> 4 width)
    for H, ci in [(56, 64), (28, 128), (14, 256), (7, 512)]:
        x2 = torch.randn(B * H * H, ci, device="cuda").bfloat16()
        w2 = torch.randn(4 * ci, ci, device="cuda").bfloat16()
        y2 = torch.empty(B * H * H, 4 * ci, device="cuda", dtype=torch.bfloat16)
        sc, sh = torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda") * 0.1
        M = B * H * H
        rec = {"H": H, "Cin": ci, "Cout": 4 * ci,
               "fwd1": bench(lambda: G.gemm(x2, w2, y2, M=M, N=4 * ci, K=ci, lda=ci, ldb=ci, ldc=4 * ci)),
               "fwd1_affine": bench(lambda: G.gemm(x2, w2, y2, M=M, N=4 * ci, K=ci, lda=ci, ldb=ci, ldc=4 * ci,
                                                  a_affine=(sc, sh)))}
        print(json.dumps(rec), flush=True)
    # 1x1 weight gradients (ResNet-50 bottleneck shapes)
    tot1 = {}
    for H, ci, co in [(56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
                      (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]:
        x = torch.randn(B, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(B, co, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, ci, 1, 1, device="cuda").bfloat16()
        x2, dy2 = x.permute(0, 2, 3, 1).reshape(-1, ci), dy.permute(0, 2, 3, 1).reshape(-1, co)
        rec = {"H": H, "Cin": ci, "Cout": co}
        for v, tw in WG_CFGS:
            G.WGRAD_VARIANT, G.WGRAD_TARGET_WG = v, tw
            rec[f"ours_wgrad1_v{v}_{tw}"] = bench(lambda: conv1x1_wgrad_v2(dy2, x2))
        rec["miopen_wgrad1"] = bench(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
        for k, v in rec.items():
            if "wgrad" in k:
                tot1[k] = round(tot1.get(k, 0.0) + v, 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us_wgrad1": tot1}))


if __name__ == "__main__":
    main()
