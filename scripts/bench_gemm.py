#!/usr/bin/env python
"""1x1-convolution passes on ResNet-50 shapes (batch 256, bf16 NHWC): our MFMA GEMM
(fwd + BN stats epilogue, dgrad, split-K wgrad) vs MIOpen through PyTorch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops.gemm import SHARDS, conv1x1_dgrad, conv1x1_fwd, conv1x1_wgrad  # noqa: E402
from fluxmpi_amd.utils.miopen import install_tuned_db  # noqa: E402
import fluxmpi_amd.ops.gemm as G  # noqa: E402


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
    install_tuned_db()
    torch.backends.cudnn.benchmark = True
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    # (H, Cin, Cout) of the stride-1 1x1 convolutions of ResNet-50
    shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
              (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512), (7, 512, 2048), (7, 2048, 512)]
    tot = {"ours_fwd": 0, "miopen_fwd": 0, "ours_dgrad": 0, "miopen_dgrad": 0, "ours_wgrad": 0, "miopen_wgrad": 0,
           "fwd_nb1": 0, "fwd_nb2": 0, "dgrad_nb1": 0, "dgrad_nb2": 0, "wgrad_nb1": 0, "wgrad_nb2": 0}
    for H, ci, co in shapes:
        M = B * H * H
        x4 = torch.randn(B, ci, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w4 = (torch.randn(co, ci, 1, 1, device="cuda") * 0.05).to(torch.bfloat16)
        dy4 = torch.randn(B, co, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x2 = x4.permute(0, 2, 3, 1).reshape(M, ci)
        dy2 = dy4.permute(0, 2, 3, 1).reshape(M, co)
        w2 = w4.view(co, ci)
        stats = torch.zeros(SHARDS, 2, co, device="cuda")
        dwbuf = torch.zeros(co, ci, device="cuda")
        r = {"H": H, "Cin": ci, "Cout": co}
        r["ours_fwd"] = bench(lambda: conv1x1_fwd(x2, w2, None, stats))
        r["ours_fwd_nostats"] = bench(lambda: conv1x1_fwd(x2, w2, None, None))
        for nb in (1, 2):  # forced LDS buffering variants
            G.NBUF = nb
            r[f"fwd_nb{nb}"] = bench(lambda: conv1x1_fwd(x2, w2, None, stats))
            r[f"dgrad_nb{nb}"] = bench(lambda: conv1x1_dgrad(dy2, w2))
            r[f"wgrad_nb{nb}"] = bench(lambda: conv1x1_wgrad(dy2, x2, None, dwbuf))
        G.NBUF = 0
        r["miopen_fwd"] = bench(lambda: torch.nn.functional.conv2d(x4, w4))
        r["ours_dgrad"] = bench(lambda: conv1x1_dgrad(dy2, w2))
        r["ours_wgrad"] = bench(lambda: conv1x1_wgrad(dy2, x2, None, dwbuf))

        def bwd(mask):
            return torch.ops.aten.convolution_backward(dy4, x4, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                       mask)
        r["miopen_dgrad"] = bench(lambda: bwd([True, False, False]))
        r["miopen_wgrad"] = bench(lambda: bwd([False, True, False]))
        for k in tot:
            tot[k] += r[k]
        fl = 2 * M * ci * co
        r["ours_fwd_TF"] = round(fl / r["ours_fwd"] / 1e6, 1)
        r = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        print(json.dumps(r), flush=True)
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
