#!/usr/bin/env python
"""conv3x3n.hip (narrow-channel 3x3, halo staged once per tile) vs the 128-tile LDS-DMA implicit
GEMM (gemm_glds, the previous default) vs MIOpen, at the ResNet-50 stage-1 / stage-2 shapes
(batch 256): forward with the BatchNorm-statistics epilogue, and input gradient. Interleaved rounds,
best of 3, us and TFLOP/s -> JSON lines. Every kernel is checked against fp32 first."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import gemm as G  # noqa: E402


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
    torch.backends.cudnn.benchmark = True
    for (n, c, h, w) in [(256, 64, 56, 56), (256, 128, 28, 28)]:
        x = (torch.rand(n, c, h, w, device="cuda") * 2 - 1).bfloat16().contiguous(memory_format=torch.channels_last)
        wt = ((torch.rand(c, c, 3, 3, device="cuda") * 2 - 1) * (9 * c) ** -0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        M = n * h * w
        w2 = wt.permute(0, 2, 3, 1).contiguous()
        G.note_filter(wt)
        wtt = G.filter_t(wt)
        stats = torch.zeros(G.SHARDS, 2, c, device="cuda")
        y = torch.empty(n, h, w, c, device="cuda", dtype=torch.bfloat16).permute(0, 3, 1, 2)
        ref = F.conv2d(x.float(), wt.float(), padding=1)
        G.conv3x3n(x, w2, y, M, h, w, stats)
        err = float((y.float() - ref).norm() / ref.norm())
        assert err < 5e-3, err
        dref = torch.ops.aten.convolution_backward(x.float(), x.float(), wt.float(), None, [1, 1], [1, 1], [1, 1],
                                                   False, [0, 0], 1, [True, False, False])[0]
        dx = torch.empty_like(y)
        G.conv3x3n(x, wtt, dx, M, h, w)
        err2 = float((dx.float() - dref).norm() / dref.norm())
        assert err2 < 5e-3, err2
        fl = 2.0 * M * c * 9 * c
        arms = {
            "n_fwd_stats": lambda: G.conv3x3n(x, w2, y, M, h, w, stats),
            "n_fwd": lambda: G.conv3x3n(x, w2, y, M, h, w),
            "glds_fwd_stats": lambda: G.gemm(x, w2, y, M=M, N=c, K=9 * c, lda=c, ldb=9 * c, ldc=c, mode=1, stats=stats,
                                             conv=(h, w, c)),
            "miopen_fwd": lambda: F.conv2d(x, wt, None, 1, 1),
            "n_dgrad": lambda: G.conv3x3n(x, wtt, dx, M, h, w),
            "glds_dgrad": lambda: G.gemm(x, wtt, dx, M=M, N=c, K=9 * c, lda=c, ldb=9 * c, ldc=c, conv=(h, w, c)),
            "miopen_dgrad": lambda: torch.ops.aten.convolution_backward(x, x, wt, None, [1, 1], [1, 1], [1, 1], False,
                                                                        [0, 0], 1, [True, False, False])[0],
        }
        best: dict = {}
        for _ in range(3):
            for k, f in arms.items():
                best.setdefault(k, []).append(t_us(f))
        rec = {"shape": [n, c, h, w], "check_rel": [round(err, 5), round(err2, 5)]}
        for k, v in best.items():
            rec[k + "_us"] = round(min(v), 1)
            rec[k + "_tfs"] = round(fl / min(v) / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
