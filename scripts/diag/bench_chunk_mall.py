"""Does the 256 MB MALL catch the second read of dY when a 1x1 convolution's weight gradient and input
gradient run chunk by chunk over the pixels (each chunk's dY read twice back to back) instead of
one full pass each (dY 411 MB > MALL)? ResNet-50 stage-1 conv3 / downsample backward shapes. JSON."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fluxmpi_amd.ops import gemm as G  # noqa: E402


def t_us(fn, iters=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def main():
    for (n, ci, co, h, w) in [(256, 64, 256, 56, 56), (256, 128, 512, 28, 28)]:
        M = n * h * w
        x2 = (torch.rand(M, ci, device="cuda") - 0.5).bfloat16()
        dy2 = (torch.rand(M, co, device="cuda") - 0.5).bfloat16()
        wt = ((torch.rand(co, ci, 1, 1, device="cuda") - 0.5) * 0.1).bfloat16()
        G.note_filter(wt)
        w2 = wt.view(co, ci)
        dx = torch.empty(M, ci, device="cuda", dtype=torch.bfloat16)

        def run(chunks, dgrad_first=False):
            step = -(-M // chunks)
            step = -(-step // 256) * 256
            for p0 in range(0, M, step):
                p1 = min(M, p0 + step)
                if dgrad_first:
                    G.conv1x1_dgrad(dy2[p0:p1], w2, out=dx[p0:p1], w4d=wt)
                    G.conv1x1_wgrad_v2(dy2[p0:p1], x2[p0:p1])
                else:
                    G.conv1x1_wgrad_v2(dy2[p0:p1], x2[p0:p1])
                    G.conv1x1_dgrad(dy2[p0:p1], w2, out=dx[p0:p1], w4d=wt)
        rec = {"shape": [n, ci, co, h, w], "dy_mb": round(dy2.numel() * 2 / 2 ** 20)}
        rec["wgrad_us"] = round(t_us(lambda: G.conv1x1_wgrad_v2(dy2, x2)), 1)
        rec["dgrad_us"] = round(t_us(lambda: G.conv1x1_dgrad(dy2, w2, out=dx, w4d=wt)), 1)
        for c in (1, 2, 4, 8):
            rec[f"pair_c{c}_us"] = round(t_us(lambda: run(c)), 1)
            rec[f"pair_c{c}_dfirst_us"] = round(t_us(lambda: run(c, True)), 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
