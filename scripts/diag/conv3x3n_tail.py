"""conv3x3n round quantization: us per call at batch sizes around 256 (tiles = pixels / 256 over
resident workgroup slots). If the last partial round costs a whole tile-time, time(256) / time(240)
approaches rounds(256) / rounds(240) instead of 256 / 240. With FLUXMPI_CONV3X3N_NOTAIL set the
128-channel layers run without the 64-pixel tail launch (one process per setting). JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fluxmpi_amd.ops import gemm as G  # noqa: E402


def t_us(fn, iters=20):
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


for (c, h, w) in [(64, 56, 56), (128, 28, 28)]:
    for n in (192, 224, 240, 256, 272):
        x = (torch.rand(n, c, h, w, device="cuda") - 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
        wt = ((torch.rand(c, c, 3, 3, device="cuda") - 0.5) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        w2 = wt.permute(0, 2, 3, 1).contiguous()
        M = n * h * w
        if M % 256:
            continue
        y = torch.empty(n, h, w, c, device="cuda", dtype=torch.bfloat16).permute(0, 3, 1, 2)
        stats = torch.zeros(G.SHARDS, 2, c, device="cuda")
        us = t_us(lambda: G.conv3x3n(x, w2, y, M, h, w, stats))
        print(json.dumps({"c": c, "n": n, "tail": not os.environ.get("FLUXMPI_CONV3X3N_NOTAIL"), "tiles": M // 256, "us": round(us, 1), "us_per_img": round(us / n, 3)}),
              flush=True)
