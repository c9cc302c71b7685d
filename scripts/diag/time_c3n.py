"""Time conv3x3n (forward + statistics) at the ResNet-50 stage-1 / stage-2 shapes, relative error against an fp32 conv2d (for
diagnostic builds loaded through FLUXMPI_C_VARIANT): one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import load_variant  # noqa: E402

load_variant.install()
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


rec = {"variant": os.environ.get("FLUXMPI_C_VARIANT", "default")}
for (n, c, h, w) in [(256, 64, 56, 56), (256, 128, 28, 28), (240, 128, 28, 28)]:
    x = (torch.rand(n, c, h, w, device="cuda") - 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
    w2 = ((torch.rand(c, 3, 3, c, device="cuda") - 0.5) * 0.05).bfloat16()
    y = torch.empty(n, h, w, c, device="cuda", dtype=torch.bfloat16).permute(0, 3, 1, 2)
    stats = torch.zeros(G.SHARDS, 2, c, device="cuda")
    M = n * h * w
    G.conv3x3n(x, w2, y, M, h, w, stats)
    ref = torch.nn.functional.conv2d(x.float(), w2.permute(0, 3, 1, 2).float(), padding=1)
    rec[f"{n}x{c}x{h}_rel"] = round(float((y.float() - ref).norm() / ref.norm()), 5)
    rec[f"{n}x{c}x{h}"] = round(t_us(lambda: G.conv3x3n(x, w2, y, M, h, w, stats)), 1)
    if os.environ.get("C3N_EPI0"):
        rec[f"{n}x{c}x{h}_epi0"] = round(t_us(lambda: G.conv3x3n(x, w2, y, M, h, w, None)), 1)
print(json.dumps(rec), flush=True)
