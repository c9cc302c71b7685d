"""Time wgrad3x3n (+ reduce) at the ResNet-50 stage-1 shape in a few configurations, no checks
(for diagnostic builds loaded through FLUXMPI_C_VARIANT): one JSON line."""
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
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


n, c, h, w = (int(v) for v in os.environ.get("SHAPE", "256,64,56,56").split(","))
x = (torch.rand(n, c, h, w, device="cuda") - 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
dy = (torch.rand(n, c, h, w, device="cuda") - 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
rec = {"variant": os.environ.get("FLUXMPI_C_VARIANT", "default"), "shape": [n, c, h, w]}
for cfg in [(3, 256), (1, 256), (2, 256)]:
    rec[str(cfg)] = round(min(t_us(lambda: G.conv3x3_wgrad_n(dy, x, *cfg)) for _ in range(3)), 1)
print(json.dumps(rec), flush=True)
