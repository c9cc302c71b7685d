"""conv3x3n forward + statistics (ResNet-50 stage-2 shape 256 x 128 x 28 x 28 by default, SHAPE=n,c,h,w)
for rocprofv3 passes: after a warm-up, 5 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import gemm as G  # noqa: E402

n, c, h, w = (int(v) for v in os.environ.get("SHAPE", "256,128,28,28").split(","))
x = (torch.rand(n, c, h, w, device="cuda") - 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
w2 = ((torch.rand(c, 3, 3, c, device="cuda") - 0.5) * 0.05).bfloat16()
y = torch.empty(n, h, w, c, device="cuda", dtype=torch.bfloat16).permute(0, 3, 1, 2)
stats = torch.zeros(G.SHARDS, 2, c, device="cuda")
M = n * h * w
G.conv3x3n(x, w2, y, M, h, w, stats)
torch.cuda.synchronize()
for _ in range(5):
    G.conv3x3n(x, w2, y, M, h, w, stats)
torch.cuda.synchronize()
print("pmc_c3n done")
