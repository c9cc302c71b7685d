"""The stage-1 3x3 weight gradient (ResNet-50, 256 x 64 x 56 x 56) on wgrad3x3n.hip + the split-K
reduce, for rocprofv3 passes: after a warm-up, 5 calls in the configuration W3N="variant,target"
(default 3,256)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import gemm as G  # noqa: E402

cfg = tuple(int(v) for v in os.environ.get("W3N", "3,256").split(","))
n, c, h, w = (int(v) for v in os.environ.get("SHAPE", "256,64,56,56").split(","))
x = (torch.rand(n, c, h, w, device="cuda") - 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
dy = (torch.rand(n, c, h, w, device="cuda") - 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
G.conv3x3_wgrad_n(dy, x, *cfg)
torch.cuda.synchronize()
for _ in range(5):
    G.conv3x3_wgrad_n(dy, x, *cfg)
torch.cuda.synchronize()
print("pmc_w3n done")
