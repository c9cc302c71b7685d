"""The ViT-B/16 weight gradients (wgrad256.hip + the split-K reduce) for rocprofv3 --pmc passes:
after a warm-up, 5 calls each of qkv / proj / fc1 / fc2 (K = 50432 tokens)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops.linear import weight_grad  # noqa: E402

K = 50432
shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]  # (n_out, n_in)
ops = []
for n_out, n_in in shapes:
    dy = (torch.rand(K, n_out, device="cuda") - 0.5).bfloat16()
    x = (torch.rand(K, n_in, device="cuda") - 0.5).bfloat16()
    ops.append((dy, x))
for dy, x in ops:
    weight_grad(dy, x, torch.bfloat16)
torch.cuda.synchronize()
for dy, x in ops:
    for _ in range(5):
        weight_grad(dy, x, torch.bfloat16)
torch.cuda.synchronize()
print("pmc_wgrad done")
