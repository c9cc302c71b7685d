"""Attention kernels at the ViT-B/16 shape (B=256, T=197, H=12) for rocprofv3 --pmc passes:
5 forward and 5 backward calls (dq / dkv pair) after a warm-up."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops.attention import attn_bwd_packed, attn_fwd_packed  # noqa: E402

B, T, H = int(os.environ.get("B", 256)), 197, 12
qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
dy = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
for _ in range(2):
    o, st = attn_fwd_packed(qkv, H)
    attn_bwd_packed(qkv, o, dy, H, st)
torch.cuda.synchronize()
for _ in range(5):
    o, st = attn_fwd_packed(qkv, H)
for _ in range(5):
    attn_bwd_packed(qkv, o, dy, H, st)
torch.cuda.synchronize()
print("pmc_attn done")
