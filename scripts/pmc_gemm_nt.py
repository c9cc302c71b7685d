"""gemm_nt kernels at the ViT-B/16 / ResNet-50 shapes for rocprofv3 --pmc passes: after a warm-up,
5 calls each of qkv forward (plain epilogue), fc1 forward (bias + GELU + derivative epilogue), fc2
input gradient (GELU-backward epilogue) and the 14x14x256 3x3 convolution (statistics epilogue)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import gemm as GM  # noqa: E402
from fluxmpi_amd.ops import gemm_nt as G  # noqa: E402

M = 50432


def u(*s, scale=1.0):
    return ((torch.rand(*s, device="cuda") * 2 - 1) * scale).bfloat16()


x, wq, w1, w2 = u(M, 768), u(2304, 768, scale=768 ** -0.5), u(3072, 768, scale=768 ** -0.5), u(768, 3072, scale=3072 ** -0.5)
b1 = torch.zeros(3072, device="cuda")
dy2 = u(M, 768)
img = u(256, 256, 14, 14).contiguous(memory_format=torch.channels_last)
wc = u(256, 256, 3, 3, scale=2304 ** -0.5).contiguous(memory_format=torch.channels_last)
stats = torch.zeros(GM.SHARDS, 2, 256, device="cuda")
d1, _ = G.linear_fwd(x, w1, b1, gelu=True)
calls = [lambda: G.linear_fwd(x, wq), lambda: G.linear_fwd(x, w1, b1, gelu=True),
         lambda: G.linear_dgrad(dy2, w2, gelu_d=d1), lambda: GM.conv3x3_fwd(img, wc, stats=stats)]
for f in calls:
    f()
torch.cuda.synchronize()
for f in calls:
    for _ in range(5):
        f()
torch.cuda.synchronize()
print("pmc_gemm_nt done")
