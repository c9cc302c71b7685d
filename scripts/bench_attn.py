"""Attention backward micro-benchmark at the ViT-B/16 shape (B=256, T=197, H=12, Dh=64):
our HIP kernels vs PyTorch's flash backward + interleaving copy. Prints us per call."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops.attention import attn_bwd_packed, attn_fwd_packed  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    B, T, H = int(os.environ.get("B", 256)), int(os.environ.get("T", 197)), 12
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    q, k, v = qkv.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    out, lse, cq, ck, mq, mk, seed, off, _ = torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.0, False)
    dy = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
    o2, st = attn_fwd_packed(qkv, H)
    ours = timeit(lambda: attn_bwd_packed(qkv, o2, dy, H, st))
    ours_fwd = timeit(lambda: attn_fwd_packed(qkv, H))

    def aten():
        dq, dk, dv = torch.ops.aten._scaled_dot_product_flash_attention_backward(
            dy.view(B, T, H, 64).transpose(1, 2), q, k, v, out, lse, cq, ck, mq, mk, 0.0, False, seed, off)
        return torch.stack([dq.transpose(1, 2), dk.transpose(1, 2), dv.transpose(1, 2)], dim=2)

    ref = timeit(aten)
    fwd = timeit(lambda: torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.0, False))
    print(f"attn bwd B={B} T={T} H={H}: ours {ours:.1f} us, aten+stack {ref:.1f} us; aten fwd {fwd:.1f} us, ours fwd {ours_fwd:.1f} us", flush=True)


if __name__ == "__main__":
    main()
