"""Whole-model ViT numerics (VERDICT r2 next #8a): the fused bf16 ViT — gemm_nt forward /
input-gradient GEMMs with bias / GELU / GELU-backward epilogues, the GELU link into fc2's
input gradient, proj / fc2 + residual + LayerNorm nodes, packed attention, the CLS-only last
block — against a plain PyTorch model with the same (bf16-rounded) weights, in fp32 and in
bf16. Width 768, 197 tokens, depth 2, batch 256 (50432 rows: every gemm_nt path is taken).
Criterion (the ResNet pattern of test_fused_block_gpu.py): the fused model's error against
fp32 stays within a small multiple of plain bf16 PyTorch's error against fp32."""
import math

import pytest
import torch
import torch.nn.functional as F

from fluxmpi_amd.ops.gelu import gelu

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _plain_forward(P, x, depth, heads, patch=16):
    """ViT-B/16 forward in plain PyTorch ops from a parameter dict (dtype of the tensors)."""
    n, c, hh, ww = x.shape
    t = x.reshape(n, c, hh // patch, patch, ww // patch, patch).permute(0, 2, 4, 1, 3, 5)
    t = t.reshape(n, (hh // patch) * (ww // patch), c * patch * patch)
    z = F.linear(t, P["embed.proj.weight"], P["embed.proj.bias"])
    z = torch.cat([P["cls"].expand(n, -1, -1), z], 1) + P["pos"]
    d = z.shape[-1]
    for i in range(depth):
        p = f"blocks.{i}."
        y = F.layer_norm(z, (d,), P[p + "ln1.weight"], P[p + "ln1.bias"], 1e-6)
        qkv = F.linear(y, P[p + "qkv.weight"], P[p + "qkv.bias"])
        q, k, v = qkv.view(n, -1, 3, heads, d // heads).permute(2, 0, 3, 1, 4)
        att = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(d // heads), -1) @ v
        a = att.transpose(1, 2).reshape(n, -1, d)
        z = z + F.linear(a, P[p + "proj.weight"], P[p + "proj.bias"])
        y = F.layer_norm(z, (d,), P[p + "ln2.weight"], P[p + "ln2.bias"], 1e-6)
        g = gelu(F.linear(y, P[p + "fc1.weight"], P[p + "fc1.bias"]))  # the model's GELU form
        z = z + F.linear(g, P[p + "fc2.weight"], P[p + "fc2.bias"])
    cl = F.layer_norm(z[:, 0], (d,), P["ln.weight"], P["ln.bias"], 1e-6)
    return F.linear(cl, P["head.weight"], P["head.bias"])


def test_vit_whole_model_matches_fp32(gpu_ext):
    from fluxmpi_amd.models.vit import ViT
    depth, heads = 2, 12
    torch.manual_seed(0)
    model = ViT(depth=depth, heads=heads, num_classes=100).cuda()
    with torch.no_grad():  # nonzero biases so the bias epilogues / gradients are exercised
        for n_, p in model.named_parameters():
            if n_.endswith("bias"):
                p.normal_(0, 0.02)
    model = model.to(torch.bfloat16)
    B = 256
    x = torch.randn(B, 3, 224, 224, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 100, (B,), device="cuda")
    names = [n_ for n_, _ in model.named_parameters()]
    P32 = {n_: p.detach().float().clone().requires_grad_() for n_, p in model.named_parameters()}
    P16 = {n_: p.detach().clone().requires_grad_() for n_, p in model.named_parameters()}

    out = model(x)
    F.cross_entropy(out.float(), y).backward()
    out32 = _plain_forward(P32, x.float(), depth, heads)
    F.cross_entropy(out32, y).backward()
    out16 = _plain_forward(P16, x, depth, heads)
    F.cross_entropy(out16.float(), y).backward()

    e_ours, e_plain = _rel(out, out32), _rel(out16, out32)
    assert e_ours < 2 * e_plain + 1e-2, (e_ours, e_plain)
    grads = dict(model.named_parameters())
    worst = []
    for n_ in names:
        go, g32, g16 = grads[n_].grad, P32[n_].grad, P16[n_].grad
        assert go is not None and torch.isfinite(go).all(), n_
        eo, ep = _rel(go, g32), _rel(g16, g32)
        worst.append((eo - 2 * ep, n_, eo, ep))
        assert eo < 2 * ep + 2e-2, f"{n_}: fused {eo:.4f} vs plain bf16 {ep:.4f} (relative to fp32)"
    worst.sort(reverse=True)
    print("worst gradient margins:", worst[:4])
