"""ViT pieces vs PyTorch fp32: packed-QKV attention (forward + packed gradient)."""
import pytest
import torch
import torch.nn.functional as F


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _ref_attention(qkv, heads):
    b, t, d3 = qkv.shape
    d = d3 // 3
    q, k, v = qkv.view(b, t, 3, heads, d // heads).permute(2, 0, 3, 1, 4)
    return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, t, d)


def test_packed_attention_cpu_fallback():
    from fluxmpi_amd.models.vit import packed_attention
    qkv = torch.randn(2, 9, 3 * 32)
    torch.testing.assert_close(packed_attention(qkv, 4), _ref_attention(qkv, 4))


@pytest.mark.gpu
@pytest.mark.parametrize("b,t,heads,dh", [(4, 197, 12, 64), (2, 50, 4, 32), (1, 7, 2, 64)])
def test_packed_attention_vs_fp32(gpu_ext, b, t, heads, dh):
    from fluxmpi_amd.models.vit import packed_attention
    torch.manual_seed(0)
    x = torch.randn(b, t, 3 * heads * dh, device="cuda")
    xa = x.to(torch.bfloat16).requires_grad_()
    xr = x.to(torch.bfloat16).float().requires_grad_()
    y = packed_attention(xa, heads)
    yr = _ref_attention(xr, heads)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 2e-2
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)
    assert xa.grad.shape == xa.shape and xa.grad.is_contiguous()
    assert _rel(xa.grad, xr.grad) < 3e-2


@pytest.mark.gpu
def test_vit_tiny_step(gpu_ext):
    from fluxmpi_amd.models.vit import vit_tiny
    torch.manual_seed(0)
    m = vit_tiny().cuda().to(torch.bfloat16)
    x = torch.randn(4, 3, 32, 32, device="cuda", dtype=torch.bfloat16)
    loss = m(x).float().logsumexp(-1).mean()
    loss.backward()
    assert torch.isfinite(loss)
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
