"""HIP attention backward (csrc/kernels/attention.hip) vs a plain PyTorch fp32 reference:
the packed [B, T, 3*D] q|k|v gradient of softmax(q k^T / 8) v, head dim 64."""
import pytest
import torch
import torch.nn.functional as F


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _ref(qkv, heads):
    b, t, d3 = qkv.shape
    d = d3 // 3
    q, k, v = qkv.view(b, t, 3, heads, d // heads).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) / (d // heads) ** 0.5
    return (s.softmax(-1) @ v).transpose(1, 2).reshape(b, t, d)


def test_supported_gate_cpu():
    from fluxmpi_amd.ops.attention import supported
    assert not supported(torch.zeros(1, 4, 3 * 64, dtype=torch.bfloat16), 1)  # CPU tensor


@pytest.mark.gpu
@pytest.mark.parametrize("b,t,heads", [(4, 197, 12), (2, 50, 4), (1, 7, 2), (2, 64, 3), (1, 1, 1), (3, 300, 2),
                                       (2, 33, 5)])
def test_attn_bwd_vs_fp32(gpu_ext, b, t, heads):
    from fluxmpi_amd.ops.attention import attn_bwd_packed
    torch.manual_seed(0)
    x = torch.randn(b, t, 3 * heads * 64, device="cuda") * 1.5
    xb = x.to(torch.bfloat16)
    xr = xb.float().requires_grad_()
    yr = _ref(xr, heads)
    g = torch.randn_like(yr)
    yr.backward(g)
    q, k, v = xb.view(b, t, 3, heads, 64).permute(2, 0, 3, 1, 4)
    out = F.scaled_dot_product_attention(q, k, v)  # [B, H, T, 64] (forward output, bf16)
    dqkv = attn_bwd_packed(xb, out, g.to(torch.bfloat16), heads)
    assert dqkv.shape == xb.shape and dqkv.dtype == torch.bfloat16
    assert torch.isfinite(dqkv).all()
    for i in range(3):
        got = dqkv.view(b, t, 3, -1)[:, :, i]
        ref = xr.grad.view(b, t, 3, -1)[:, :, i]
        assert _rel(got, ref) < 2e-2, (i, _rel(got, ref))


@pytest.mark.gpu
def test_attn_bwd_strided_out(gpu_ext):
    """out in the [B, T, H, 64] memory layout (transposed view), as some forwards return it."""
    from fluxmpi_amd.ops.attention import attn_bwd_packed
    torch.manual_seed(1)
    b, t, heads = 2, 77, 3
    xb = torch.randn(b, t, 3 * heads * 64, device="cuda").to(torch.bfloat16)
    xr = xb.float().requires_grad_()
    yr = _ref(xr, heads)
    g = torch.randn_like(yr)
    yr.backward(g)
    out = yr.detach().to(torch.bfloat16).view(b, t, heads, 64).transpose(1, 2)
    dqkv = attn_bwd_packed(xb, out, g.to(torch.bfloat16), heads)
    assert _rel(dqkv, xr.grad) < 2e-2


@pytest.mark.gpu
def test_packed_attention_uses_native_bwd(gpu_ext, monkeypatch):
    """The ViT attention path runs our backward and agrees with PyTorch's flash backward."""
    from fluxmpi_amd.models import vit
    torch.manual_seed(2)
    x = torch.randn(4, 197, 3 * 768, device="cuda").to(torch.bfloat16)
    grads = {}
    for mode in ("native", "aten"):
        monkeypatch.setenv("FLUXMPI_ATTN_BWD", mode)
        xa = x.clone().requires_grad_()
        y = vit.packed_attention(xa, 12)
        y.backward(torch.ones_like(y))
        grads[mode] = xa.grad
        assert vit._attn_native(x, 12) == (mode == "native")
    assert _rel(grads["native"], grads["aten"]) < 2e-2
