"""HIP attention (csrc/kernels/attention.hip) vs a plain PyTorch fp32 reference: the output of
softmax(q k^T / 8) v and the packed [B, T, 3*D] q|k|v gradient, head dim 64."""
import math

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


SHAPES = [(4, 197, 12), (2, 50, 4), (1, 7, 2), (2, 64, 3), (1, 1, 1), (3, 300, 2), (2, 33, 5)]


@pytest.mark.gpu
@pytest.mark.parametrize("b,t,heads", SHAPES + [(64, 197, 12)])
def test_attn_fwd_vs_fp32(gpu_ext, b, t, heads):
    """The resident forward (two workgroups per head; FLUXMPI_ATTN_FWD_PARTS) vs fp32."""
    from fluxmpi_amd.ops.attention import attn_fwd_packed
    torch.manual_seed(0)
    xb = (torch.randn(b, t, 3 * heads * 64, device="cuda") * 1.5).to(torch.bfloat16)
    out, stats = attn_fwd_packed(xb, heads)
    ref = _ref(xb.float(), heads)
    assert out.shape == ref.shape and out.dtype == torch.bfloat16
    assert _rel(out, ref) < 1e-2
    # stats[..., 0]: base-2 log-sum-exp of the scaled scores
    q, k, _ = xb.float().view(b, t, 3, heads, 64).permute(2, 0, 3, 1, 4)
    lse2 = torch.logsumexp((q @ k.transpose(-1, -2)) / 8, -1) / math.log(2)
    torch.testing.assert_close(stats[..., 0], lse2, rtol=1e-3, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("b,t,heads", SHAPES)
def test_attn_bwd_vs_fp32(gpu_ext, b, t, heads):
    from fluxmpi_amd.ops.attention import attn_bwd_packed, attn_fwd_packed
    torch.manual_seed(0)
    xb = (torch.randn(b, t, 3 * heads * 64, device="cuda") * 1.5).to(torch.bfloat16)
    xr = xb.float().requires_grad_()
    yr = _ref(xr, heads)
    g = torch.randn_like(yr)
    yr.backward(g)
    out, stats = attn_fwd_packed(xb, heads)
    dqkv = attn_bwd_packed(xb, out, g.to(torch.bfloat16), heads, stats)
    assert dqkv.shape == xb.shape and dqkv.dtype == torch.bfloat16
    assert torch.isfinite(dqkv).all()
    for i in range(3):
        got = dqkv.view(b, t, 3, -1)[:, :, i]
        ref = xr.grad.view(b, t, 3, -1)[:, :, i]
        assert _rel(got, ref) < 2e-2, (i, _rel(got, ref))


@pytest.mark.gpu
def test_packed_attention_native_vs_aten(gpu_ext, monkeypatch):
    """The ViT attention path runs our kernels and agrees with PyTorch's flash kernels."""
    from fluxmpi_amd.models import vit
    torch.manual_seed(2)
    x = torch.randn(4, 197, 3 * 768, device="cuda").to(torch.bfloat16)
    g = torch.randn(4, 197, 768, device="cuda").to(torch.bfloat16)
    res = {}
    for mode in ("native", "aten"):
        monkeypatch.setenv("FLUXMPI_ATTN", mode)
        assert vit._attn_native(x, 12) == (mode == "native")
        xa = x.clone().requires_grad_()
        y = vit.packed_attention(xa, 12)
        y.backward(g)
        res[mode] = (y.detach(), xa.grad)
    assert _rel(res["native"][0], res["aten"][0]) < 1e-2
    assert _rel(res["native"][1], res["aten"][1]) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("b,t,heads", [(3, 197, 4), (2, 50, 2), (2, 7, 1), (1, 256, 2)])
def test_attn_bwd_colsum_partials(gpu_ext, b, t, heads):
    """The resident backward pair's per-wave column sums of dQ / dK / dV (the packed QKV bias
    gradient) vs the column sums of the dQKV it wrote; the hand-off is taken once."""
    from fluxmpi_amd.ops.attention import attn_bwd_packed, attn_fwd_packed, take_colpart
    torch.manual_seed(3)
    xb = (torch.randn(b, t, 3 * heads * 64, device="cuda") * 1.5).to(torch.bfloat16)
    out, stats = attn_fwd_packed(xb, heads)
    g = torch.randn(b, t, heads * 64, device="cuda").to(torch.bfloat16)
    dqkv = attn_bwd_packed(xb, out, g, heads, stats)
    part = take_colpart(dqkv.view(b * t, -1))
    assert part is not None and part.shape[1] == 3 * heads * 64
    assert take_colpart(dqkv.view(b * t, -1)) is None  # consumed
    ref = dqkv.float().sum((0, 1))
    got = part.sum(0)
    # the partials sum the fp32 values before their bf16 rounding
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item() / 10 + 1e-3)
    # a gradient accumulated into dQKV in place (same pointer, same size) invalidates the hand-off
    dqkv2 = attn_bwd_packed(xb, out, g, heads, stats)
    dqkv2.add_(1.0)
    assert take_colpart(dqkv2.view(b * t, -1)) is None


@pytest.mark.gpu
def test_attn_bwd_pair_variant(gpu_ext):
    """The dq / dkv pair (FLUXMPI_ATTN_BWD=pair, read once per process by the native library; the
    default for 13 key tiles, T 193..208, is the fused kernel): the fp32-reference and column-sum
    tests of this file, in a child process with the pair."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, FLUXMPI_ATTN_BWD="pair")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(root, "tests", "test_attention_gpu.py"), "-k",
                        "attn_bwd_vs_fp32 or colsum_partials or fused_matches_pair"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.gpu
def test_attn_bwd_fused_matches_pair(gpu_ext):
    """At the ViT shape (the fused kernel by default; the pair in test_attn_bwd_pair_variant's
    child process) dQKV and its column sums agree with the fp32 reference."""
    from fluxmpi_amd.ops.attention import attn_bwd_packed, attn_fwd_packed, take_colpart
    torch.manual_seed(5)
    b, t, heads = 4, 197, 12
    xb = (torch.randn(b, t, 3 * heads * 64, device="cuda") * 1.5).to(torch.bfloat16)
    xr = xb.float().requires_grad_()
    yr = _ref(xr, heads)
    g = torch.randn_like(yr)
    yr.backward(g)
    out, stats = attn_fwd_packed(xb, heads)
    dqkv = attn_bwd_packed(xb, out, g.to(torch.bfloat16), heads, stats)
    assert torch.isfinite(dqkv).all()
    for i in range(3):
        assert _rel(dqkv.view(b, t, 3, -1)[:, :, i], xr.grad.view(b, t, 3, -1)[:, :, i]) < 2e-2, i
    part = take_colpart(dqkv.view(b * t, -1))
    assert part is not None
    ref = dqkv.float().sum((0, 1))
    torch.testing.assert_close(part.sum(0), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item() / 10 + 1e-3)
