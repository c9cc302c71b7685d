"""Fused LayerNorm (+ residual add) vs the PyTorch fp32 composition."""
import pytest
import torch
import torch.nn.functional as F


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def test_add_layer_norm_cpu_fallback():
    from fluxmpi_amd.ops.layernorm import FusedLayerNorm
    ln = FusedLayerNorm(16)
    x, r = torch.randn(3, 5, 16), torch.randn(3, 5, 16)
    h, y = ln.add_forward(x, r)
    torch.testing.assert_close(h, x + r)
    torch.testing.assert_close(y, F.layer_norm(x + r, (16,), ln.weight, ln.bias, ln.eps))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 197, 768), (3, 5, 64), (2, 7, 1032), (2, 3, 4096), (64, 197, 768)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("add", [False, True])
@pytest.mark.parametrize("affine", ["act", "fp32"])
def test_layer_norm_vs_reference(gpu_ext, shape, dtype, add, affine):
    """``affine="act"``: w / b in the activation dtype, read by the kernels as they are (dw / db
    reduced straight into that dtype); ``"fp32"``: fp32 parameters with bf16 activations."""
    from fluxmpi_amd.ops.layernorm import add_layer_norm, layer_norm
    torch.manual_seed(0)
    d = shape[-1]
    x = torch.randn(shape, device="cuda").to(dtype)
    r = torch.randn(shape, device="cuda").to(dtype)
    wdt = dtype if affine == "act" else torch.float32
    w = (torch.rand(d, device="cuda") + 0.5).to(wdt)
    b = (torch.randn(d, device="cuda") * 0.1).to(wdt)
    xa, ra, wa, ba = (t.clone().requires_grad_() for t in (x, r, w, b))
    xr, rr, wr, br = (t.float().clone().requires_grad_() for t in (x, r, w, b))
    if add:
        h, y = add_layer_norm(xa, ra, wa, ba, 1e-6)
        hr = (xr + rr).to(dtype).float()  # the kernel normalises the stored (rounded) h
        yr = F.layer_norm(hr, (d,), wr, br, 1e-6)
        torch.testing.assert_close(h.float(), (xr + rr).detach(), rtol=1e-2, atol=1e-2)
        gh = torch.randn_like(yr)
        gy = torch.randn_like(yr)
        ((h.float() * gh).sum() + (y.float() * gy).sum()).backward()
        ((hr * gh).sum() + (yr * gy).sum()).backward()
    else:
        y = layer_norm(xa, wa, ba, 1e-6)
        yr = F.layer_norm(xr, (d,), wr, br, 1e-6)
        gy = torch.randn_like(yr)
        (y.float() * gy).sum().backward()
        (yr * gy).sum().backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert _rel(y, yr) < tol
    assert _rel(xa.grad, xr.grad) < tol
    assert wa.grad.dtype == wdt and ba.grad.dtype == wdt
    assert _rel(wa.grad, wr.grad) < tol and _rel(ba.grad, br.grad) < tol
    if add:
        assert _rel(ra.grad, rr.grad) < tol


@pytest.mark.gpu
def test_layer_norm_no_affine(gpu_ext):
    from fluxmpi_amd.ops.layernorm import layer_norm
    torch.manual_seed(0)
    x = torch.randn(8, 33, 768, device="cuda").to(torch.bfloat16)
    xa, xr = x.clone().requires_grad_(), x.float().clone().requires_grad_()
    y = layer_norm(xa, None, None, 1e-6)
    yr = F.layer_norm(xr, (768,), None, None, 1e-6)
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    assert _rel(y, yr) < 2e-2 and _rel(xa.grad, xr.grad) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 197, 768), (2, 7, 1032)])
def test_linear_add_layer_norm(gpu_ext, dtype, shape):
    """proj + residual add + LayerNorm as one node (the LayerNorm backward's dx column sums are the
    projection's bias gradient) vs the fp32 PyTorch composition."""
    from fluxmpi_amd.ops.layernorm import linear_add_layer_norm
    torch.manual_seed(3)
    d = shape[-1]
    k = 256
    a = (torch.randn(*shape[:-1], k, device="cuda") * 0.5).to(dtype)
    W = (torch.randn(d, k, device="cuda") * 0.05).to(dtype)
    b = (torch.randn(d, device="cuda") * 0.1).to(dtype)
    x = torch.randn(shape, device="cuda").to(dtype)
    lw = (torch.rand(d, device="cuda") + 0.5).to(dtype)
    lb = (torch.randn(d, device="cuda") * 0.1).to(dtype)
    ins = [t.clone().requires_grad_() for t in (a, W, b, x, lw, lb)]
    ref = [t.float().clone().requires_grad_() for t in (a, W, b, x, lw, lb)]
    h, y = linear_add_layer_norm(*ins, 1e-6)
    hr = ref[3] + F.linear(ref[0], ref[1], ref[2])
    yr = F.layer_norm(hr, (d,), ref[4], ref[5], 1e-6)
    gh, gy = torch.randn_like(hr), torch.randn_like(yr)
    ((h.float() * gh).sum() + (y.float() * gy).sum()).backward()
    ((hr * gh).sum() + (yr * gy).sum()).backward()
    assert _rel(h, hr) < 2e-2 and _rel(y, yr) < 2e-2
    for t, r in zip(ins, ref):
        assert t.grad is not None and t.grad.dtype == t.dtype
        assert _rel(t.grad, r.grad) < 3e-2
