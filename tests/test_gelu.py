"""Fused GELU backward + bias gradient (``csrc/kernels/gelu.hip``, ``ops/gelu.py``) against the
fp32 PyTorch composition ``gelu(linear(x, W, b))``, for both GELU forms (tanh: NNlib's ``gelu``,
the default; erf)."""
import pytest
import torch
import torch.nn.functional as F

from fluxmpi_amd.ops import gelu as GL
from fluxmpi_amd.ops.gelu import gelu_bwd_bias, linear_gelu


@pytest.fixture(params=["tanh", "erf"])
def form(request):
    old = GL.FORM
    GL.set_form(request.param)
    yield request.param
    GL.set_form(old)


def _ref(x, w, b, dy):
    xr, wr, br = (t.detach().float().clone().requires_grad_() for t in (x, w, b))
    y = GL.gelu(F.linear(xr, wr, br))
    y.backward(dy.float())
    return y, xr.grad, wr.grad, br.grad


def test_default_form_is_nnlib_tanh():
    assert GL.FORM == "tanh"  # FLUXMPI_GELU unset in the test environment
    x = torch.linspace(-6, 6, 101, dtype=torch.float64)
    nnlib = 0.5 * x * (1 + torch.tanh((2 / torch.pi) ** 0.5 * (x + 0.044715 * x ** 3)))
    torch.testing.assert_close(GL.gelu(x), nnlib)


def test_gelu_grad_ref_matches_autograd(form):
    x = torch.linspace(-8, 8, 1001, dtype=torch.float64, requires_grad=True)
    GL.gelu(x).sum().backward()
    torch.testing.assert_close(GL._gelu_grad_ref(x.detach()), x.grad)


def test_set_form_rejects_unknown():
    with pytest.raises(ValueError):
        GL.set_form("sigmoid")


def test_linear_gelu_cpu_fallback(form):
    torch.manual_seed(0)
    x, w, b = torch.randn(3, 5, 16, requires_grad=True), torch.randn(24, 16, requires_grad=True), torch.randn(24, requires_grad=True)
    y = linear_gelu(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr, dxr, dwr, dbr = _ref(x, w, b, dy)
    torch.testing.assert_close(y, yr)
    torch.testing.assert_close(x.grad, dxr)
    torch.testing.assert_close(w.grad, dwr)
    torch.testing.assert_close(b.grad, dbr)
    h = torch.randn(7, 24)
    dh, db = gelu_bwd_bias(dy.reshape(-1, 24)[:7], h)
    torch.testing.assert_close(db, dh.sum(0))


@pytest.mark.gpu
@pytest.mark.parametrize("rows,k,n", [(197 * 4, 768, 3072), (1000, 64, 512), (37, 128, 8192), (50432, 768, 3072)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_linear_gelu_gpu(form, rows, k, n, dtype):
    torch.manual_seed(rows + n)
    x = (torch.randn(rows, k, device="cuda") * 0.5).to(dtype).requires_grad_()
    w = (torch.randn(n, k, device="cuda") / k ** 0.5).to(dtype).requires_grad_()
    b = (torch.randn(n, device="cuda") * 0.1).to(dtype).requires_grad_()
    y = linear_gelu(x, w, b)
    dy = torch.randn(rows, n, device="cuda").to(dtype)
    y.backward(dy)
    yr, dxr, dwr, dbr = _ref(x, w, b, dy)
    tol = dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(x.grad.float(), dxr, rtol=3e-2, atol=5e-2 * (n / k) ** 0.5)
    scale = rows ** 0.5
    torch.testing.assert_close(w.grad.float(), dwr, rtol=3e-2, atol=3e-2 * scale)
    torch.testing.assert_close(b.grad.float(), dbr, rtol=3e-2, atol=3e-2 * scale)


@pytest.mark.gpu
def test_gelu_bwd_bias_kernel_gpu(form):
    torch.manual_seed(5)
    h = torch.randn(3001, 1024, device="cuda").to(torch.bfloat16)
    dy = torch.randn_like(h)
    dh, db = gelu_bwd_bias(dy, h)
    hf = h.float().requires_grad_()
    GL.gelu(hf).backward(dy.float())
    torch.testing.assert_close(dh.float(), hf.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(db, dh.float().sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [8, 4096 * 8 + 8, 50432 * 3072])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gelu_fwd_kernel_gpu(gpu_ext, form, n, dtype):
    torch.manual_seed(n % 97)
    h = (torch.randn(n, device="cuda") * 3).to(dtype)
    g = GL._gelu_fwd(h)
    ref = GL.gelu(h.float())
    torch.testing.assert_close(g.float(), ref, rtol=1e-2, atol=1e-2)
    assert float((g.float() - ref).abs().max()) < 2e-2
