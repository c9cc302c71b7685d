"""gemm256.hip (ViT forward / input-gradient GEMMs with fused epilogues) vs PyTorch fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.fixture(params=["tanh", "erf"], autouse=True)
def gelu_form(request):
    from fluxmpi_amd.ops import gelu as GL
    old = GL.FORM
    GL.set_form(request.param)
    yield request.param
    GL.set_form(old)


def _gelu_ref(h):
    from fluxmpi_amd.ops import gelu as GL
    return GL.gelu(h.float())


def _gelu_grad_ref(h):
    from fluxmpi_amd.ops import gelu as GL
    return GL._gelu_grad_ref(h.float())


@pytest.mark.parametrize("m,n,k", [(512, 768, 768), (768, 256, 3072), (256, 512, 520), (1024, 2304, 768)])
@pytest.mark.parametrize("bias", [None, "f32", "bf16"])
def test_linear_fwd(gpu_ext, m, n, k, bias):
    from fluxmpi_amd.ops import gemm256 as G
    torch.manual_seed(0)
    x = torch.randn(m, k, device="cuda").bfloat16()
    w = (torch.randn(n, k, device="cuda") * k ** -0.5).bfloat16()
    b = None if bias is None else (torch.randn(n, device="cuda") * 0.5).to(torch.float32 if bias == "f32" else torch.bfloat16)
    assert G.supported(m, n, k, x, w, fused=True)
    y = G.linear_fwd(x, w, b)
    ref = x.float() @ w.float().t() + (b.float() if b is not None else 0)
    assert _rel(y, ref) < 5e-3
    yy, g = G.linear_fwd(x, w, b, gelu=True)
    assert torch.equal(yy, y)
    assert _rel(g, _gelu_ref(y)) < 5e-3  # GELU of the rounded pre-activation


@pytest.mark.parametrize("m,n,k", [(512, 768, 768), (256, 3072, 768), (768, 520, 256), (1024, 768, 2304)])
def test_linear_dgrad(gpu_ext, m, n, k):
    from fluxmpi_amd.ops import gemm256 as G
    torch.manual_seed(1)
    dy = torch.randn(m, n, device="cuda").bfloat16()
    w = (torch.randn(n, k, device="cuda") * n ** -0.5).bfloat16()
    assert G.supported(m, k, n, dy, w, b_t=True, fused=True)
    dx = G.linear_dgrad(dy, w)
    ref = dy.float() @ w.float()
    assert _rel(dx, ref) < 5e-3
    h = torch.randn(m, k, device="cuda").bfloat16()
    dh, db = G.linear_dgrad(dy, w, gelu_h=h)
    dh_ref = ref.bfloat16().float() * _gelu_grad_ref(h)
    assert _rel(dh, dh_ref) < 5e-3
    torch.testing.assert_close(db, dh.float().sum(0), rtol=1e-3, atol=1e-2)
    _, db16 = G.linear_dgrad(dy, w, gelu_h=h, bias_dtype=torch.bfloat16)
    assert db16.dtype == torch.bfloat16 and _rel(db16, db) < 1e-2


def test_unsupported_shapes(gpu_ext):
    from fluxmpi_amd.ops import gemm256 as G
    x = torch.zeros(200, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(768, 768, device="cuda", dtype=torch.bfloat16)
    assert not G.supported(200, 768, 768, x, w, fused=True)  # rows not a multiple of 256
    assert not G.supported(256, 768, 768, x.float(), w, fused=True)
