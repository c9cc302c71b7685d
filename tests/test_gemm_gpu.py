"""MFMA GEMM / fused 1x1-conv kernels vs PyTorch fp32 references (GPU only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(4096, 64, 256), (1000, 96, 160), (512, 256, 64), (2048, 512, 1024), (200, 32, 32), (777, 64, 192)]


@pytest.fixture(params=[0, 1, 2], ids=["nbuf_auto", "nbuf1", "nbuf2"], autouse=True)
def nbuf(request, monkeypatch):
    """Every case runs with the launcher's choice and with both LDS buffering variants forced."""
    from fluxmpi_amd.ops import gemm
    monkeypatch.setattr(gemm, "NBUF", request.param)
    return request.param


def _rand(*s):
    return torch.randn(*s, device="cuda").to(torch.bfloat16)


def _affine(c):
    return (torch.rand(c, device="cuda") + 0.5), torch.randn(c, device="cuda") * 0.5


def _act(x, aff):
    if aff is None:
        return x.float()
    s, t = aff
    # the kernel computes fmaf(x, s, t): emulate the single rounding in fp64
    y = (x.double() * s.double() + t.double()).float()
    return torch.relu(y).to(torch.bfloat16).float()


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("use_aff", [False, True])
def test_fwd(gpu_ext, M, K, N, use_aff):
    from fluxmpi_amd.ops.gemm import SHARDS, conv1x1_fwd
    x, w = _rand(M, K), _rand(N, K)
    aff = _affine(K) if use_aff else None
    stats = torch.zeros(SHARDS, 2, N, device="cuda")
    y = conv1x1_fwd(x, w, aff, stats)
    ref = _act(x, aff) @ w.float().t()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    yf = y.float()
    torch.testing.assert_close(stats[:, 0].sum(0), yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(stats[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_dgrad(gpu_ext, M, K, N):
    from fluxmpi_amd.ops.gemm import conv1x1_dgrad
    dy, w = _rand(M, N), _rand(N, K)
    dx = conv1x1_dgrad(dy, w)
    torch.testing.assert_close(dx.float(), dy.float() @ w.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("use_aff", [False, True])
@pytest.mark.parametrize("splits", [None, 1, 7])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_wgrad(gpu_ext, M, K, N, use_aff, splits, out_dtype):
    from fluxmpi_amd.ops.gemm import conv1x1_wgrad
    dy, x = _rand(M, N), _rand(M, K)
    aff = _affine(K) if use_aff else None
    dw = conv1x1_wgrad(dy, x, aff, out_dtype=out_dtype, splits=splits)
    assert dw.dtype == out_dtype
    ref = dy.float().t() @ _act(x, aff)
    tol = dict(rtol=1e-2, atol=5e-2) if out_dtype == torch.float32 else dict(rtol=2e-2, atol=1e-1)
    torch.testing.assert_close(dw.float(), ref, **tol)


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_dgrad_residual(gpu_ext, M, K, N):
    from fluxmpi_amd.ops.gemm import conv1x1_dgrad
    dy, w, r = _rand(M, N), _rand(N, K), _rand(M, K)
    dx = conv1x1_dgrad(dy, w, residual=r)
    ref = (dy.float() @ w.float()).to(torch.bfloat16).float() + r.float()
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2)


def test_asymmetric_identity(gpu_ext):
    """A = I with an asymmetric B catches row/col swaps in the fragment maps (guide §3)."""
    from fluxmpi_amd.ops.gemm import conv1x1_dgrad, conv1x1_fwd
    n = 64
    eye = torch.eye(n, device="cuda").to(torch.bfloat16)
    b = (torch.arange(n * n, device="cuda").reshape(n, n) % 97).to(torch.bfloat16)
    assert torch.equal(conv1x1_fwd(eye, b).float(), b.float().t())
    assert torch.equal(conv1x1_dgrad(eye, b).float(), b.float())


@pytest.mark.parametrize("n,h,w,ci,co", [(2, 8, 8, 64, 128), (3, 7, 5, 32, 64), (1, 14, 14, 256, 512)])
@pytest.mark.parametrize("engine", [2, 3, 6, 9])
def test_stride2_rows(gpu_ext, n, h, w, ci, co, engine):
    """a_sub: the stride-2 1x1 convolution as a GEMM whose A rows are gathered from the even
    pixels (odd image sizes included), with the BatchNorm statistics epilogue."""
    from fluxmpi_amd.ops.gemm import SHARDS, gemm
    x = _rand(n, h, w, ci)
    wt = _rand(co, ci) * 0.1
    ho, wo = (h + 1) // 2, (w + 1) // 2
    c = torch.empty(n * ho * wo, co, device="cuda", dtype=torch.bfloat16)
    stats = torch.zeros(SHARDS, 2, co, device="cuda")
    gemm(x.reshape(-1, ci), wt, c, M=n * ho * wo, N=co, K=ci, lda=ci, ldb=ci, ldc=co, mode=1, stats=stats,
         a_sub=(h, w), engine=engine)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), wt.float()[:, :, None, None], stride=2)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, co)
    torch.testing.assert_close(c.float(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2)
    cf = c.float()
    torch.testing.assert_close(stats[:, 0].sum(0), cf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(stats[:, 1].sum(0), (cf * cf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("n,h,w,ci,co", [(2, 8, 8, 64, 128), (3, 7, 5, 32, 64), (2, 14, 14, 256, 512)])
@pytest.mark.parametrize("variant", [1, 2])
def test_wgrad_stride2_rows(gpu_ext, n, h, w, ci, co, variant, monkeypatch):
    """b_sub: the stride-2 1x1 convolution's weight gradient with the B rows gathered from the even
    pixels (odd image sizes, several splits) vs the fp32 reference."""
    from fluxmpi_amd.ops import gemm as G
    monkeypatch.setattr(G, "WGRAD_VARIANT", variant)
    x = _rand(n, ci, h, w).contiguous(memory_format=torch.channels_last)
    ho, wo = (h + 1) // 2, (w + 1) // 2
    dy = _rand(n * ho * wo, co)
    for splits in (1, 3):
        dw = G.conv1x1_wgrad_s2(dy, x, out_dtype=torch.float32, splits=splits)
        xs = x[:, :, ::2, ::2].permute(0, 2, 3, 1).reshape(-1, ci).float()
        ref = dy.float().t() @ xs
        torch.testing.assert_close(dw, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("n,h,w,ci,co", [(2, 8, 8, 32, 64), (3, 7, 5, 32, 32), (2, 14, 14, 64, 128)])
@pytest.mark.parametrize("variant", [1, 2])
def test_wgrad_conv3x3_stride2(gpu_ext, n, h, w, ci, co, variant, monkeypatch):
    """The 3x3 / stride 2 / pad 1 weight gradient over the implicit stride-2 im2col (odd sizes
    included) vs torch's fp32 convolution backward."""
    from fluxmpi_amd.ops import gemm as G
    monkeypatch.setattr(G, "WGRAD_VARIANT", variant)
    x = _rand(n, ci, h, w).contiguous(memory_format=torch.channels_last)
    ho, wo = (h + 1) // 2, (w + 1) // 2
    dy = _rand(n, co, ho, wo).contiguous(memory_format=torch.channels_last)
    for splits in (1, 3):
        dw = G.conv3x3_wgrad_s2(dy, x, splits=splits)
        ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), torch.zeros(co, ci, 3, 3, device="cuda"),
                                                  None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
                                                  [False, True, False])[1]
        torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("n,h,w,ci,co", [(2, 8, 8, 32, 64), (3, 7, 5, 64, 32), (2, 14, 14, 128, 128)])
def test_conv3x3_stride2_fwd(gpu_ext, n, h, w, ci, co):
    """The 3x3 / stride 2 / pad 1 forward on the implicit GEMM (odd sizes included) with the
    BatchNorm statistics epilogue vs torch's fp32 convolution."""
    from fluxmpi_amd.ops.gemm import SHARDS, conv3x3_s2_fwd
    x = _rand(n, ci, h, w).contiguous(memory_format=torch.channels_last)
    wt = _rand(co, ci, 3, 3) * 0.1
    stats = torch.zeros(SHARDS, 2, co, device="cuda")
    y = conv3x3_s2_fwd(x, wt, stats=stats)
    ref = torch.nn.functional.conv2d(x.float(), wt.float(), None, 2, 1)
    assert y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, co)
    torch.testing.assert_close(stats[:, 0].sum(0), yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(stats[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)

