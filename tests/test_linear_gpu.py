"""Token-major Linear backward kernels (ops/linear.py) vs fp32 PyTorch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [8, 768, 2304, 3072, 5000 // 8 * 8])
@pytest.mark.parametrize("rows", [1, 63, 1000, 50432])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_colsum_bias_grad(gpu_ext, n, rows, dtype):
    from fluxmpi_amd.ops.linear import bias_grad
    if rows * n > 60_000_000:
        pytest.skip("size")
    g = torch.Generator(device="cuda").manual_seed(rows + n)
    dy = torch.randn(rows, n, device="cuda", generator=g).to(dtype)
    ref = dy.double().sum(0)
    for odt in (torch.float32, torch.bfloat16):
        out = bias_grad(dy, odt)
        assert out.dtype == odt and out.shape == (n,)
        tol = 1e-4 * max(1.0, rows ** 0.5) if odt == torch.float32 else 1e-2 * max(1.0, rows ** 0.5)
        torch.testing.assert_close(out.double(), ref, rtol=1e-2 if odt == torch.bfloat16 else 1e-5, atol=tol)


@pytest.mark.parametrize("shape", [(2304, 768), (768, 768), (3072, 768), (768, 3072), (64, 40)])
def test_linear_backward_matches_fp32(gpu_ext, shape):
    from fluxmpi_amd.ops.linear import Linear
    n_out, n_in = shape
    torch.manual_seed(0)
    lin = Linear(n_in, n_out).cuda().to(torch.bfloat16)
    ref = torch.nn.Linear(n_in, n_out).cuda()
    ref.load_state_dict({k: v.float() for k, v in lin.state_dict().items()})
    x = torch.randn(8, 197, n_in, device="cuda").to(torch.bfloat16).requires_grad_()
    xr = x.detach().float().requires_grad_()
    g = torch.randn(8, 197, n_out, device="cuda").to(torch.bfloat16)
    lin(x).backward(g)
    ref(xr).backward(g.float())
    M = 8 * 197
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2 * (n_out ** 0.5) / 10)
    scale = (M ** 0.5)
    torch.testing.assert_close(lin.weight.grad.float(), ref.weight.grad, rtol=2e-2, atol=2e-2 * scale)
    torch.testing.assert_close(lin.bias.grad.float(), ref.bias.grad, rtol=2e-2, atol=2e-2 * scale)


def test_linear_gelu_wgrad_native(gpu_ext):
    from fluxmpi_amd.ops.gelu import linear_gelu
    torch.manual_seed(1)
    w = (torch.randn(3072, 768, device="cuda") * 0.02).to(torch.bfloat16).requires_grad_()
    b = torch.zeros(3072, device="cuda", dtype=torch.bfloat16).requires_grad_()
    x = torch.randn(4, 197, 768, device="cuda").to(torch.bfloat16).requires_grad_()
    gy = torch.randn(4, 197, 3072, device="cuda").to(torch.bfloat16)
    linear_gelu(x, w, b).backward(gy)
    wr, br, xr = (t.detach().float().requires_grad_() for t in (w, b, x))
    from fluxmpi_amd.ops.gelu import gelu
    gelu(torch.nn.functional.linear(xr, wr, br)).backward(gy.float())
    # dh is rounded to bf16 before both GEMMs (as in the torch path): compare against the
    # fp32 reference at the error the bf16 torch GEMM of the same dh makes, with margin
    from fluxmpi_amd.ops.gelu import gelu_bwd_bias
    h = torch.nn.functional.linear(x.detach(), w.detach(), b.detach())
    dh, _ = gelu_bwd_bias(gy, h, torch.bfloat16)
    dw_torch = (dh.reshape(-1, 3072).t() @ x.detach().reshape(-1, 768)).float()
    e_ours = (w.grad.float() - wr.grad).abs().max()
    e_torch = (dw_torch - wr.grad).abs().max()
    assert e_ours <= 1.5 * e_torch + 1e-3, (float(e_ours), float(e_torch))
    # db sums 788 bf16-rounded dh values (like the torch path) and is stored in bf16
    torch.testing.assert_close(b.grad.float(), br.grad, rtol=1e-2, atol=0.25)


@pytest.mark.parametrize("shape", [(256, 256), (768, 768), (3072, 768), (768, 3072), (512, 1024)])
@pytest.mark.parametrize("K", [64, 1000, 50432])
@pytest.mark.parametrize("splits", [None, 1, 3, 28])
def test_wgrad256_matches_fp32(gpu_ext, shape, K, splits):
    """The 256x256-tile weight-gradient kernel (wgrad256.hip) vs an fp32 GEMM of the same bf16 operands."""
    from fluxmpi_amd.ops.linear import weight_grad
    n_out, n_in = shape
    if K * (n_out + n_in) > 120_000_000:
        pytest.skip("size")
    assert gpu_ext.wgrad256_supported(n_out, n_in, K, n_out, n_in)
    g = torch.Generator(device="cuda").manual_seed(K + n_out)
    dy = torch.randn(K, n_out, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(K, n_in, device="cuda", generator=g).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = weight_grad(dy, x, torch.float32, splits=splits)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)
    outb = weight_grad(dy, x, torch.bfloat16, splits=splits)
    torch.testing.assert_close(outb.float(), ref, rtol=1e-2, atol=1e-2 * K ** 0.5)


def test_wgrad256_strided_rows(gpu_ext):
    """Row strides wider than the matrix (a column slice of a packed projection)."""
    from fluxmpi_amd.ops.linear import weight_grad
    K = 4096
    big = torch.randn(K, 1024, device="cuda").to(torch.bfloat16)
    x = torch.randn(K, 512, device="cuda").to(torch.bfloat16)
    dy = big[:, 256:768]
    ref = dy.float().t() @ x.float()
    out = weight_grad(dy, x, torch.float32)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)
