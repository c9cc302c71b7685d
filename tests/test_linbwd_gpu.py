"""linbwd.hip — a token-major Linear's input and weight gradients in one launch — against fp32
PyTorch: both grid orders, several split counts (the last split shorter), the ViT-B/16 widths,
delivery of the weight gradient into a bucket slice, and the Linear modules that route to it."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _run(M, N, K, splits, first, seed=0):
    from fluxmpi_amd.ops import _ext
    C = _ext.get(required=True)
    torch.manual_seed(seed)
    dy = (torch.randn(M, N, device="cuda") * 0.5).bfloat16()
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * N ** -0.5).bfloat16()
    s = C.linear_bwd_splits(M, N, K, splits)
    dx = torch.full((M, K), float("nan"), device="cuda").bfloat16()
    ws = torch.full((s, N, K), float("nan"), device="cuda")
    C.linear_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), dx.data_ptr(), ws.data_ptr(), M, N, K, N, K, K, K, splits,
                 first, torch.cuda.current_stream().cuda_stream)
    ref_dx = dy.float() @ w.float()
    ref_dw = dy.float().t() @ x.float()
    return dx, ws.sum(0), ref_dx, ref_dw


@pytest.mark.parametrize("M,N,K", [(2048, 768, 768), (1024, 2304, 768), (1536, 3072, 768), (512, 768, 3072),
                                   (256, 256, 256)])
@pytest.mark.parametrize("splits,first", [(1, 0), (3, 1), (7, 0)])
def test_linbwd_matches_fp32(gpu_ext, M, N, K, splits, first):
    dx, dw, rdx, rdw = _run(M, N, K, splits, first)
    assert torch.isfinite(dx.float()).all() and torch.isfinite(dw).all()
    assert _rel(dx, rdx) < 5e-3
    assert _rel(dw, rdw) < 2e-3


def test_linbwd_vit_shape(gpu_ext):
    """The ViT-B/16 qkv backward at batch 256 (M = 50432 tokens) at each timed split count."""
    from fluxmpi_amd.ops.linear import linbwd_candidates
    cands, default = linbwd_candidates(50432, 2304, 768, 256)
    assert default in range(1, 65) and all(1 <= c <= 64 for c in cands)
    dx, dw, rdx, rdw = _run(50432, 2304, 768, cands[-1], 0, seed=1)
    assert _rel(dx, rdx) < 5e-3 and _rel(dw, rdw) < 2e-3


def test_dgrad_wgrad_measures_once_and_matches(gpu_ext):
    from fluxmpi_amd.ops import conv_choice
    from fluxmpi_amd.ops.linear import dgrad_wgrad
    torch.manual_seed(3)
    M, N, K = 4096, 768, 768
    dy = (torch.randn(M, N, device="cuda") * 0.5).bfloat16()
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * N ** -0.5).bfloat16()
    conv_choice._LB_CHOICE.clear()
    dx, dw = dgrad_wgrad(dy, x, w, torch.bfloat16)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert (M, N, K, cus) in conv_choice._LB_CHOICE
    assert _rel(dx, dy.float() @ w.float()) < 5e-3 and _rel(dw, dy.float().t() @ x.float()) < 5e-3


@pytest.mark.parametrize("N,K", [(768, 768), (2304, 768)])
def test_linear_module_routes_to_linbwd(gpu_ext, N, K):
    from fluxmpi_amd.ops import graddst
    from fluxmpi_amd.ops.linear import Linear, linbwd_ok
    torch.manual_seed(2)
    lin = Linear(K, N).cuda().bfloat16()
    x = torch.randn(4, 512, K, device="cuda").bfloat16().requires_grad_()
    assert linbwd_ok(torch.empty(2048, N, device="cuda", dtype=torch.bfloat16),
                     torch.empty(2048, K, device="cuda", dtype=torch.bfloat16), lin.weight)
    flat = torch.zeros(lin.weight.numel() + 256, device="cuda", dtype=torch.bfloat16)
    graddst.attach(lin.weight, flat, 128)
    try:
        y = lin(x)
        g = torch.randn_like(y)
        y.backward(g)
        assert graddst.delivered(lin.weight)
        xf = x.detach().float().reshape(-1, K)
        gf = g.float().reshape(-1, N)
        assert _rel(x.grad.reshape(-1, K), gf @ lin.weight.float()) < 5e-3
        assert _rel(lin.weight.grad, gf.t() @ xf) < 2e-3
        assert _rel(lin.bias.grad, gf.sum(0)) < 2e-3
    finally:
        graddst.detach(lin.weight)
