"""Fused NHWC BatchNorm(+ReLU)(+residual) vs the PyTorch fp32 composition."""
import pytest
import torch
import torch.nn.functional as F


def _ref(x, w, b, rm, rv, relu, res, training=True):
    y = F.batch_norm(x.float(), rm, rv, w, b, training, 0.1, 1e-5)
    if res is not None:
        y = y + res.float()
    return F.relu(y) if relu else y


def test_module_cpu_matches_batchnorm2d():
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    torch.manual_seed(0)
    a, b = FusedBatchNorm2d(16), torch.nn.BatchNorm2d(16)
    x = torch.randn(4, 16, 5, 5, requires_grad=True)
    x2 = x.detach().clone().requires_grad_()
    r = torch.randn(4, 16, 5, 5)
    y1 = a(x, relu=True, residual=r)
    y2 = F.relu(b(x2) + r)
    torch.testing.assert_close(y1, y2)
    y1.sum().backward()
    y2.sum().backward()
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a.running_var, b.running_var)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 8, 3, 5), (4, 64, 14, 14), (8, 256, 7, 7), (3, 2048, 2, 3), (5, 96, 9, 9),
                                   (64, 128)])
@pytest.mark.parametrize("relu,use_res", [(False, False), (True, False), (True, True)])
def test_fused_bn_gpu(gpu_ext, dtype, shape, relu, use_res):
    from fluxmpi_amd.ops.batchnorm import fused_batch_norm
    torch.manual_seed(1)
    dev = "cuda"
    C = shape[1]
    x = (torch.randn(shape, device=dev) * 2 + 0.5)
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    x = x.to(dtype).requires_grad_()
    res = torch.randn(shape, device=dev).to(dtype) if use_res else None
    if res is not None and res.dim() == 4:
        res = res.contiguous(memory_format=torch.channels_last).requires_grad_()
    elif res is not None:
        res.requires_grad_()
    w = (torch.rand(C, device=dev) + 0.5).requires_grad_()
    b = torch.randn(C, device=dev).requires_grad_()
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm.clone(), rv.clone()
    y = fused_batch_norm(x, w, b, rm, rv, True, 0.1, 1e-5, relu, res)

    xr = x.detach().float().requires_grad_()
    resr = res.detach().float().requires_grad_() if res is not None else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = _ref(xr, wr, br, rm2, rv2, relu, resr)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv, rv2, rtol=1e-4, atol=1e-5)
    g = torch.randn(shape, device=dev)
    (y.float() * g).sum().backward()
    (yr * g).sum().backward()
    gtol = dict(rtol=1e-3, atol=1e-3) if dtype == torch.float32 else dict(rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, **gtol)
    torch.testing.assert_close(w.grad, wr.grad, rtol=1e-2 if dtype != torch.float32 else 1e-3, atol=gtol["atol"] * 4)
    torch.testing.assert_close(b.grad, br.grad, rtol=1e-2 if dtype != torch.float32 else 1e-3, atol=gtol["atol"] * 4)
    if use_res:
        torch.testing.assert_close(res.grad.float(), resr.grad, **gtol)


@pytest.mark.gpu
def test_fused_bn_eval_gpu(gpu_ext):
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    m = FusedBatchNorm2d(64).cuda()
    m.running_mean.uniform_(-1, 1)
    m.running_var.uniform_(0.5, 2)
    m.eval()
    x = torch.randn(4, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(x, relu=True)
        ref = F.relu(F.batch_norm(x, m.running_mean, m.running_var, m.weight, m.bias, False, 0.1, m.eps))
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_resnet_fused_vs_torch_norm(gpu_ext):
    """One training step of a small bottleneck ResNet: fused BN == nn.BatchNorm2d (fp32)."""
    from fluxmpi_amd.models import resnet18ish
    torch.manual_seed(0)
    a = resnet18ish(norm="fused").cuda().to(memory_format=torch.channels_last)
    b = resnet18ish(norm="torch").cuda().to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    x = torch.randn(4, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    ya, yb = a(x), b(x)
    torch.testing.assert_close(ya, yb, rtol=1e-3, atol=1e-3)
    ya.square().sum().backward()
    yb.square().sum().backward()
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        # deep-chain gradients accumulate fp32 rounding differences elementwise; compare norms
        rel = float((p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-12))
        assert rel < 5e-3, f"{n}: relative grad error {rel:.2e}"


@pytest.mark.gpu
@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 32, 32), 3, 2, 1), ((2, 16, 17, 15), 3, 2, 1),
                                          ((2, 32, 12, 12), 2, 2, 0), ((3, 8, 9, 11), 3, 1, 1),
                                          ((2, 24, 10, 10), 3, 2, 1)])
def test_bn_relu_maxpool_vs_reference(gpu_ext, shape, k, s, p):
    """Fused stem tail vs max_pool2d(relu(batch_norm(x))) in fp32 on the same bf16 input."""
    import torch.nn.functional as F
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    from fluxmpi_amd.ops.pool import bn_relu_maxpool
    torch.manual_seed(3)
    n, c, h, w = shape
    x = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    bn = FusedBatchNorm2d(c).cuda()
    with torch.no_grad():
        bn.weight.uniform_(-1.5, 1.5)  # negative scales: the max must be taken after the affine
        bn.bias.uniform_(-0.5, 0.5)
    ref_bn = torch.nn.BatchNorm2d(c).cuda()
    ref_bn.load_state_dict(bn.state_dict())
    xa = x.clone().requires_grad_()
    xr = x.float().clone().requires_grad_()
    y = bn_relu_maxpool(xa, bn, k, s, p)
    yr = F.max_pool2d(F.relu(ref_bn(xr)), k, s, p)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-3, atol=1e-4)
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1
    g = torch.randn_like(yr)
    (y.float() * g).sum().backward()
    (yr * g).sum().backward()
    rel = lambda a, b: float((a.float() - b.float()).norm() / b.float().norm())  # noqa: E731
    assert rel(xa.grad, xr.grad) < 3e-2
    assert rel(bn.weight.grad, ref_bn.weight.grad) < 2e-2
    assert rel(bn.bias.grad, ref_bn.bias.grad) < 2e-2


def test_bn_relu_maxpool_cpu_fallback():
    import torch.nn.functional as F
    from fluxmpi_amd.ops.pool import bn_relu_maxpool
    x = torch.randn(2, 8, 10, 10)
    bn = torch.nn.BatchNorm2d(8)
    ref = torch.nn.BatchNorm2d(8)
    y = bn_relu_maxpool(x, bn)
    torch.testing.assert_close(y, F.max_pool2d(F.relu(ref(x)), 3, 2, 1))
    torch.testing.assert_close(bn.running_mean, ref.running_mean)


def test_side_grad_link_never_drops_or_doubles():
    """SideGradLink: delivered when the producer runs first; handed back to autograd when the
    consumer already ran (closed link) — the gradient is counted exactly once either way."""
    from fluxmpi_amd.ops.batchnorm import SideGradLink
    g = torch.ones(3)
    lk = SideGradLink()
    assert lk.offer(g)  # producer first: accepted
    assert lk.take() is g and lk.delivered and lk.grad is None
    lk = SideGradLink()
    assert lk.take() is None and not lk.delivered  # consumer first: closes the link
    assert not lk.offer(g)  # producer must return its gradient itself
