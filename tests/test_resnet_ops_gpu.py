"""ResNet stem / head helpers vs PyTorch: the 3->4 channel pad kernel and the global
average pool with the single-pass backward."""
import pytest
import torch
import torch.nn.functional as F


def test_global_avg_pool_cpu():
    from fluxmpi_amd.models.resnet import global_avg_pool
    for cl in (False, True):
        x = torch.randn(3, 8, 5, 7)
        if cl:
            x = x.contiguous(memory_format=torch.channels_last)
        xa, xr = x.clone().requires_grad_(), x.clone().requires_grad_()
        y = global_avg_pool(xa)
        yr = torch.flatten(F.adaptive_avg_pool2d(xr, 1), 1)
        torch.testing.assert_close(y, yr)
        g = torch.randn_like(yr)
        y.backward(g)
        yr.backward(g)
        torch.testing.assert_close(xa.grad, xr.grad)
        assert xa.grad.is_contiguous(memory_format=torch.channels_last) == cl or not cl


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 3, 224, 224), (3, 3, 7, 5), (1, 3, 1, 3)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_pad_c3_to_c4(gpu_ext, shape, dtype):
    from fluxmpi_amd.ops.pool import pad_c3_to_c4
    x = torch.randn(shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    y = pad_c3_to_c4(x)
    ref = F.pad(x.permute(0, 2, 3, 1), (0, 1)).permute(0, 3, 1, 2)
    assert y.shape == (shape[0], 4, shape[2], shape[3])
    assert torch.equal(y, ref)


@pytest.mark.gpu
def test_global_avg_pool_gpu_bf16(gpu_ext):
    from fluxmpi_amd.models.resnet import global_avg_pool
    x = torch.randn(4, 2048, 7, 7, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xa, xr = x.clone().requires_grad_(), x.float().clone().requires_grad_()
    y = global_avg_pool(xa)
    yr = xr.mean((2, 3))
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(xa.grad.float(), xr.grad, rtol=1e-2, atol=1e-3)
