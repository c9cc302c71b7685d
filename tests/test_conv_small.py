"""ops/conv_small.py: the small-channel 3x3 convolution whose filter gradient is one GEMM over the NHWC
im2col, written into the filter's DDP bucket slice. CPU fp32 against autograd through F.conv2d."""
import pytest
import torch
import torch.nn.functional as F


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("cl", [True, False])
def test_small_conv_grads_match_conv2d(stride, cl):
    from fluxmpi_amd.ops.conv_small import conv3x3_small
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(3, 16, 3, stride=stride, padding=1, bias=False)
    x = torch.randn(4, 3, 12, 10)
    if cl:
        conv = conv.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = conv3x3_small(x, conv)
    g = torch.randn_like(y)
    y.backward(g)
    dw, dx = conv.weight.grad.clone(), x.grad.clone()
    conv.weight.grad = None
    x2 = x.detach().clone().requires_grad_(True)
    ref = F.conv2d(x2, conv.weight, None, stride, 1)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    ref.backward(g)
    torch.testing.assert_close(dw, conv.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dx, x2.grad, rtol=1e-4, atol=1e-4)


def test_small_conv_delivers_into_bucket_slice():
    """With a destination attached (what a communicating DDP engine does), the filter gradient IS
    the slice: no copy left for the bucket pack."""
    from fluxmpi_amd.ops import graddst
    from fluxmpi_amd.ops.conv_small import conv3x3_small
    torch.manual_seed(1)
    conv = torch.nn.Conv2d(3, 8, 3, padding=1, bias=False).to(memory_format=torch.channels_last)
    flat = torch.zeros(conv.weight.numel() + 64)
    graddst.attach(conv.weight, flat, 64)
    try:
        x = torch.randn(2, 3, 8, 8).contiguous(memory_format=torch.channels_last)
        conv3x3_small(x, conv).sum().backward()
        assert graddst.delivered(conv.weight)
        ref = torch.nn.grad.conv2d_weight(x, conv.weight.shape, torch.ones(2, 8, 8, 8), padding=1)
        torch.testing.assert_close(conv.weight.grad, ref, rtol=1e-4, atol=1e-4)
    finally:
        graddst.detach(conv.weight)
