"""conv_c3.hip — the 3-input-channel 3x3 convolution (the CIFAR DEQ stem) forward and filter
gradient on packed-bf16 dot products, against PyTorch fp32: stride 1 and 2, odd sizes (the last
workgroup's partial pixel range, an odd pixel count for the pixel-pair packing), image borders,
several Cout column blocks, and delivery of the filter gradient into a bucket slice."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(256, 32, 32, 1, 128), (4, 32, 32, 2, 128), (3, 7, 9, 1, 256), (5, 17, 13, 2, 128), (1, 1, 1, 1, 128),
          (2, 64, 48, 1, 384)]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("N,H,W,stride,co", SHAPES)
def test_conv_c3_fwd_and_wgrad(gpu_ext, N, H, W, stride, co):
    from fluxmpi_amd.ops.conv_small import _native, conv3x3_small
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(3, co, 3, stride=stride, padding=1, bias=False).cuda().bfloat16()
    conv = conv.to(memory_format=torch.channels_last)
    x = torch.randn(N, 3, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    assert _native(x, conv.weight, stride, 1) is not None
    y = conv3x3_small(x, conv)
    ref = F.conv2d(x.float(), conv.weight.float(), None, stride, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 5e-3
    g = torch.randn_like(ref).bfloat16().contiguous(memory_format=torch.channels_last)
    y.backward(g)
    wref = torch.nn.grad.conv2d_weight(x.float(), conv.weight.shape, g.float(), stride=stride, padding=1)
    assert conv.weight.grad.shape == conv.weight.shape
    assert _rel(conv.weight.grad, wref) < 1e-2


def test_conv_c3_wgrad_into_bucket_slice(gpu_ext):
    from fluxmpi_amd.ops import graddst
    from fluxmpi_amd.ops.conv_small import conv3x3_small
    torch.manual_seed(1)
    conv = torch.nn.Conv2d(3, 128, 3, padding=1, bias=False).cuda().bfloat16().to(memory_format=torch.channels_last)
    flat = torch.zeros(conv.weight.numel() + 64, device="cuda", dtype=torch.bfloat16)
    graddst.attach(conv.weight, flat, 64)
    try:
        x = torch.randn(8, 3, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        conv3x3_small(x, conv).float().sum().backward()
        assert graddst.delivered(conv.weight)
        ref = torch.nn.grad.conv2d_weight(x.float(), conv.weight.shape, torch.ones(8, 128, 16, 16, device="cuda"),
                                          padding=1)
        assert _rel(conv.weight.grad, ref) < 1e-2
    finally:
        graddst.detach(conv.weight)
