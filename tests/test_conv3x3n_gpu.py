"""conv3x3n.hip — the narrow-channel (C = Cout in {64, 128}) 3x3 / stride 1 implicit GEMM with the
input halo staged once per 256-pixel tile — against PyTorch fp32: forward (+ BatchNorm statistics
epilogue) and input gradient, at the ResNet-50 stage 1 / 2 shapes and at tiles that span image rows
and image boundaries (every padding case), the widest supported images (W = 64 / 32)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(4, 64, 56, 56), (16, 128, 28, 28), (4, 64, 8, 8), (2, 64, 16, 24), (3, 128, 16, 16), (1, 64, 64, 64),
          (2, 128, 32, 32), (16, 64, 7, 16), (96, 128, 28, 28)]


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("N,C,H,W", SHAPES)
def test_conv3x3n_fwd_stats(gpu_ext, N, C, H, W):
    from fluxmpi_amd.ops import gemm as G
    torch.manual_seed(0)
    x = _nhwc(torch.randn(N, C, H, W, device="cuda").bfloat16())
    w = _nhwc((torch.randn(C, C, 3, 3, device="cuda") * (9 * C) ** -0.5).bfloat16())
    assert G.conv_n_ok(N * H * W, C, C, H, W, x, w.permute(0, 2, 3, 1).contiguous(), x)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    for _ in range(2):
        stats = torch.zeros(G.SHARDS, 2, C, device="cuda")
        y = G.conv3x3_fwd(x, w, stats=stats)
        assert y.is_contiguous(memory_format=torch.channels_last) and y.shape == ref.shape
        assert _rel(y, ref) < 5e-3
        yb = y.float()
        torch.testing.assert_close(stats[:, 0].sum(0), yb.sum((0, 2, 3)), rtol=1e-3, atol=5e-2)
        torch.testing.assert_close(stats[:, 1].sum(0), (yb * yb).sum((0, 2, 3)), rtol=1e-3, atol=5e-2)
    y0 = G.conv3x3_fwd(x, w)
    assert torch.equal(y0, y)  # the statistics epilogue does not change the output


@pytest.mark.parametrize("N,C,H,W", SHAPES)
def test_conv3x3n_dgrad(gpu_ext, N, C, H, W):
    from fluxmpi_amd.ops import gemm as G
    torch.manual_seed(1)
    x = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    w = (torch.randn(C, C, 3, 3, device="cuda") * (9 * C) ** -0.5).bfloat16()
    dy = _nhwc(torch.randn(N, C, H, W, device="cuda").bfloat16())
    F.conv2d(x, w.float(), padding=1).backward(dy.float())
    G.note_filter(w)
    dx = G.conv3x3_dgrad(dy, _nhwc(w))
    assert dx.shape == x.shape and dx.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dx, x.grad) < 5e-3


@pytest.mark.parametrize("tail_co", [32, 16])
def test_conv3x3n_tail_split(gpu_ext, tail_co):
    """More 256-pixel tiles than the 128-channel kernel has resident slots on THIS device: the
    leftover tiles run as 32-output-channel workgroups (more than slots / 8 left) or 16-channel
    ones (at most slots / 8 left). Shapes derived from the runtime slot count, one
    16 x 16 image = one tile."""
    from fluxmpi_amd.ops import _ext
    slots = _ext.get(required=True).conv3x3n_slots128()
    rem = slots // 8 + 2 if tail_co == 32 else max(1, slots // 16)
    assert (rem * 8 > slots) == (tail_co == 32) and rem * 4 <= slots
    n = slots + rem
    test_conv3x3n_fwd_stats(gpu_ext, n, 128, 16, 16)
    test_conv3x3n_dgrad(gpu_ext, n, 128, 16, 16)


def test_conv3x3n_unsupported_routes_elsewhere(gpu_ext):
    from fluxmpi_amd.ops import gemm as G
    x = torch.zeros(8, device="cuda", dtype=torch.bfloat16)
    assert not G.conv_n_ok(300, 64, 64, 10, 30, x)       # pixels not a multiple of 256
    assert not G.conv_n_ok(256 * 10, 64, 128, 16, 16, x)  # C != Cout
    assert not G.conv_n_ok(256 * 40, 128, 128, 40, 64, x)  # W beyond the C = 128 halo
    assert G.conv_n_ok(802816, 64, 64, 56, 56, x) and G.conv_n_ok(200704, 128, 128, 28, 28, x)
