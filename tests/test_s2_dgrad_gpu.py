"""The stride-2 3x3 input gradient as four parity-class implicit GEMMs (gemm.conv3x3_s2_dgrad,
gemm_glds.hip conv_s = 16 + class) against PyTorch fp32: ResNet-50's three stride-2 3x3 shapes,
the CIFAR DEQ stem, non-square images, and the autograd route through fused_block."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _s2_dgrad_on(monkeypatch):
    """The parity-class path is opt-in (FLUXMPI_S2_DGRAD=1: measured slower than MIOpen on the
    ResNet-50 shapes, profiles/rd6e_s2_dgrad_ab.jsonl); these tests switch it on."""
    from fluxmpi_amd.ops import gemm as G
    monkeypatch.setattr(G, "S2_DGRAD", True)

SHAPES = [(4, 128, 56, 56, 128), (4, 256, 28, 28, 256), (4, 512, 14, 14, 512), (3, 128, 32, 32, 512),
          (2, 64, 10, 6, 96), (1, 32, 2, 2, 64)]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("N,Ci,H,W,Co", SHAPES)
def test_s2_dgrad_matches_fp32(gpu_ext, N, Ci, H, W, Co):
    from fluxmpi_amd.ops import gemm as G
    torch.manual_seed(0)
    x = torch.randn(N, Ci, H, W, device="cuda", requires_grad=True)
    w = (torch.randn(Co, Ci, 3, 3, device="cuda") * (9 * Ci) ** -0.5).bfloat16().contiguous(
        memory_format=torch.channels_last)
    y = F.conv2d(x, w.float(), None, 2, 1)
    dy = torch.randn_like(y).bfloat16().contiguous(memory_format=torch.channels_last)
    y.backward(dy.float())
    assert G.s2_dgrad_ok(dy, w, x.shape)
    G.note_filter(w)
    dx = G.conv3x3_s2_dgrad(dy, w, x.shape)
    assert dx.shape == x.shape and dx.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dx, x.grad) < 5e-3


def test_s2_dgrad_through_autograd(gpu_ext):
    from fluxmpi_amd.ops.fused_block import conv3x3_s2, conv3x3_s2_supported
    torch.manual_seed(1)
    conv = torch.nn.Conv2d(128, 256, 3, stride=2, padding=1, bias=False).cuda().bfloat16().to(
        memory_format=torch.channels_last)
    x = torch.randn(4, 128, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    assert conv3x3_s2_supported(x, conv)
    y = conv3x3_s2(x, conv.weight)
    g = torch.randn_like(y)
    y.backward(g)
    xf = x.detach().float().requires_grad_()
    F.conv2d(xf, conv.weight.float(), None, 2, 1).backward(g.float())
    assert _rel(x.grad, xf.grad) < 5e-3
