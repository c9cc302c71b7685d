"""LDS-halo 3x3 convolution (csrc/kernels/conv3x3.hip) vs an fp32 PyTorch reference: forward
(+ BatchNorm statistics epilogue) and input gradient, on ResNet-50's 3x3 shapes at small
batches (tiles span image rows and images; partial last tiles)."""
import pytest
import torch
import torch.nn.functional as F

from fluxmpi_amd.ops import _ext
from fluxmpi_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _halo_on(monkeypatch):
    monkeypatch.setattr(G, "HALO", True)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("n,h,c,co", [(2, 56, 64, 64), (3, 28, 128, 128), (5, 14, 256, 256), (4, 7, 512, 512),
                                      (1, 9, 32, 64), (2, 28, 128, 64)])
def test_halo_fwd_and_stats(n, h, c, co):
    C = _ext.get(required=True)
    assert C.conv3x3_halo_supported(n, h, h, c, co)
    torch.manual_seed(n * h + c)
    x = torch.randn(n, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, c, 3, 3, device="cuda") * (2.0 / (9 * c)) ** 0.5).bfloat16()
    ws = torch.zeros(64 * 2 * 2048, device="cuda")
    y = G.conv3x3_fwd(x, w, stats=ws)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert _rel(y, ref) < 1e-2, _rel(y, ref)
    sums = ws[: 64 * 2 * co].reshape(64, 2, co).sum(0)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, co)
    assert _rel(sums[0], yf.sum(0)) < 1e-3 and _rel(sums[1], (yf * yf).sum(0)) < 1e-3


@pytest.mark.parametrize("n,h,c,co", [(2, 56, 64, 64), (3, 28, 128, 128), (5, 14, 256, 256), (4, 7, 512, 512)])
def test_halo_dgrad(n, h, c, co):
    torch.manual_seed(7 + n)
    dy = torch.randn(n, co, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, c, 3, 3, device="cuda") * (2.0 / (9 * c)) ** 0.5).bfloat16()
    dx = G.conv3x3_dgrad(dy, w)
    ref = torch.nn.grad.conv2d_input((n, c, h, h), w.float(), dy.float(), padding=1)
    assert _rel(dx, ref) < 1e-2, _rel(dx, ref)
