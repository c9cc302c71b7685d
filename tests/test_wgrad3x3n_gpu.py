"""wgrad3x3n.hip — the narrow-channel (C in {64, 128}) 3x3 / stride 1 weight gradient with the input
rows staged once per block of 4 image rows — against PyTorch fp32 (the filter gradient of
F.conv2d on the same bf16 operands): every variant and split count, the ResNet-50 stage 1 / 2
shapes, rows whose width leaves a partial last k-step (W % 8 == 4), several output-channel
groups (Cout > 64; variant bit 2: 128-channel groups where Cout % 128 == 0, else 64), and the
autotuned route through the fused 3x3 block."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, C, Cout, H, W)
SHAPES = [(8, 64, 64, 56, 56), (8, 128, 128, 28, 28), (2, 64, 64, 8, 16), (3, 64, 128, 12, 20),
          (2, 128, 64, 4, 28), (1, 64, 64, 4, 4), (2, 128, 128, 8, 12)]


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _ref(x, dy, co):
    xf = x.float().requires_grad_(False)
    w = torch.zeros(co, x.shape[1], 3, 3, device=x.device, requires_grad=True)
    F.conv2d(xf, w, padding=1).backward(dy.float())
    return w.grad


@pytest.mark.parametrize("N,C,CO,H,W", SHAPES)
@pytest.mark.parametrize("cfg", [(1, 256), (0, 256), (1, 512), (0, 7), (2, 256), (2, 7), (2, 5), (1, 5), (5, 256),
                                 (4, 256), (5, 7), (4, 5)])
def test_wgrad3x3n_matches_fp32(gpu_ext, N, C, CO, H, W, cfg):
    from fluxmpi_amd.ops import gemm as G
    torch.manual_seed(0)
    x = _nhwc(torch.randn(N, C, H, W, device="cuda").bfloat16())
    dy = _nhwc(torch.randn(N, CO, H, W, device="cuda").bfloat16())
    assert G.wgrad3x3n_ok(tuple(x.shape), CO)
    ref = _ref(x, dy, CO)
    dw = G.conv3x3_wgrad_n(dy, x, *cfg)
    assert dw.shape == ref.shape and dw.dtype == torch.bfloat16
    assert dw.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dw, ref) < 5e-3
    # the same as the split-K im2col kernel it replaces
    assert _rel(dw, G.conv3x3_wgrad(dy, x)) < 5e-3


def test_wgrad3x3n_support_bounds(gpu_ext):
    from fluxmpi_amd.ops import gemm as G
    assert G.wgrad3x3n_ok((256, 64, 56, 56), 64) and G.wgrad3x3n_ok((256, 128, 28, 28), 128)
    assert not G.wgrad3x3n_ok((2, 256, 14, 14), 256)  # C beyond the narrow kernel
    assert not G.wgrad3x3n_ok((2, 64, 14, 14), 64)    # H not a multiple of the 4-row block
    assert not G.wgrad3x3n_ok((2, 64, 8, 64), 64)     # W beyond the staged row
    assert not G.wgrad3x3n_ok((2, 128, 8, 32), 128)
    assert not G.wgrad3x3n_ok((2, 64, 8, 18), 64)     # W % 4 != 0
    assert not G.wgrad3x3n_ok((2, 64, 8, 16), 96)     # Cout % 64 != 0


def test_wgrad3x3n_through_fused_conv(gpu_ext, monkeypatch):
    """The fused 3x3 block's backward offers the kernel to the weight-gradient autotune; forced
    choice: its gradient matches fp32 autograd."""
    from fluxmpi_amd.ops import conv_choice as CC
    from fluxmpi_amd.ops import fused_block as fb
    torch.manual_seed(2)
    N, C, H, W = 4, 64, 8, 56
    x = _nhwc(torch.randn(N, C, H, W, device="cuda").bfloat16())
    wt = _nhwc((torch.randn(C, C, 3, 3, device="cuda") * (9 * C) ** -0.5).bfloat16()).requires_grad_(True)
    dy = _nhwc(torch.randn(N, C, H, W, device="cuda").bfloat16())
    key = ("3x3", tuple(x.shape), C)
    monkeypatch.setitem(CC._WG_CHOICE, key, ("w3n", (1, 256)))
    y = fb.conv3x3(x, wt)
    y.backward(dy)
    assert _rel(wt.grad, _ref(x, dy, C)) < 5e-3
