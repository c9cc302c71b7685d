"""conv1x1n.hip — the narrow-K (K in {64, 128}) 1x1 forward with the BatchNorm statistics epilogue,
persistent over 128-row tiles of 256-column slices — against PyTorch fp32, at the ResNet-50
stage-1 / 2 expansion shapes (scaled-down batches), a single tile, several column slices and tile
counts that do not divide by the grid; and the model's routing to it."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (M, K, N)
SHAPES = [(12544, 64, 256), (6272, 128, 512), (128, 64, 256), (4736, 64, 512), (25088, 128, 256),
          (128 * 257, 64, 768)]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("m,k,n", SHAPES)
def test_conv1x1n_fwd_stats(gpu_ext, m, k, n):
    from fluxmpi_amd.ops import gemm as G
    torch.manual_seed(0)
    x = torch.randn(m, k, device="cuda").bfloat16()
    w = (torch.randn(n, k, device="cuda") * k ** -0.5).bfloat16()
    assert G.conv1x1n_ok(m, k, n, x, w)
    ref = x.float() @ w.float().t()
    y0 = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    G.conv1x1n(x, w, y0)
    assert _rel(y0, ref) < 5e-3
    for _ in range(2):
        stats = torch.zeros(G.SHARDS, 2, n, device="cuda")
        y = torch.empty_like(y0)
        G.conv1x1n(x, w, y, stats)
        assert torch.equal(y, y0)  # the statistics epilogue does not change the output
        yf = y.float()
        torch.testing.assert_close(stats[:, 0].sum(0), yf.sum(0), rtol=1e-3, atol=5e-2)
        torch.testing.assert_close(stats[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-3, atol=5e-2)


def test_conv1x1n_unsupported(gpu_ext):
    from fluxmpi_amd.ops import gemm as G
    x = torch.randn(256, 96, device="cuda").bfloat16()
    assert not G.conv1x1n_ok(256, 96, 256, x)                      # K
    assert not G.conv1x1n_ok(200, 64, 256, x)                      # M % 128
    assert not G.conv1x1n_ok(256, 64, 320, x)                      # N % 256
    assert not G.conv1x1n_ok(256, 64, 256, x.float())              # dtype


def test_fwd1x1_routes_to_conv1x1n(gpu_ext):
    """The hybrid blocks' 1x1 forward with statistics (fused_block._fwd1x1_stats) takes the narrow-K
    kernel for a stage-1 expansion and matches conv2d."""
    from fluxmpi_amd.ops import fused_block as fb
    from fluxmpi_amd.ops import gemm as G
    torch.manual_seed(1)
    x = torch.randn(4, 64, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(256, 64, 1, 1, device="cuda") * 0.125).bfloat16().contiguous(memory_format=torch.channels_last)
    assert G.conv1x1n_ok(4 * 16 * 16, 64, 256, fb._nhwc2d(x), w.reshape(256, 64))
    stats = torch.zeros(G.SHARDS, 2, 256, device="cuda")
    c = fb._fwd1x1_stats(x, w, stats)
    ref = torch.nn.functional.conv2d(x.float(), w.float())
    assert c.is_contiguous(memory_format=torch.channels_last) and _rel(c, ref) < 5e-3
    torch.testing.assert_close(stats[:, 0].sum(0), c.float().sum((0, 2, 3)), rtol=1e-3, atol=5e-2)
