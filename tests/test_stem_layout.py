"""CPU checks of the MFMA stem's packed-K layout (fluxmpi_amd/ops/stem.py, csrc/kernels/stem.hip):
the im2col-through-chunks evaluation equals conv2d(stride 2, pad 3), and the filter-gradient
unpack map is the adjoint of the filter pack."""
import torch
import torch.nn.functional as F

from fluxmpi_amd.ops import stem as S


def test_emulated_layout_matches_conv2d():
    torch.manual_seed(0)
    for h in (16, 22):
        x = torch.randn(2, 3, h, h)
        w = torch.randn(64, 3, 7, 7)
        ref = F.conv2d(x, w, stride=2, padding=3)
        out = S.emulate_conv(x, w)
        assert (out - ref).abs().max() <= 1e-4 * ref.abs().max()


def test_pack_unpack_are_adjoint():
    torch.manual_seed(1)
    w = torch.randn(64, 3, 7, 7)
    g = torch.randn(64, 256)
    fwd, bwd = S._maps_cpu(3)
    wp = torch.cat([w.reshape(-1), torch.zeros(1)])[fwd]
    perm = torch.tensor([S._row_channel(r) for r in range(64)])
    assert sorted(perm.tolist()) == list(range(64))
    wnat = torch.empty_like(wp)
    wnat[perm] = wp
    lhs = (wnat * g).sum()
    rhs = (w * g.reshape(-1)[bwd]).sum()
    assert torch.allclose(lhs, rhs, rtol=1e-5, atol=1e-4)
    # every real tap appears exactly once in the packed filter
    real = fwd[fwd < 64 * 3 * 49]
    assert real.numel() == 64 * 147 and real.unique().numel() == 64 * 147
