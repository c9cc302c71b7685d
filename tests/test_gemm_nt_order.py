"""The persistent gemm_nt kernel's tile assignment (csrc/kernels/gemm_nt.hip, gemm_nt_kernel prologue),
replayed in Python: with either tile order every tile of the grid is computed exactly once, and no
workgroup gets more than ceil(tiles / G) tiles, for any tile count and grid size (G = min(tiles, CUs))."""
import pytest


def _range_start(tiles, g, r):
    return tiles * r // g


def _assignment(tiles, G, order):
    out = {}
    q, r = G // 8, G % 8
    for b in range(G):
        xcd, pos = b % 8, b // 8
        gx0 = xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q
        nx = q + (1 if xcd < r else 0)
        if order == 0:
            base, stride = _range_start(tiles, G, gx0 + pos), 1
            n = _range_start(tiles, G, gx0 + pos + 1) - base
        else:
            tb, te = _range_start(tiles, G, gx0), _range_start(tiles, G, gx0 + nx)
            base, stride = tb + pos, nx
            n = (te - tb - pos + nx - 1) // nx if pos < te - tb else 0
        out[b] = [base + j * stride for j in range(max(n, 0))]
    return out


@pytest.mark.parametrize("cus", [256, 80, 304])
@pytest.mark.parametrize("order", [0, 1])
def test_every_tile_once_and_balanced(cus, order):
    for tiles in list(range(1, 600)) + [1773, 2364, 591, 196, 98, 4096]:
        G = min(tiles, cus)
        a = _assignment(tiles, G, order)
        got = sorted(t for ts in a.values() for t in ts)
        assert got == list(range(tiles)), (tiles, G, order)
        assert max(len(ts) for ts in a.values()) <= -(-tiles // G), (tiles, G, order)
        assert all(len(ts) >= 1 for ts in a.values()), (tiles, G, order)  # no idle persistent workgroup
