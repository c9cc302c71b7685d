"""The persistent gemm_nt kernel's schedule (csrc/kernels/gemm_nt.hip: TailPlan / tail_plan, the job
list of gemm_nt_kernel and the split-tile fix-up's slot arithmetic), replayed in Python.

Without split: every tile is computed exactly once, no workgroup gets more than ceil(tiles / G)
tiles and none is idle. With the split tail (stream-K on each XCD's last, partial round): every
(tile, k-tile) unit is computed exactly once, every job has an even number (>= 2) of k-tiles (the
kernel's DMA look-ahead needs two units per job), the pieces of a split tile are exactly the
workgroups wg_of() names, their workspace slots are distinct and below max_q per workgroup, and the
tail is spread evenly (no workgroup takes more than a round's worth of units beyond its full tiles).
"""
import pytest


def _range_start(tiles, g, r):
    return tiles * r // g


class Plan:
    def __init__(self, tiles, G, nk, split, split_min, b):
        q, r = G // 8, G % 8
        xcd, pos = b % 8, b // 8
        gx0 = xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q
        nx = q + (1 if xcd < r else 0)
        tb, te = _range_start(tiles, G, gx0), _range_start(tiles, G, gx0 + nx)
        self.tb, self.nx, self.pos, self.xcd = tb, nx, pos, xcd
        T = te - tb
        F = T // nx if nx else 0
        R = T - F * nx
        self.tt0 = tb + F * nx
        self.s = self.e = 0
        if split and R > 0:
            self.u2 = R * nk // 2
            want = (2 * self.u2) // max(split_min, 2)
            self.nw = min(max(want, 1), nx)
            self.nfull = F
            if pos < self.nw:
                self.s, self.e = self.bnd(pos), self.bnd(pos + 1)
        else:
            self.u2 = self.nw = 0
            self.nfull = F + (1 if pos < R else 0)

    def bnd(self, w):
        return 2 * (self.u2 * w // self.nw)

    def wg_of(self, x):
        return ((x // 2 + 1) * self.nw - 1) // self.u2


def _jobs(plan, nk):
    out = [(plan.tb + plan.pos + j * plan.nx, 0, nk, -1) for j in range(plan.nfull)]
    if plan.e > plan.s:
        for r in range(plan.s // nk, (plan.e - 1) // nk + 1):
            out.append((plan.tt0 + r, max(plan.s - r * nk, 0), min(plan.e - r * nk, nk), r))
    return out


def _host_max_q(tiles, G, nk, sm):
    mq = 0
    for b in range(G):
        p = Plan(tiles, G, nk, 1, sm, b)
        if p.e > p.s:
            mq = max(mq, (p.e - 1) // nk - p.s // nk + 1)
    return mq


def _check(tiles, G, nk, split, sm):
    covered = {}
    slots = set()
    mq = _host_max_q(tiles, G, nk, sm) if split else 0
    per_wg = []
    for b in range(G):
        p = Plan(tiles, G, nk, split, sm, b)
        units = 0
        for tile, k0, k1, r in _jobs(p, nk):
            assert 0 <= tile < tiles
            assert k1 - k0 >= 2 and (k1 - k0) % 2 == 0 and 0 <= k0 < k1 <= nk, (tiles, G, nk, b, k0, k1)
            units += k1 - k0
            for k in range(k0, k1):
                assert (tile, k) not in covered, (tiles, G, nk, tile, k)
                covered[(tile, k)] = b
            if r >= 0:
                x0 = r * nk
                wlo, whi = p.wg_of(x0), p.wg_of(x0 + nk - 1)
                assert wlo <= p.pos <= whi
                assert p.bnd(wlo) <= x0 < p.bnd(wlo + 1) and p.bnd(whi) <= x0 + nk - 1 < p.bnd(whi + 1)
                qw = r - p.bnd(p.pos) // nk
                assert 0 <= qw < mq
                slot = (p.pos * 8 + p.xcd) * mq + qw
                assert slot not in slots
                slots.add(slot)
                # the fix-up's slot of piece pc == this job's own slot when pc == pos - wlo
                assert ((wlo + (p.pos - wlo)) * 8 + p.xcd) * mq + (r - p.bnd(wlo + (p.pos - wlo)) // nk) == slot
        per_wg.append(units)
    assert len(covered) == tiles * nk, (tiles, G, nk, split)
    return per_wg


@pytest.mark.parametrize("cus", [256, 80])
def test_unsplit_every_tile_once_and_balanced(cus):
    for tiles in list(range(1, 600)) + [1773, 2364, 591, 196, 98, 4096]:
        G = min(tiles, cus)
        per_wg = _check(tiles, G, 4, 0, 8)
        assert max(per_wg) <= -(-tiles // G) * 4
        assert min(per_wg) >= 4  # no idle persistent workgroup


@pytest.mark.parametrize("nk,sm", [(12, 8), (36, 8), (48, 8), (16, 8), (48, 16), (72, 8), (36, 2)])
def test_split_tail_covers_every_unit_once(nk, sm):
    G = 256
    for tiles in [591, 2364, 196, 1773, 98, 300, 513, 255, 257, 1000] + list(range(1, 80, 7)):
        per_wg = _check(tiles, G, nk, 1, sm)
        full = tiles // G
        # balanced: at most one full round plus the tail's even share beyond the full tiles
        assert max(per_wg) <= (full + 1) * nk + 2 * nk, (tiles, nk, sm, max(per_wg))
