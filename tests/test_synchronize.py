"""Mirror of reference test/test_synchronize.jl (+ FluxMPIFluxModel / nn.Module)."""
from collections import namedtuple

NT = namedtuple("NT", ["a", "d"])


def _rank_array(shape, root_rank):
    import torch
    import fluxmpi_amd as FluxMPI
    return torch.ones(shape) if FluxMPI.local_rank() == root_rank else torch.zeros(shape)


def worker():
    import numpy as np
    import torch
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as Optimisers

    FluxMPI.Init(verbose=True)
    root = 0
    r = FluxMPI.local_rank()

    # NamedTuple-like nested dict
    gs = {"a": {"b": _rank_array((2, 3), root), "c": _rank_array((2, 3), root)}, "d": _rank_array((2, 3), root)}
    gs_ = FluxMPI.synchronize(gs, root_rank=root)
    assert torch.all(gs_["a"]["b"] == 1) and torch.all(gs_["a"]["c"] == 1) and torch.all(gs_["d"] == 1)

    # Optimisers state: Adam (mt, vt, βt)
    st_opt = Optimisers.setup(Optimisers.Adam(0.001), gs)
    if r == root:
        for leaf in (st_opt["a"]["b"], st_opt["a"]["c"], st_opt["d"]):
            leaf.state[0].fill_(1)
            leaf.state[1].fill_(1)
            leaf.state = (leaf.state[0], leaf.state[1], (0.5, 0.25))
    st_opt = FluxMPI.synchronize(st_opt, root_rank=root)
    for leaf in (st_opt["a"]["b"], st_opt["a"]["c"], st_opt["d"]):
        assert torch.all(leaf.state[0] == 1) and torch.all(leaf.state[1] == 1)
        assert leaf.state[2] == (0.5, 0.25)
    # Descent: no state
    st_opt = Optimisers.setup(Optimisers.Descent(0.001), gs)
    FluxMPI.synchronize(st_opt, root_rank=root)

    # ComponentArray analogue: one flat buffer
    gs = {"a": {"b": _rank_array((2, 3), root), "c": _rank_array((2, 3), root)}, "d": _rank_array((2, 3), root)}
    cgs = FluxMPI.FlatParams(gs)
    cgs_ = FluxMPI.synchronize(cgs, root_rank=root)
    assert torch.all(cgs_.a.b == 1) and torch.all(cgs_.a.c == 1) and torch.all(cgs_.d == 1)

    # Tuple
    t = ((_rank_array((2, 3), root), _rank_array((2, 3), root)), _rank_array((2, 3), root))
    t = FluxMPI.synchronize(t, root_rank=root)
    assert torch.all(t[0][0] == 1) and torch.all(t[0][1] == 1) and torch.all(t[1] == 1)
    nt = FluxMPI.synchronize(NT(a=_rank_array((2,), root), d=3.0 * (r + 1)), root_rank=root)
    assert isinstance(nt, NT) and torch.all(nt.a == 1) and nt.d == 3.0

    # Misc
    assert FluxMPI.synchronize(None, root_rank=root) is None
    x = "x" if r == root else "y"
    assert FluxMPI.synchronize(x, root_rank=root) == x  # symbols are not synchronised
    assert FluxMPI.synchronize(FluxMPI.local_rank(), root_rank=root) == root
    assert FluxMPI.synchronize(True if r == root else False, root_rank=root) is True
    assert FluxMPI.synchronize({}, root_rank=root) == {}
    mixed = FluxMPI.synchronize([r, float(r), np.full(3, float(r)), 2j * r], root_rank=root)
    assert mixed[0] == root and mixed[1] == float(root) and np.all(mixed[2] == root) and mixed[3] == 0j

    # tied arrays are broadcast once and stay tied
    w = _rank_array((4,), root)
    tied = FluxMPI.synchronize({"enc": w, "dec": w}, root_rank=root)
    assert tied["enc"] is tied["dec"] and torch.all(w == 1)

    # nn.Module via FluxMPIFluxModel (returns the unwrapped module)
    torch.manual_seed(100 + r)
    m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.BatchNorm1d(4))
    m[1].running_mean.fill_(float(r))
    m2 = FluxMPI.synchronize(FluxMPI.FluxMPIFluxModel(m), root_rank=root)
    assert m2 is m
    ref = FluxMPI.bcast(m[0].weight.detach().clone(), root)
    assert torch.equal(m[0].weight, ref) and torch.all(m[1].running_mean == float(root))

    # non-zero root
    last = FluxMPI.total_workers() - 1
    v = FluxMPI.synchronize({"v": torch.full((3,), float(r))}, root_rank=last)
    assert torch.all(v["v"] == last)
    FluxMPI.Finalize()


def test_synchronize(spmd):
    spmd("tests.test_synchronize:worker")
