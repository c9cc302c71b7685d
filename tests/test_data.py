"""Mirror of reference test/test_data.jl (DistributedDataContainer)."""
import math

import pytest


def worker():
    import torch
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import DistributedDataContainer

    g = torch.Generator().manual_seed(19)
    FluxMPI.Init(verbose=True)
    data = torch.randn(10, generator=g)
    W = FluxMPI.total_workers()
    r = FluxMPI.local_rank()
    dc = DistributedDataContainer(data)
    if r != W - 1:
        assert len(dc) == math.ceil(len(data) / W)
    else:
        assert len(dc) == len(data) - math.ceil(len(data) / W) * (W - 1)
    dsum = 0.0
    for i in range(len(dc)):
        dsum += float(dc[i])
    total = FluxMPI.allreduce(torch.tensor([dsum], dtype=torch.float64), "+")[0]
    assert math.isclose(float(total), float(data.double().sum()), rel_tol=1e-6)
    # list-of-samples datasets + fancy indexing
    ds = DistributedDataContainer(list(range(10)))
    j = len(ds) - 1
    assert ds[0] == ds.idxs[0] and ds[[0, j]] == [ds.idxs[0], ds.idxs[j]]
    FluxMPI.Finalize()


@pytest.mark.parametrize("n", [2, 3, 4])
def test_data(spmd, n):
    spmd("tests.test_data:worker", nprocs=n)


def test_partition_formula_and_q6():
    from fluxmpi_amd import DistributedDataContainer
    lens = [len(DistributedDataContainer(list(range(10)), rank=r, world=3)) for r in range(3)]
    assert lens == [4, 4, 2]
    with pytest.raises(ValueError, match="partitions"):
        DistributedDataContainer(list(range(10)), rank=5, world=6)
