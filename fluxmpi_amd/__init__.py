"""fluxmpi_amd — MI355X-native distributed data-parallel training (FluxMPI.jl capabilities).

Public API (reference ``src/FluxMPI.jl:88-96`` exports + qualified names)::

    import fluxmpi_amd as FluxMPI

    FluxMPI.Init()                                   # process group + GPU + RCCL communicator
    FluxMPI.local_rank(), FluxMPI.total_workers()
    ps = FluxMPI.synchronize(ps, root_rank=0)        # bucketed RCCL broadcast
    opt = FluxMPI.DistributedOptimizer(FluxMPI.optimisers.Adam(1e-3))
    st = FluxMPI.optimisers.setup(opt, ps)
    st = FluxMPI.synchronize(st, root_rank=0)
    st, ps = FluxMPI.optimisers.update(st, ps, gs)   # SUM-allreduce + fused HIP Adam
    FluxMPI.fluxmpi_println("loss ", l)              # rank-ordered printing

plus the comm primitives ``allreduce``/``bcast``/``reduce``/``Iallreduce``/``Ibcast``,
``allreduce_gradients``, ``DistributedDataContainer``, ``FluxMPIFluxModel``,
``FlatParams`` (ComponentArray analogue) and the high-performance
:class:`fluxmpi_amd.parallel.ddp.DDP` engine (flat bucket views, backward/comm
overlap, fused optimiser, HIP-graph capture).
"""
from __future__ import annotations

import torch  # noqa: F401  (loads libamdhip64 / librccl before our extension)

from . import optimisers, ops, utils  # noqa: F401
from .parallel import (COMM_WORLD, Barrier, DistributedDataContainer, DistributedOptimizer,  # noqa: F401
                       Finalize, Finalized, FlatParams, FluxMPIFluxModel, Iallreduce, Ibcast, Init, Initialized,
                       ReduceOp, Wait, Waitall, allgather, allreduce, allreduce_gradients, backend_name, barrier,
                       bcast, device, fluxmpi_print, fluxmpi_println, local_rank, reduce, reduce_scatter,
                       synchronize, total_workers)
from .utils.config import disable_cudampi_support  # noqa: F401
from .utils.errors import FluxMPINotInitializedError  # noqa: F401

__version__ = "0.1.0"

# Julia spellings
synchronize_ = synchronize
allreduce_ = allreduce
bcast_ = bcast
reduce_ = reduce
Iallreduce_ = Iallreduce
Ibcast_ = Ibcast


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the gfx950 native library in-tree (``fluxmpi_amd/_C*.so``)."""
    from ._build import build as _b

    return _b(force=force, verbose=verbose)


__all__ = [
    "Init", "Initialized", "Finalize", "Finalized", "local_rank", "total_workers", "fluxmpi_print",
    "fluxmpi_println", "synchronize", "DistributedOptimizer", "allreduce_gradients", "DistributedDataContainer",
    "FluxMPIFluxModel", "FlatParams", "allreduce", "bcast", "reduce", "Iallreduce", "Ibcast", "Wait", "Waitall",
    "allgather", "reduce_scatter", "COMM_WORLD", "ReduceOp", "disable_cudampi_support",
    "FluxMPINotInitializedError", "optimisers", "build", "barrier", "Barrier", "device", "backend_name",
]
