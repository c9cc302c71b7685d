"""Data-parallel runtime: process group, RCCL communicator, collectives, sync, DDP."""
from .runtime import (Init, Initialized, Finalize, Finalized, local_rank, total_workers,  # noqa: F401
                      fluxmpi_print, fluxmpi_println, barrier, device, backend_name)
from .comm import ReduceOp  # noqa: F401
from .collectives import (COMM_WORLD, Iallreduce, Ibcast, Wait, Waitall, allreduce, bcast, reduce,  # noqa: F401
                          allgather, reduce_scatter, Barrier)
from .sync import FluxMPIFluxModel, synchronize  # noqa: F401
from .optimizer import DistributedOptimizer, allreduce_gradients  # noqa: F401
from .data import DistributedDataContainer  # noqa: F401
from .flat import FlatParams  # noqa: F401
