"""Self-verification of the device communicator before a measurement.

The driver's multi-GPU scaling runs are the only place RCCL ever sees more than one rank
(the development pool has one GPU per box: ``profiles/r2_probe_rccl_two_ranks_one_gpu.json``),
so a run must prove from the communicator itself that it is what the JSON line claims:
``ncclCommCount`` equals WORLD_SIZE, ``ncclCommUserRank`` equals RANK and ``ncclCommCuDevice``
is the pinned device (reference: the process group is ``MPI.COMM_WORLD``,
/root/reference/src/common.jl:16-45, exercised by 2-4 ranks, /root/reference/test/runtests.jl:3-16).
"""
from __future__ import annotations


class CommSelfCheckError(RuntimeError):
    """The communicator's own report disagrees with the launch (rank count, rank or device)."""


def comm_selfcheck(comm, world: int, rank: int, device_index: int | None) -> dict:
    """Return ``comm.self_report()`` after checking it against the launch; raises
    :class:`CommSelfCheckError` on any mismatch. Backends without a report pass (``{}``)."""
    rep = dict(comm.self_report()) if hasattr(comm, "self_report") else {}
    if not rep:
        return rep
    # RcclComm reports rccl_*; the host-collective backends (gloo on device tensors) comm_*
    pre = "rccl_" if "rccl_nranks" in rep else "comm_"
    nranks, crank, cdev = rep.get(pre + "nranks"), rep.get(pre + "rank"), rep.get(pre + "device")
    problems = []
    if nranks != world:
        problems.append(f"communicator has {nranks} ranks, WORLD_SIZE is {world}")
    if crank != rank:
        problems.append(f"communicator rank {crank} != RANK {rank}")
    if device_index is not None and cdev not in (None, device_index):
        problems.append(f"communicator device {cdev} != pinned device {device_index}")
    if problems:
        raise CommSelfCheckError("; ".join(problems))
    return rep


__all__ = ["CommSelfCheckError", "comm_selfcheck"]
