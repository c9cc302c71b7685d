"""Error types.

Mirrors ``FluxMPINotInitializedError`` (reference ``src/FluxMPI.jl:59-63``):
raised by :func:`local_rank` / :func:`total_workers` (and everything that
needs a communicator) before :func:`fluxmpi_amd.Init` was called.
"""


class FluxMPINotInitializedError(RuntimeError):
    """Raised when a FluxMPI function is used before ``Init()``."""

    MESSAGE = "Please call FluxMPI.init(...) before using FluxMPI functionalities!"

    def __init__(self, msg: str | None = None):
        super().__init__(msg or self.MESSAGE)


class NativeExtensionError(RuntimeError):
    """The compiled HIP extension (``fluxmpi_amd._C``) is required but missing.

    On a GPU box the HIP path is mandatory: ops never silently fall back to an
    eager PyTorch implementation there (call ``fluxmpi_amd.build()`` first).
    """


class CollectiveMismatchError(RuntimeError):
    """Ranks disagree about the structure of a bucketed collective.

    The reference would hang in that situation (one MPI call per
    leaf, so a rank with a missing gradient leaf deadlocks). We hash the
    bucket plan across ranks and raise instead.
    """
