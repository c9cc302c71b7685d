"""Hand-written gfx950 HIP kernels (``fluxmpi_amd._C``) and their Python wrappers."""
from . import _ext, multi_tensor, optim  # noqa: F401
