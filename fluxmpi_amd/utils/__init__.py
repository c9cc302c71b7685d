"""Utilities: configuration, errors, pytree walker, profiling."""
from .config import Config, disable_cudampi_support, get_config  # noqa: F401
from .errors import CollectiveMismatchError, FluxMPINotInitializedError, NativeExtensionError  # noqa: F401
from .tree import fmap, leaves, register_node  # noqa: F401
