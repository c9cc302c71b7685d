"""Import a variant build of the native library (scripts/diag/build_variant.py) as fluxmpi_amd._C,
before anything else imports the package's own copy: FLUXMPI_C_VARIANT=<path to .so>."""
import importlib.machinery
import importlib.util
import os
import sys


def install():
    path = os.environ.get("FLUXMPI_C_VARIANT")
    if not path:
        return None
    import torch  # noqa: F401  (the extension links torch's libraries)
    loader = importlib.machinery.ExtensionFileLoader("fluxmpi_amd._C", os.path.abspath(path))
    spec = importlib.util.spec_from_file_location("fluxmpi_amd._C", os.path.abspath(path), loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules["fluxmpi_amd._C"] = mod
    return mod
