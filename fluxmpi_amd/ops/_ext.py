"""Loader for the in-tree native extension ``fluxmpi_amd._C``.

``_C`` is one shared object, built by ``fluxmpi_amd/_build.py`` with hipcc for
gfx950, that contains

* the CDNA4 HIP kernels (multi-tensor pack/unpack/scale, fused Adam/SGD
  families, fused BatchNorm(+ReLU) for NHWC), and
* the native RCCL communicator (``csrc/comm/rccl_comm.cpp``).

The binding layer is plain pybind11 that takes raw device pointers and a HIP
stream handle, so the kernels are independent of the ATen C++ ABI and can be
launched on any PyTorch stream (including inside HIP-graph capture).

Policy: on a machine with a GPU the native path is mandatory. If the
extension is missing we raise :class:`NativeExtensionError` instead of
silently running an eager PyTorch fallback (``FLUXMPI_ALLOW_FALLBACK=1``
overrides this for debugging only). On CPU-only machines the kernels are not
needed: every op has a PyTorch reference implementation used for CPU tensors
and as the numerics oracle in tests.
"""
from __future__ import annotations

import importlib
import os

import torch

from ..utils.errors import NativeExtensionError

_MOD = None
_TRIED = False
_ERR: Exception | None = None


def _try_import():
    global _MOD, _TRIED, _ERR
    if _TRIED:
        return _MOD
    _TRIED = True
    try:
        _MOD = importlib.import_module("fluxmpi_amd._C")
    except Exception as e:  # ImportError, or undefined-symbol OSError
        _MOD = None
        _ERR = e
    return _MOD


def available() -> bool:
    return _try_import() is not None


def gpu_present() -> bool:
    try:
        return torch.cuda.is_available()
    except Exception:
        return False


def get(required: bool = True):
    """Return the ``_C`` module.

    ``required=True`` raises when it cannot be imported. Callers handling CPU
    tensors pass ``required=False`` and use the PyTorch path on ``None``.
    """
    mod = _try_import()
    if mod is None and required:
        if os.environ.get("FLUXMPI_ALLOW_FALLBACK", "0") == "1":
            return None
        raise NativeExtensionError(
            "fluxmpi_amd._C (the gfx950 HIP extension) is not built or failed to load: "
            f"{_ERR!r}. Run `python -c 'import fluxmpi_amd; fluxmpi_amd.build()'`."
        )
    return mod


def require_for(t: torch.Tensor):
    """The extension if ``t`` lives on the GPU (mandatory there), else ``None``."""
    if t.is_cuda:
        return get(required=True)
    return None
