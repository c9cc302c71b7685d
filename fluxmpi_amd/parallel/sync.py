"""``synchronize``: broadcast parameters / states / optimiser trees from a root rank.

Reference: ``src/synchronize.jl:1-35`` (+ ``ext/FluxMPIFluxExt.jl``,
``ext/FluxMPIComponentArraysExt.jl``). Dispatch, case by case:

==========================================  ===========================================
input                                        behaviour
==========================================  ===========================================
dict / list / tuple / namedtuple container   walk (Functors.fmap), rebuild, sync leaves
empty container                              returned as is (``synchronize.jl:11``)
numeric tensor / numpy array                 broadcast in place (``synchronize.jl:15-17``)
``optimisers.Leaf``                          state synchronised (``synchronize.jl:24-27``)
Python number (int/float/bool/complex)       root's value returned (``synchronize.jl:29-31``)
``FlatParams`` (ComponentArray)              ONE broadcast of the flat buffer
``torch.nn.Module`` / ``FluxMPIFluxModel``   parameters + buffers broadcast in place
anything else (None, str, enum, ...)         returned unchanged, NOT synchronised
==========================================  ===========================================

Performance: instead of one blocking broadcast per leaf, every tensor leaf
is packed (HIP multi-tensor kernel) into per-(device, dtype) buckets, each
bucket is one RCCL broadcast, and non-root ranks unpack. All scalars of a
tree travel in one extra small message. Tied tensors are sent once.
"""
from __future__ import annotations

import numbers
from typing import Any

import numpy as np
import torch

from ..optimisers import Leaf
from ..utils.tree import fmap, is_numeric_array, node_def
from . import runtime
from .bucket import broadcast_tensors
from .flat import FlatParams


class FluxMPIFluxModel:
    """Marker wrapper for an arbitrary model object (reference ``src/FluxMPI.jl:84-86``).

    ``synchronize(FluxMPIFluxModel(m))`` synchronises every array inside ``m``
    and returns the *unwrapped* model (``ext/FluxMPIFluxExt.jl:6-8``).
    """

    def __init__(self, model: Any):
        self.model = model


def _is_num(x) -> bool:
    return isinstance(x, numbers.Number) and not isinstance(x, np.ndarray)


def _as_tensor(x):
    if isinstance(x, np.ndarray):
        if not (x.flags.c_contiguous and x.flags.writeable):
            raise ValueError("synchronize: numpy arrays must be C-contiguous and writeable")
        return torch.from_numpy(x)
    return x


def _sync_scalars(values: list, root: int) -> list:
    """Broadcast a list of Python numbers in one message per numeric kind."""
    if not values:
        return values
    comm = runtime.cpu_comm()
    out = list(values)
    ints = [i for i, v in enumerate(values) if isinstance(v, (bool, int, np.integer, np.bool_))]
    cplx = [i for i, v in enumerate(values) if isinstance(v, complex)]
    floats = [i for i in range(len(values)) if i not in set(ints) | set(cplx)]
    if ints:
        t = torch.tensor([int(values[i]) for i in ints], dtype=torch.int64)
        comm.broadcast(t, root)
        for k, i in enumerate(ints):
            v = int(t[k])
            out[i] = bool(v) if isinstance(values[i], (bool, np.bool_)) else type(values[i])(v)
    if floats:
        t = torch.tensor([float(values[i]) for i in floats], dtype=torch.float64)
        comm.broadcast(t, root)
        for k, i in enumerate(floats):
            out[i] = type(values[i])(float(t[k]))
    if cplx:
        t = torch.tensor([[values[i].real, values[i].imag] for i in cplx], dtype=torch.float64)
        comm.broadcast(t, root)
        for k, i in enumerate(cplx):
            out[i] = complex(float(t[k, 0]), float(t[k, 1]))
    return out


def _sync_module(m: torch.nn.Module, root: int) -> torch.nn.Module:
    from .ddp import engine_for

    eng = engine_for(m)
    if eng is not None and eng.communicate:
        # a module under a DDP engine: its flat buckets AND fp32 masters are broadcast, so
        # masters stay bit-identical across ranks (a parameter-only broadcast would leave the
        # root with m_root and the others with bf16(m_root))
        eng.broadcast_parameters(root)
        return m
    ts, seen = [], set()
    for t in list(m.parameters()) + list(m.buffers()):
        if id(t) not in seen and t.numel() > 0:
            seen.add(id(t))
            # detach() (not .data) shares the version counter, so the write is visible to
            # the DDP engine's stale-master check
            ts.append(t.detach())
    _broadcast_any(ts, root)
    return m


def _broadcast_any(tensors: list, root: int) -> None:
    if not tensors:
        return
    with torch.no_grad():
        broadcast_tensors(tensors, root)


def synchronize(x: Any, root_rank: int = 0) -> Any:
    """Synchronise ``x`` across all ranks from ``root_rank``; use the return value."""
    runtime._require()
    if isinstance(x, FluxMPIFluxModel):
        m = x.model
        if isinstance(m, torch.nn.Module):
            return _sync_module(m, root_rank)
        return synchronize(m, root_rank)
    if isinstance(x, torch.nn.Module):
        return _sync_module(x, root_rank)
    if isinstance(x, FlatParams):
        _broadcast_any([x.data], root_rank)
        return FlatParams(data=x.data, axes=x.axes)
    if isinstance(x, torch.Tensor):
        if x.numel():
            _broadcast_any([x], root_rank)
        return x
    if isinstance(x, np.ndarray):
        if x.dtype == object:  # array of containers: synchronize elementwise (synchronize.jl:19-22)
            out = np.empty_like(x)
            for i, v in np.ndenumerate(x):
                out[i] = synchronize(v, root_rank)
            return out
        if x.size:
            _broadcast_any([_as_tensor(x)], root_rank)
        return x
    if _is_num(x):
        return _sync_scalars([x], root_rank)[0]
    if isinstance(x, Leaf):
        return Leaf(x.rule, synchronize(x.state, root_rank), x.frozen)
    nd = node_def(x)
    if nd is None:
        return x  # symbols, None, strings, ...: not synchronised (synchronize.jl:33-35)
    children, _ = nd[0](x)
    if len(children) == 0:
        return x
    return _sync_tree(x, root_rank)


def _sync_tree(x: Any, root: int) -> Any:
    tensors: list = []
    scalars: list = []
    seen: set = set()

    def collect(leaf):
        if isinstance(leaf, torch.Tensor) or (isinstance(leaf, np.ndarray) and is_numeric_array(leaf)):
            if id(leaf) not in seen:
                seen.add(id(leaf))
                t = _as_tensor(leaf)
                if t.numel():
                    tensors.append(t)
        elif isinstance(leaf, torch.nn.Module):
            for t in list(leaf.parameters()) + list(leaf.buffers()):
                if id(t) not in seen:
                    seen.add(id(t))
                    tensors.append(t.detach())
        elif isinstance(leaf, FlatParams):
            if id(leaf.data) not in seen:
                seen.add(id(leaf.data))
                tensors.append(leaf.data)
        elif _is_num(leaf):
            scalars.append(leaf)
        return leaf

    exclude = lambda n: isinstance(n, (torch.nn.Module, FlatParams))  # noqa: E731
    fmap(collect, x, exclude=exclude)
    _broadcast_any(tensors, root)
    synced = iter(_sync_scalars(scalars, root))

    def rebuild(leaf):
        if _is_num(leaf):
            return next(synced)
        if isinstance(leaf, np.ndarray) and leaf.dtype == object:
            return synchronize(leaf, root)
        if isinstance(leaf, FlatParams):
            return FlatParams(data=leaf.data, axes=leaf.axes)
        return leaf

    # Same walk order as `collect` (fmap caches arrays, never scalars), so the
    # scalar iterator lines up.
    return fmap(rebuild, x, exclude=exclude)


synchronize_ = synchronize
