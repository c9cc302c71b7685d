"""``FlatParams``: a contiguous parameter vector with named, nested views.

The ComponentArrays.jl stand-in (reference ``ext/FluxMPIComponentArraysExt.jl``):
the whole parameter tree lives in ONE flat buffer, so ``synchronize`` is a
single broadcast (``bcast!(getdata(x))`` in the reference) and the flat
buffer can be fed directly to fused optimiser kernels.

    fp = FlatParams({"a": {"b": t1, "c": t2}, "d": t3})
    fp.a.b          # view into fp.data
    fp["d"]         # same as fp.d
    fp.to_tree()    # {"a": {"b": view, "c": view}, "d": view}
"""
from __future__ import annotations

from typing import Any

import torch

from ..ops import multi_tensor as mt
from ..utils.tree import node_def


class _Axis:
    __slots__ = ("offset", "shape", "numel")

    def __init__(self, offset: int, shape: tuple):
        self.offset = offset
        self.shape = tuple(shape)
        n = 1
        for s in shape:
            n *= s
        self.numel = n

    def __repr__(self):
        return f"Axis({self.offset}, {self.shape})"


class FlatParams:
    """Contiguous parameter vector + nested axes (``ComponentArray`` analogue)."""

    def __init__(self, tree: Any = None, *, data: torch.Tensor | None = None, axes: Any = None,
                 dtype: torch.dtype | None = None, device: torch.device | str | None = None, align: bool = False):
        if data is not None:
            self.__dict__["data"] = data
            self.__dict__["axes"] = axes
            return
        leaves: list = []

        def shape_tree(x):
            if isinstance(x, torch.Tensor):
                leaves.append(x)
                return len(leaves) - 1
            nd = node_def(x)
            if nd is None:
                raise TypeError(f"FlatParams: unsupported leaf {type(x)}")
            ch, aux = nd[0](x)
            return ("node", nd, aux, [shape_tree(c) for c in ch])

        skel = shape_tree(tree)
        if not leaves:
            raise ValueError("FlatParams needs at least one tensor")
        dt = dtype or leaves[0].dtype
        dev = torch.device(device) if device is not None else leaves[0].device
        numels = [t.numel() for t in leaves]
        if align:
            offs, total = mt.aligned_offsets(numels, dt)
        else:
            offs, total = [], 0
            for n in numels:
                offs.append(total)
                total += n
        buf = torch.zeros(total, dtype=dt, device=dev)
        for t, o in zip(leaves, offs):
            buf[o:o + t.numel()].copy_(t.detach().reshape(-1))

        def axes_of(s):
            if isinstance(s, int):
                return _Axis(offs[s], leaves[s].shape)
            _, nd, aux, ch = s
            return ("node", nd, aux, [axes_of(c) for c in ch])

        self.__dict__["data"] = buf
        self.__dict__["axes"] = axes_of(skel)

    # --- access ------------------------------------------------------------
    def _view(self, ax):
        if isinstance(ax, _Axis):
            return self.data[ax.offset:ax.offset + ax.numel].view(ax.shape)
        return FlatParams(data=self.data, axes=ax)

    def _child(self, key):
        ax = self.axes
        if isinstance(ax, _Axis):
            raise KeyError(key)
        _, nd, aux, ch = ax
        # dict: aux = (type, keys); namedtuple/list/tuple: aux = type
        if isinstance(aux, tuple) and len(aux) == 2 and isinstance(aux[1], list):
            keys = aux[1]
            if key in keys:
                return self._view(ch[keys.index(key)])
            raise KeyError(key)
        if isinstance(aux, type) and hasattr(aux, "_fields") and isinstance(key, str):
            return self._view(ch[aux._fields.index(key)])
        if isinstance(key, int):
            return self._view(ch[key])
        raise KeyError(key)

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        try:
            return self._child(name)
        except (KeyError, ValueError):
            raise AttributeError(name) from None

    def __getitem__(self, key):
        return self._child(key)

    def __len__(self):
        return self.data.numel()

    def to_tree(self):
        def build(ax):
            if isinstance(ax, _Axis):
                return self.data[ax.offset:ax.offset + ax.numel].view(ax.shape)
            _, nd, aux, ch = ax
            return nd[1](aux, [build(c) for c in ch])
        return build(self.axes)

    def like(self, data: torch.Tensor) -> "FlatParams":
        """Same axes over another flat buffer (e.g. gradients, optimiser moments)."""
        if data.numel() != self.data.numel():
            raise ValueError("like(): size mismatch")
        return FlatParams(data=data, axes=self.axes)

    def __repr__(self):
        return f"FlatParams(numel={self.data.numel()}, dtype={self.data.dtype}, device={self.data.device})"


def getdata(x: FlatParams) -> torch.Tensor:
    return x.data


def getaxes(x: FlatParams):
    return x.axes
