"""Pytree walker (the Functors.jl ``fmap`` stand-in).

The reference walks parameter / gradient / optimiser-state containers with
``Functors.fmap`` (``src/synchronize.jl:12``, ``src/optimizer.jl:47,58,62``).
Two properties of ``fmap`` matter for correctness and are reproduced here:

1. the container is *rebuilt* with the same node types (dict, list, tuple,
   namedtuple, registered classes such as ``optimisers.Leaf``), and
2. identical (tied) array leaves are visited **once**; every occurrence in the
   output refers to the same result (Functors' ``IdDict`` cache).
   For collectives that means a tied weight is reduced once, not twice.

Non-container, non-array leaves (numbers, strings, ``None`` ...) are passed
to ``f`` as well; ``f`` decides what to do with them (``synchronize`` leaves
symbols untouched, broadcasts numbers, ...).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Callable, Iterable

import numpy as np
import torch

# type -> (flatten(x) -> (children, aux), unflatten(aux, children) -> x)
_REGISTRY: "OrderedDict[type, tuple[Callable, Callable]]" = OrderedDict()


def register_node(cls: type, flatten: Callable, unflatten: Callable) -> None:
    """Register ``cls`` as a container node (like ``Functors.@functor``)."""
    _REGISTRY[cls] = (flatten, unflatten)


def _is_namedtuple(x) -> bool:
    return isinstance(x, tuple) and hasattr(x, "_fields")


def node_def(x):
    """Return ``(flatten, unflatten)`` for a container node, or ``None`` for a leaf."""
    t = type(x)
    if t in _REGISTRY:
        return _REGISTRY[t]
    if isinstance(x, (torch.Tensor, np.ndarray, str, bytes)):
        return None
    if _is_namedtuple(x):
        return (lambda v: (list(v), type(v)), lambda aux, ch: aux(*ch))
    if isinstance(x, (list, tuple)):
        return (lambda v: (list(v), type(v)), lambda aux, ch: aux(ch))
    if isinstance(x, dict):
        def _flat(v):
            return list(v.values()), (type(v), list(v.keys()))

        def _unflat(aux, ch):
            typ, keys = aux
            try:
                return typ(zip(keys, ch))
            except TypeError:  # exotic mapping types
                return dict(zip(keys, ch))
        return (_flat, _unflat)
    for base, fns in _REGISTRY.items():
        if isinstance(x, base):
            return fns
    return None


def is_leaf(x) -> bool:
    return node_def(x) is None


def is_array(x) -> bool:
    return isinstance(x, (torch.Tensor, np.ndarray))


def is_numeric_array(x) -> bool:
    if isinstance(x, torch.Tensor):
        return True
    if isinstance(x, np.ndarray):
        return x.dtype.kind in "biufc"
    return False


def _cacheable(x) -> bool:
    # Functors caches non-isbits leaves only: arrays, not numbers.
    return is_array(x)


def fmap(f: Callable, x: Any, *ys: Any, cache: dict | None = None, exclude: Callable | None = None) -> Any:
    """Apply ``f`` to every leaf of ``x`` (and the matching leaves of ``ys``) and rebuild.

    ``exclude(node) -> True`` stops the recursion at ``node`` and hands it to ``f``
    (Functors' ``exclude`` keyword).
    """
    if cache is None:
        cache = {}
    keep_alive: list = []

    def walk(node, others):
        if (exclude is not None and exclude(node)) or node_def(node) is None:
            if _cacheable(node):
                key = id(node)
                if key in cache:
                    return cache[key]
                out = f(node, *others)
                cache[key] = out
                keep_alive.append(node)
                return out
            return f(node, *others)
        flat, unflat = node_def(node)
        children, aux = flat(node)
        other_children = []
        for o in others:
            if node_def(o) is None:
                # a leaf (typically ``None`` = "no gradient for this subtree") is
                # broadcast to every child, like Optimisers.jl's `nothing` grads.
                other_children.append([o] * len(children))
            else:
                oc, _ = node_def(o)[0](o)
                if len(oc) != len(children):
                    raise ValueError("fmap: trees have different structure")
                other_children.append(oc)
        new_children = [walk(c, [oc[i] for oc in other_children]) for i, c in enumerate(children)]
        return unflat(aux, new_children)

    return walk(x, list(ys))


def foreach(f: Callable, x: Any, *ys: Any, exclude: Callable | None = None) -> None:
    """Like :func:`fmap` but only for side effects (no rebuild)."""
    fmap(lambda *a: f(*a), x, *ys, exclude=exclude)


def leaves(x: Any, exclude: Callable | None = None, unique: bool = True) -> list:
    """Leaves of ``x`` in walk order (tied array leaves reported once when ``unique``)."""
    out: list = []
    seen: set = set()

    def walk(node):
        if (exclude is not None and exclude(node)) or node_def(node) is None:
            if unique and _cacheable(node):
                if id(node) in seen:
                    return
                seen.add(id(node))
            out.append(node)
            return
        children, _ = node_def(node)[0](node)
        for c in children:
            walk(c)

    walk(x)
    return out


def structure_signature(x: Any) -> str:
    """A rank-independent description of a tree (types, shapes, dtypes).

    Used to hash bucket plans across ranks so mismatched trees raise instead
    of deadlocking.
    """
    parts: list[str] = []

    def walk(node):
        nd = node_def(node)
        if nd is None:
            if isinstance(node, torch.Tensor):
                parts.append(f"T{tuple(node.shape)}{node.dtype}")
            elif isinstance(node, np.ndarray):
                parts.append(f"A{node.shape}{node.dtype}")
            elif isinstance(node, (bool, int, float, complex)):
                parts.append(type(node).__name__)
            else:
                parts.append("o")
            return
        children, aux = nd[0](node)
        parts.append(f"({type(node).__name__}:{len(children)}")
        for c in children:
            walk(c)
        parts.append(")")

    walk(x)
    return "".join(parts)


def tree_map_leaves(f: Callable, leaves_list: Iterable) -> list:
    return [f(l) for l in leaves_list]
