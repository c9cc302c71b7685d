"""``DistributedOptimizer`` and ``allreduce_gradients`` (reference ``src/optimizer.jl``).

Semantics kept from the reference:

* gradients are **summed** across ranks, not averaged (``src/optimizer.jl:11-14``,
  changelog v0.5.0): scale the loss by ``1/total_workers()`` to average, or
  pass ``average=True`` (extension);
* ``init`` delegates, so the state tree of ``DistributedOptimizer(rule)`` is
  identical to ``rule``'s (``test/test_optimizer.jl:13-14``);
* ``allreduce_gradients`` returns the reduced gradient tree; non-array leaves
  pass through.

Irregular gradient trees: in the reference a rank whose gradient
for some leaf is ``nothing`` skips that leaf's ``MPI_Allreduce`` while the
others issue it, and the job hangs. Here the reduction plan comes from the
*state* tree: ``Optimisers.update_`` zero-fills a missing gradient for a
``collective`` rule, so every rank reduces the same leaves in the same order.
Before each bucketed reduction the plan's structure hash is compared across
ranks (one tiny host allreduce, ``FLUXMPI_CHECK_PLANS``), so a tree that
really differs raises :class:`CollectiveMismatchError` instead of deadlocking.

What changed (the MI355X design): the reference performs one blocking,
host-staged ``MPI_Allreduce`` per leaf inside ``apply!``. Here
:meth:`DistributedOptimizer.apply_batch` receives *all* leaves of an update
at once, reduces them with a handful of bucketed RCCL allreduces (packed by
the HIP multi-tensor kernel), then hands the whole batch to the wrapped
rule's fused kernel (multi-tensor Adam etc.). Gradients are reduced in place.
"""
from __future__ import annotations

from typing import Any

import numpy as np
import torch

from ..optimisers import AbstractRule
from ..utils.config import get_config
from ..utils.debug import check_same_structure, structure_hash
from ..utils.errors import CollectiveMismatchError
from ..utils.tree import fmap, node_def, structure_signature
from . import runtime
from .bucket import allreduce_tensors
from .comm import ReduceOp

_CHECKED: set = set()
# structure hash of a `like` tree -> signature of the zero-filled gradient tree checked across ranks
_LIKE_CHECKED: dict = {}
# the same key -> leaf dtypes of that checked tree (what a zero-filled leaf is created as)
_LIKE_DTYPES: dict = {}


def check_plan(obj, what: str, derived: bool = False) -> None:
    """Cross-rank structure check of a reduction plan (``FLUXMPI_CHECK_PLANS``).

    ``always`` (default): every call, one 16-byte host allreduce — every rank
    checks, so a rank can never sit in the check while another is already in the
    gradient collective. ``first``: once per distinct plan on this rank (cheaper;
    only safe when trees can differ from the first step on). ``never``: off. Set with
    ``FLUXMPI_CHECK_PLANS`` or the ``check_plans`` preference (the environment wins, as for
    every other knob); measured cost of ``always``: one gloo allreduce of 16 bytes per call
    (``scripts/bench_check_plan.py``).

    ``derived``: the plan is a function of an argument that is identical on every rank (the
    parameter tree of ``allreduce_gradients(like=...)``: missing gradients are zero-filled, so
    the structure cannot vary between steps on one rank and not another) — ``always`` then
    checks once per distinct plan, as ``first`` does.
    """
    mode = get_config().check_plans
    if mode == "never" or not runtime.Initialized() or runtime.total_workers() == 1:
        return
    if mode == "first" or derived:
        h = structure_hash(obj)
        if h in _CHECKED:
            return
        check_same_structure(obj, what=what)
        _CHECKED.add(h)
        return
    check_same_structure(obj, what=what)


class DistributedOptimizer(AbstractRule):
    """Wrap an Optimisers-style rule; gradients are allreduce-SUMmed before it runs."""

    collective = True

    def __init__(self, optimizer: AbstractRule, average: bool = False):
        self.optimizer = optimizer
        self.average = average

    def init(self, x):
        return self.optimizer.init(x)

    def _reduce(self, grads: list) -> None:
        grads = [g for g in grads if g is not None]
        check_plan(grads, "DistributedOptimizer gradient batch")
        if not grads:
            return
        op = ReduceOp.AVG if self.average else ReduceOp.SUM
        with torch.no_grad():
            allreduce_tensors(grads, op)

    def apply(self, state, x, dx):
        """Per-leaf form (reference ``src/optimizer.jl:20-23``)."""
        self._reduce([dx])
        return self.optimizer.apply(state, x, dx)

    def apply_batch(self, items: list) -> list:
        """Bucketed reduction of every gradient, then the wrapped rule's fused batch step."""
        self._reduce([dx for _, _, dx in items])
        return self.optimizer.apply_batch(items)

    def __repr__(self):
        return f"DistributedOptimizer({self.optimizer!r})"


def _zero_fill(gs: Any, like: Any, dtypes: list | None = None, record: list | None = None) -> Any:
    """``gs`` with every missing (``None``) gradient replaced by zeros shaped like ``like``.

    ``record`` receives the dtype of every array leaf of the result (traversal order);
    ``dtypes`` (such a record from the call whose plan was checked across ranks) gives a
    zero-filled leaf that recorded dtype instead of its parameter's, so a gradient that arrives
    in another dtype than its parameter (fp32 grads of bf16 params) and later goes missing on
    every rank keeps the checked signature."""
    pos = [0]

    def leaf(g, p):
        i = pos[0]
        pos[0] += 1
        if g is None:
            dt = dtypes[i] if dtypes is not None and i < len(dtypes) else None
            if isinstance(p, torch.Tensor):
                g = torch.zeros_like(p, dtype=dt if isinstance(dt, torch.dtype) else None)
            elif isinstance(p, np.ndarray):
                g = np.zeros_like(p, dtype=dt if isinstance(dt, np.dtype) else None)
        if record is not None:
            record.append(g.dtype if isinstance(g, (torch.Tensor, np.ndarray)) else None)
        return g

    def walk(g, p):
        if isinstance(p, (torch.Tensor, np.ndarray)):
            return leaf(g, p)
        if isinstance(p, torch.nn.Module):
            named = dict(p.named_parameters())
            gd = g if isinstance(g, dict) else {n: q.grad for n, q in named.items()}
            return {n: walk(gd.get(n), q) for n, q in named.items()}
        nd = node_def(p)
        if nd is None:
            return g
        lc, aux = nd[0](p)
        gc = [None] * len(lc) if g is None else nd[0](g)[0]
        if len(gc) != len(lc):
            raise ValueError("allreduce_gradients: gradient tree and `like` tree differ in structure")
        return nd[1](aux, [walk(a, c) for a, c in zip(gc, lc)])

    return walk(gs, like)


def _check_like_plan(gs: Any, like: Any, key=None) -> None:
    """Plan check for ``allreduce_gradients(like=...)``.

    The gate is the structure hash of ``like`` (the parameter tree: identical on every rank
    after ``synchronize``), so every rank takes the same branch. The first call for a given
    ``like`` structure compares the zero-filled gradient tree (shapes and dtypes included)
    across ranks; later calls compare it LOCALLY against the signature that was checked, so a
    gradient whose shape or dtype changed on one rank raises instead of entering a mismatched
    collective. Zero-filled leaves take the dtypes of the checked plan (:func:`_zero_fill`), so
    a gradient missing on every rank never changes the signature by itself. The table is keyed
    by structure, so it stays bounded however often callers build fresh ``like`` trees.
    """
    if not _plan_checks_on():
        return
    key = structure_hash(like) if key is None else key
    sig = structure_signature(gs)
    seen = _LIKE_CHECKED.get(key)
    if seen is None:
        check_same_structure(gs, what="gradient tree")
        _LIKE_CHECKED[key] = sig
    elif seen != sig:
        raise CollectiveMismatchError(
            "allreduce_gradients(like=...): a gradient's shape or dtype differs from the plan "
            "checked across ranks for this parameter tree; the collectives would mismatch")


def _plan_checks_on() -> bool:
    return get_config().check_plans != "never" and runtime.Initialized() and runtime.total_workers() > 1


def allreduce_gradients(gs: Any, on_gpu: bool | None = None, op=ReduceOp.SUM, like: Any = None) -> Any:
    """Allreduce (SUM) every array leaf of the gradient tree ``gs``; returns the tree.

    ``on_gpu`` is accepted for API parity with the reference (which staged
    GPU gradients through the host when set). Collectives here are always
    device-direct, so it only serves as an assertion when given explicitly.

    ``like`` (the parameter tree, or the module) makes the reduction plan come from
    the parameters: a ``None`` gradient is zero-filled, so a rank missing one still
    joins every collective. Without it, the gradient tree's structure
    (``None`` positions included) is checked across ranks and a mismatch raises
    :class:`CollectiveMismatchError` instead of hanging.
    """
    runtime._require()
    if like is not None:
        key = structure_hash(like) if _plan_checks_on() else None
        rec: list = []
        gs = _zero_fill(gs, like, dtypes=_LIKE_DTYPES.get(key), record=rec)
        if key is not None:
            _check_like_plan(gs, like, key)
            _LIKE_DTYPES.setdefault(key, rec)
    else:
        check_plan(gs, "gradient tree")
    leaves: list = []
    seen: set = set()

    def collect(g):
        if isinstance(g, torch.Tensor):
            if id(g) not in seen:
                seen.add(id(g))
                leaves.append(g)
        elif isinstance(g, np.ndarray) and g.dtype.kind in "biufc":
            if id(g) not in seen:
                seen.add(id(g))
                leaves.append(torch.from_numpy(g))
        return g

    fmap(collect, gs)
    if on_gpu is True and leaves and not any(t.is_cuda for t in leaves):
        raise ValueError("allreduce_gradients(on_gpu=True) but no gradient lives on a GPU")
    with torch.no_grad():
        allreduce_tensors(leaves, op)
    return fmap(lambda g: g, gs)
