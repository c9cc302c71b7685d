"""Optimisers.jl-shaped optimiser API on PyTorch tensors.

The reference wraps Optimisers.jl rules (``src/optimizer.jl:16-25``) and its
tests compare state trees leaf by leaf (``test/test_optimizer.jl:13-14``), so
the *state layout* must match Optimisers.jl:

=============  ==============================================  =======================
rule           per-leaf state                                   update ``dx'``
=============  ==============================================  =======================
Descent(η)     ``None``                                         ``η·dx``
Momentum(η,ρ)  ``vel`` (zeros like x)                           ``vel = ρ·vel + η·dx``
Nesterov(η,ρ)  ``vel``                                          ``-ρ²·vel + (1+ρ)·η·dx``
RMSProp(η,ρ,ϵ) ``acc``                                          ``dx·η / (sqrt(acc)+ϵ)``
Adam(η,β,ϵ)    ``(mt, vt, (β1ᵗ, β2ᵗ))``, βᵗ starts at β         ``mt/(1-β1ᵗ)/(sqrt(vt/(1-β2ᵗ))+ϵ)·η``
AdamW(η,β,γ,ϵ) ``OptimiserChain(Adam, WeightDecay(γ))``         Adam's dx' + γ·x
WeightDecay(γ) ``None``                                         ``dx + γ·x``
ClipGrad(δ)    ``None``                                         ``clamp(dx, -δ, δ)``
ClipNorm(ω,p)  ``None``                                         ``dx · min(1, ω/‖dx‖ₚ)``
=============  ==============================================  =======================

``setup(rule, model)`` builds a tree of :class:`Leaf` mirroring the model
tree (tied arrays share one Leaf); ``update(state, model, grads)`` is
out-of-place (copies state and model first, like Optimisers.jl) and
``update_`` (Julia's ``update!``) mutates in place. Leaves are *batched*:
``update_`` collects every (leaf, x, dx) first and hands whole batches to
rules that implement ``apply_batch`` — that is where the fused multi-tensor
HIP kernels run on GPU and where :class:`DistributedOptimizer` performs one
bucketed allreduce for all gradients instead of one collective per leaf.
"""
from __future__ import annotations

import copy
import dataclasses
from typing import Any

import numpy as np
import torch

from ..ops import optim as _fused
from ..utils.tree import fmap, is_numeric_array, node_def, register_node


class AbstractRule:
    """Base class of optimisation rules (``Optimisers.AbstractRule``)."""

    def init(self, x: torch.Tensor) -> Any:
        return None

    def apply(self, state, x: torch.Tensor, dx: torch.Tensor):
        """Return ``(new_state, dx')``; ``x -= dx'`` is applied by the caller."""
        raise NotImplementedError

    #: True for rules that issue collectives (``DistributedOptimizer``): every rank must then
    #: hand them the same leaves, so a missing gradient is zero-filled instead of skipped.
    collective = False

    def apply_batch(self, items: list) -> list:
        """``items``: list of ``(leaf, x, dx)``. Returns the ``dx'`` list; updates ``leaf.state``.

        Default: per-leaf :meth:`apply`. Rules override this to fuse.
        Returning ``None`` in place of ``dx'`` means "x already updated in place".
        """
        out = []
        for leaf, x, dx in items:
            leaf.state, d = self.apply(leaf.state, x, dx)
            out.append(d)
        return out

    def __repr__(self):
        fields = ", ".join(f"{k}={v!r}" for k, v in vars(self).items())
        return f"{type(self).__name__}({fields})"


@dataclasses.dataclass(eq=False)
class Leaf:
    """Optimiser state of one array (``Optimisers.Leaf``)."""

    rule: AbstractRule
    state: Any
    frozen: bool = False

    def __repr__(self):
        return f"Leaf({self.rule!r}, {_short(self.state)})"


def _short(s):
    if isinstance(s, torch.Tensor):
        return f"tensor{tuple(s.shape)}"
    if isinstance(s, tuple):
        return "(" + ", ".join(_short(x) for x in s) + ")"
    return repr(s)


# Functors: Leaf's children is its state only (the rule holds hyperparameters).
register_node(Leaf, lambda l: ([l.state], (l.rule, l.frozen)), lambda aux, ch: Leaf(aux[0], ch[0], aux[1]))


def _as_tensor(x):
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    return x


_T_CACHE: dict = {}


def _T(x: torch.Tensor, v: float) -> float:
    """Julia's ``T(η)`` cast (Optimisers.jl rules convert η, β, ϵ to ``eltype(x)``): round a
    hyperparameter to the array's precision — fp32, and for bf16 / fp16 arrays bf16 / fp16
    (``BFloat16(0.9) == 0.8984375``; ``Float16(1e-8) == 0``), exactly as the Julia rule does.
    fp64 (and non-float) arrays keep the double."""
    dt = x.dtype
    if dt not in (torch.float32, torch.bfloat16, torch.float16):
        return float(v)
    key = (dt, v)
    r = _T_CACHE.get(key)
    if r is None:
        r = float(np.float32(v)) if dt == torch.float32 else float(torch.tensor(float(v), dtype=dt))
        if len(_T_CACHE) < 4096:
            _T_CACHE[key] = r
    return r


def _eps(x: torch.Tensor, e: float) -> float:
    """Optimisers.jl's ``_eps(T, ϵ)``: ``T(ϵ)``, except that a Float16 ϵ is floored at
    ``Float16(1e-7)`` (a nonzero ϵ must not round to 0: ``Float16(1e-8) == 0`` would give
    ``0 / (sqrt(0) + 0) = NaN`` on every element whose gradient has been zero so far)."""
    if x.dtype == torch.float16:
        return 0.0 if e == 0 else max(_T(x, 1e-7), _T(x, e))
    return _T(x, e)


# ------------------------------------------------------------------ rules
class Descent(AbstractRule):
    def __init__(self, eta: float = 0.1):
        self.eta = eta

    def apply(self, state, x, dx):
        return state, dx * _T(x, self.eta)

    def apply_batch(self, items):
        return _sgd_batch(self, items, 0.0, False)


class Momentum(AbstractRule):
    def __init__(self, eta: float = 0.01, rho: float = 0.9):
        self.eta, self.rho = eta, rho

    def init(self, x):
        return torch.zeros_like(x)

    def apply(self, vel, x, dx):
        eta, rho = _T(x, self.eta), _T(x, self.rho)
        vel.mul_(rho).add_(dx, alpha=eta)
        return vel, vel

    def apply_batch(self, items):
        return _sgd_batch(self, items, self.rho, False)


class Nesterov(AbstractRule):
    def __init__(self, eta: float = 0.001, rho: float = 0.9):
        self.eta, self.rho = eta, rho

    def init(self, x):
        return torch.zeros_like(x)

    def apply(self, vel, x, dx):
        eta, rho = _T(x, self.eta), _T(x, self.rho)
        newdx = -(rho ** 2) * vel + (1 + rho) * eta * dx
        vel.mul_(rho).sub_(dx, alpha=eta)
        return vel, newdx

    def apply_batch(self, items):
        return _sgd_batch(self, items, self.rho, True)


def _sgd_batch(rule, items, rho, nesterov):
    """Fused GPU path for Descent / Momentum / Nesterov; per-leaf math elsewhere."""
    gpu = [i for i, (l, x, dx) in enumerate(items)
           if x.is_cuda and dx is not None
           and _same_dense(x, dx, *([l.state] if rho != 0.0 and isinstance(l.state, torch.Tensor) else []))
           and _fused.supported(x.dtype, dx.dtype, x.dtype, False)]
    out: list = [None] * len(items)
    gset = set(gpu)
    for i, (leaf, x, dx) in enumerate(items):
        if i not in gset:
            leaf.state, out[i] = rule.apply(leaf.state, x, dx)
    if gpu:
        by_dtype: dict = {}
        for i in gpu:
            by_dtype.setdefault(items[i][1].dtype, []).append(i)
        for idx in by_dtype.values():
            x0 = items[idx[0]][1]
            xs = [items[i][1] for i in idx]
            gs = [items[i][2] for i in idx]
            bufs = [items[i][0].state for i in idx] if rho != 0.0 else None
            # hyperparameters rounded to the leaves' precision, as in Julia (``_T``)
            _fused.sgd_(xs, gs, bufs, lr=_T(x0, rule.eta), momentum=_T(x0, rho) if rho else 0.0,
                        nesterov=nesterov)
    return out


class RMSProp(AbstractRule):
    def __init__(self, eta: float = 0.001, rho: float = 0.9, epsilon: float = 1e-8):
        self.eta, self.rho, self.epsilon = eta, rho, epsilon

    def init(self, x):
        return torch.zeros_like(x)

    def apply(self, acc, x, dx):
        eta, rho, eps = _T(x, self.eta), _T(x, self.rho), _eps(x, self.epsilon)
        acc.mul_(rho).addcmul_(dx, dx, value=1 - rho)
        return acc, dx * eta / (torch.sqrt(acc) + eps)


class AdaGrad(AbstractRule):
    def __init__(self, eta: float = 0.1, epsilon: float = 1e-8):
        self.eta, self.epsilon = eta, epsilon

    def init(self, x):
        return torch.full_like(x, self.epsilon)

    def apply(self, acc, x, dx):
        acc.addcmul_(dx, dx)
        return acc, dx * _T(x, self.eta) / (torch.sqrt(acc) + _eps(x, self.epsilon))


class Adam(AbstractRule):
    """``Adam(η=0.001, β=(0.9, 0.999), ϵ=1e-8)``; state ``(mt, vt, βt)``."""

    def __init__(self, eta: float = 0.001, beta: tuple = (0.9, 0.999), epsilon: float = 1e-8):
        self.eta, self.beta, self.epsilon = eta, tuple(beta), epsilon
        self.weight_decay = 0.0  # set by AdamW's fused path only

    def init(self, x):
        return (torch.zeros_like(x), torch.zeros_like(x), (_T(x, self.beta[0]), _T(x, self.beta[1])))

    def apply(self, state, x, dx):
        eta, b1, b2, eps = _T(x, self.eta), _T(x, self.beta[0]), _T(x, self.beta[1]), _eps(x, self.epsilon)
        mt, vt, bt = state
        mt.mul_(b1).add_(dx, alpha=1 - b1)
        vt.mul_(b2).addcmul_(dx, dx, value=1 - b2)
        dxp = mt / (1 - bt[0]) / (torch.sqrt(vt / (1 - bt[1])) + eps) * eta
        return (mt, vt, (_T(x, bt[0] * b1), _T(x, bt[1] * b2))), dxp

    def apply_batch(self, items):
        return _adam_batch(self, items, 0.0)


def _same_dense(*ts) -> bool:
    """All tensors dense (no gaps or overlaps) with identical shape and strides: the flat
    multi-tensor kernels then see matching elements at matching offsets (contiguous, or e.g.
    a channels_last filter with its channels_last gradient and zeros_like moments)."""
    from ..ops.graddst import _dense
    t0 = ts[0]
    if not (t0.is_contiguous() or _dense(t0)):
        return False
    return all(t.shape == t0.shape and t.stride() == t0.stride() for t in ts[1:])


def _adam_batch(rule: Adam, items, weight_decay: float):
    """Fused multi-tensor Adam on GPU leaves (x updated in place, dx' = None)."""
    out: list = [None] * len(items)
    fused: dict = {}
    host: dict = {}
    for i, (leaf, x, dx) in enumerate(items):
        ok = (x.is_cuda and dx is not None and isinstance(leaf.state, tuple) and len(leaf.state) == 3
              and _same_dense(x, dx, leaf.state[0], leaf.state[1])
              and _fused.supported(x.dtype, dx.dtype, leaf.state[0].dtype, False))
        if ok:
            key = (x.device, x.dtype, tuple(leaf.state[2]))  # same precision and beta^t -> one launch
            fused.setdefault(key, []).append(i)
        elif (not x.is_cuda and dx is not None and x.dtype in (torch.float32, torch.float64)
              and dx.dtype == x.dtype and isinstance(leaf.state, tuple) and len(leaf.state) == 3
              and leaf.state[0].dtype == x.dtype and x.shape == dx.shape):
            host.setdefault((x.dtype, tuple(leaf.state[2])), []).append(i)
        else:
            st, d = Adam.apply(rule, leaf.state, x, dx)
            if weight_decay:
                d = d + _T(x, weight_decay) * x
            leaf.state, out[i] = st, d
    for (dt, bt), idx in host.items():
        # CPU leaves: the same formulas as Adam.apply, term by term, as multi-tensor (foreach)
        # ops — one dispatch per term for the whole batch instead of ~10 per leaf
        x0 = items[idx[0]][1]
        eta, b1, b2, eps = _T(x0, rule.eta), _T(x0, rule.beta[0]), _T(x0, rule.beta[1]), _eps(x0, rule.epsilon)
        xs = [items[i][1] for i in idx]
        gs = [items[i][2] for i in idx]
        ms = [items[i][0].state[0] for i in idx]
        vs = [items[i][0].state[1] for i in idx]
        torch._foreach_mul_(ms, b1)
        torch._foreach_add_(ms, gs, alpha=1 - b1)
        torch._foreach_mul_(vs, b2)
        torch._foreach_addcmul_(vs, gs, gs, value=1 - b2)
        num = torch._foreach_div(ms, 1 - bt[0])
        den = torch._foreach_div(vs, 1 - bt[1])
        torch._foreach_sqrt_(den)
        torch._foreach_add_(den, eps)
        torch._foreach_div_(num, den)
        torch._foreach_mul_(num, eta)
        if weight_decay:
            torch._foreach_add_(num, xs, alpha=_T(x0, weight_decay))
        for k, i in enumerate(idx):
            leaf = items[i][0]
            m, v, b = leaf.state
            leaf.state = (m, v, (_T(x0, b[0] * b1), _T(x0, b[1] * b2)))
            out[i] = num[k]
    for (_, _, bt), idx in fused.items():
        x0 = items[idx[0]][1]
        xs = [items[i][1] for i in idx]
        gs = [items[i][2] for i in idx]
        ms = [items[i][0].state[0] for i in idx]
        vs = [items[i][0].state[1] for i in idx]
        # hyperparameters rounded to the leaves' precision, as in Julia (``_T``)
        _fused.adam_(xs, gs, ms, vs, lr=_T(x0, rule.eta), beta1=_T(x0, rule.beta[0]), beta2=_T(x0, rule.beta[1]),
                     eps=_eps(x0, rule.epsilon), bc1=1.0 - bt[0], bc2=1.0 - bt[1],
                     weight_decay=_T(x0, weight_decay) if weight_decay else 0.0)
        for i in idx:
            leaf, x = items[i][0], items[i][1]
            m, v, b = leaf.state
            leaf.state = (m, v, (_T(x, b[0] * _T(x, rule.beta[0])), _T(x, b[1] * _T(x, rule.beta[1]))))
            out[i] = None
    return out


class WeightDecay(AbstractRule):
    def __init__(self, gamma: float = 5e-4):
        self.gamma = gamma

    def apply(self, state, x, dx):
        return state, dx + _T(x, self.gamma) * x


class ClipGrad(AbstractRule):
    def __init__(self, delta: float = 10.0):
        self.delta = delta

    def apply(self, state, x, dx):
        d = _T(x, self.delta)
        return state, torch.clamp(dx, -d, d)


class ClipNorm(AbstractRule):
    def __init__(self, omega: float = 10.0, p: float = 2.0):
        self.omega, self.p = omega, p

    def apply(self, state, x, dx):
        nrm = torch.linalg.vector_norm(dx.float() if dx.dtype in (torch.bfloat16, torch.float16) else dx, self.p)
        scale = torch.clamp(self.omega / nrm, max=1.0).to(dx.dtype)
        return state, dx * scale


class OptimiserChain(AbstractRule):
    """Apply rules in sequence; state is the tuple of member states."""

    def __init__(self, *opts: AbstractRule):
        self.opts = tuple(opts)

    @property
    def collective(self) -> bool:
        return any(getattr(o, "collective", False) for o in self.opts)

    def init(self, x):
        return tuple(o.init(x) for o in self.opts)

    def apply(self, states, x, dx):
        new = []
        for o, s in zip(self.opts, states):
            s, dx = o.apply(s, x, dx)
            new.append(s)
        return tuple(new), dx

    def apply_batch(self, items):
        # Fuse the common AdamW shape (Adam then WeightDecay) into one kernel.
        if (len(self.opts) == 2 and isinstance(self.opts[0], Adam) and isinstance(self.opts[1], WeightDecay)):
            adam, wd = self.opts
            sub = []
            for leaf, x, dx in items:
                sub.append((Leaf(adam, leaf.state[0]), x, dx))
            out = _adam_batch(adam, sub, wd.gamma)
            for (leaf, _, _), (sl, _, _) in zip(items, sub):
                leaf.state = (sl.state, leaf.state[1])
            return out
        return AbstractRule.apply_batch(self, items)


OptimizerChain = OptimiserChain


def AdamW(eta: float = 0.001, beta: tuple = (0.9, 0.999), decay: float = 0.0, epsilon: float = 1e-8):
    """Optimisers.jl ``AdamW`` = ``OptimiserChain(Adam(η, β, ϵ), WeightDecay(γ))``."""
    return OptimiserChain(Adam(eta, beta, epsilon), WeightDecay(decay))


# ------------------------------------------------------------------ tree API
def setup(rule: AbstractRule, model: Any) -> Any:
    """Build the state tree (``Optimisers.setup``). Tied arrays share one :class:`Leaf`."""
    cache: dict = {}
    keep: list = []

    def walk(x):
        if is_numeric_array(x) and (not isinstance(x, torch.Tensor) or x.is_floating_point()):
            key = id(x)
            if key in cache:
                return cache[key]
            leaf = Leaf(rule, rule.init(_as_tensor(x)))
            cache[key] = leaf
            keep.append(x)
            return leaf
        if isinstance(x, torch.nn.Module):
            return {n: walk(p) for n, p in x.named_parameters()}
        nd = node_def(x)
        if nd is None:
            return None
        ch, aux = nd[0](x)
        return nd[1](aux, [walk(c) for c in ch])

    return walk(model)


def _collect(tree, model, grads):
    """Walk (state, model, grad) in parallel; accumulate grads of tied leaves."""
    items: dict = {}
    order: list = []

    def walk(s, x, g):
        if isinstance(s, Leaf):
            if s.frozen:
                return
            if g is None:
                if not getattr(s.rule, "collective", False):
                    return
                # a rank without a gradient for this leaf still takes part in the
                # collective (the plan comes from the state tree), contributing zeros
                g = torch.zeros_like(_as_tensor(x))
            x_t, g_t = _as_tensor(x), _as_tensor(g)
            if id(s) in items:
                leaf, xx, gg = items[id(s)]
                items[id(s)] = (leaf, xx, gg + g_t)  # tied parameter: sum contributions
            else:
                items[id(s)] = (s, x_t, g_t)
                order.append(id(s))
            return
        if s is None:
            return
        if isinstance(x, torch.nn.Module):
            named = dict(x.named_parameters())
            gd = g if isinstance(g, dict) else {n: p.grad for n, p in named.items()}
            for n, p in named.items():
                walk(s.get(n), p, gd.get(n))
            return
        nd = node_def(s)
        if nd is None:
            return
        sc, _ = nd[0](s)
        xc, _ = node_def(x)[0](x) if node_def(x) is not None else ([x] * len(sc), None)
        if g is None or node_def(g) is None:
            gc = [g] * len(sc)
        else:
            gc, _ = node_def(g)[0](g)
        for a, b, c in zip(sc, xc, gc):
            walk(a, b, c)

    walk(tree, model, grads)
    return [items[k] for k in order]


def update_(tree: Any, model: Any, grads: Any):
    """In-place update (``Optimisers.update!``). Returns ``(tree, model)``."""
    items = _collect(tree, model, grads)
    # group consecutive leaves by rule object so each rule sees one batch
    by_rule: dict = {}
    for it in items:
        by_rule.setdefault(id(it[0].rule), (it[0].rule, []))[1].append(it)
    for rule, batch in by_rule.values():
        dxs = rule.apply_batch(batch)
        for (leaf, x, _), d in zip(batch, dxs):
            if d is None:
                continue
            with torch.no_grad():
                x.sub_(d.to(x.dtype) if d.dtype != x.dtype else d)
    return tree, model


update_inplace = update_


def _copy_tree(t):
    def cp(x):
        if isinstance(x, torch.Tensor):
            return x.detach().clone()
        if isinstance(x, np.ndarray):
            return x.copy()
        return x
    return fmap(cp, t)


def update(tree: Any, model: Any, grads: Any):
    """Out-of-place update (``Optimisers.update``): state and model are copied first."""
    if isinstance(model, torch.nn.Module):
        model = copy.deepcopy(model)
        if not isinstance(grads, dict):
            grads = {n: p.grad for n, p in model.named_parameters()}
    else:
        model = _copy_tree(model)
    tree = _copy_leaves(tree)
    return update_(tree, model, grads)


def _copy_leaves(tree):
    cache: dict = {}

    def walk(s):
        if isinstance(s, Leaf):
            if id(s) not in cache:
                cache[id(s)] = Leaf(s.rule, _copy_tree(s.state), s.frozen)
            return cache[id(s)]
        nd = node_def(s)
        if nd is None:
            return s
        ch, aux = nd[0](s)
        return nd[1](aux, [walk(c) for c in ch])

    return walk(tree)


def freeze_(tree):
    for l in _leaves_of(tree):
        l.frozen = True
    return tree


def thaw_(tree):
    for l in _leaves_of(tree):
        l.frozen = False
    return tree


def adjust_(tree, eta: float | None = None, **kw):
    """Change hyperparameters of every rule in ``tree`` (``Optimisers.adjust!``)."""
    seen = set()
    for l in _leaves_of(tree):
        r = l.rule
        if id(r) in seen:
            continue
        seen.add(id(r))
        _adjust_rule(r, eta, kw)
    return tree


def _adjust_rule(r, eta, kw):
    if isinstance(r, OptimiserChain):
        for o in r.opts:
            _adjust_rule(o, eta, kw)
        return
    inner = getattr(r, "optimizer", None)
    if inner is not None:
        _adjust_rule(inner, eta, kw)
        return
    if eta is not None and hasattr(r, "eta"):
        r.eta = eta
    for k, v in kw.items():
        if hasattr(r, k):
            setattr(r, k, v)


def _leaves_of(tree):
    out: list = []
    seen: set = set()

    def walk(s):
        if isinstance(s, Leaf):
            if id(s) not in seen:
                seen.add(id(s))
                out.append(s)
            return
        nd = node_def(s)
        if nd is None:
            return
        for c in nd[0](s)[0]:
            walk(c)

    walk(tree)
    return out


__all__ = [
    "AbstractRule", "Leaf", "Descent", "Momentum", "Nesterov", "RMSProp", "AdaGrad", "Adam", "AdamW",
    "WeightDecay", "ClipGrad", "ClipNorm", "OptimiserChain", "OptimizerChain", "setup", "update", "update_",
    "update_inplace", "freeze_", "thaw_", "adjust_",
]
