"""Deep Equilibrium Model (Bai et al. 2019; the FastDEQ.jl example of the reference README).

``z* = f(z*, x)`` is found by Anderson-accelerated fixed-point iteration
without building a graph; the backward pass uses implicit differentiation:
the incoming gradient ``g`` is replaced by the solution of
``u = J_f(z*)^T u + g`` (solved by fixed-point iteration on
vector-Jacobian products), so memory is independent of the solver depth.

For the DDP layer this is the "irregular gradient tree" config: parameters of
the implicit layer receive gradients only through the adjoint solve, and the
number of solver iterations differs across ranks, which must not desync
collectives (bucket plans are built from the parameter list, not from
gradient arrival order).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import anderson as AO
from ..ops.fused_block import conv3x3, conv3x3_supported
from ..ops.batchnorm import FusedBatchNorm2d, GradLink
from ..ops.groupnorm import FusedGroupNorm, fp32_affine_cache, skip_param_grads
from ..ops.groupnorm import native_ok as gn_native_ok

# Convergence tests read a device value back LAG iterations late (FLUXMPI_DEQ_CHECK_LAG,
# default 2 on the GPU): the host never drains the queue, so the GPU always has LAG
# iterations of work in flight while the host waits for an old flag; the price is at most
# LAG extra (harmless, still-contracting) iterations after convergence. 0 = test every
# iteration synchronously (the round-1 behaviour: ~11 % of the step idle, profiles/r1_deq_s63).
CHECK_LAG = int(os.environ.get("FLUXMPI_DEQ_CHECK_LAG", "2"))
# FLUXMPI_DEQ_MANUAL_VJP=0: the adjoint's VJPs through autograd.grad (A/B runs)
MANUAL_VJP = os.environ.get("FLUXMPI_DEQ_MANUAL_VJP", "1") != "0"


class LaggedFlags:
    """Scalars produced on the device, read on the host ``lag`` pushes later without a sync
    of the whole queue: each value goes to pinned memory by an async copy with an event."""

    def __init__(self, lag: int, n: int):
        self.lag = lag
        self.buf = torch.zeros(max(n, 1), dtype=torch.float32, pin_memory=True)
        self.pending: list = []

    def push(self, i: int, value: torch.Tensor) -> None:
        self.buf[i:i + 1].copy_(value.reshape(1).float(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((i, ev))

    def pop_ready(self):
        """``(i, value)`` of the push made ``lag`` pushes ago (blocks on its event only), else None."""
        if len(self.pending) <= self.lag:
            return None
        i, ev = self.pending.pop(0)
        ev.synchronize()
        return i, float(self.buf[i])


def anderson(f, x0, m=5, lam=1e-4, max_iter=30, tol=1e-4, beta=1.0, check_lag: int | None = None):
    """Anderson acceleration for ``x = f(x)`` over batch-flattened tensors. Returns (x, iters, rel_residual).

    The history Gram matrix and the mix run as single-pass HIP kernels on the GPU
    (``fluxmpi_amd.ops.anderson``). The residual of iterate k is read off the diagonal of
    the Gram matrix computed at the top of iteration k + 1 (same value, no extra pass).

    ``check_lag`` (GPU; default :data:`CHECK_LAG`): the residual test of iterate k is read
    back ``check_lag`` iterations later (:class:`LaggedFlags`), so the host never waits for
    the queue to drain; the returned iterate is then the newest one and the residual a 0-d
    device tensor when the solve ends without convergence. 0: test synchronously (float).
    """
    from ..ops import anderson as AO

    bsz = x0.shape[0]
    shape, dt = x0.shape, x0.dtype
    d = x0[0].numel()
    # the solver history and the small (m+1)^2 systems are kept in fp32 whatever the model
    # dtype (bf16 has no batched LU, and 8-bit mantissas would stall the extrapolation)
    X = torch.zeros(bsz, m, d, dtype=torch.float32, device=x0.device)
    Fv = torch.zeros_like(X)
    Gs = torch.zeros_like(X)

    # flatten in MEMORY order: a channels_last iterate stays channels_last through f (views,
    # no layout copies), which is the layout the fused NHWC GroupNorm kernels take
    cl = x0.dim() == 4 and x0.is_contiguous(memory_format=torch.channels_last) and not x0.is_contiguous()

    def flat(t):
        return (t.permute(0, 2, 3, 1) if cl else t).reshape(bsz, -1)

    def unflat(v):
        if cl:
            n_, c_, h_, w_ = shape
            return v.reshape(n_, h_, w_, c_).permute(0, 3, 1, 2)
        return v.reshape(shape)

    def fx(v):  # f in the model dtype; the fp32 history slot assignment is the (one) cast
        return flat(f(unflat(v.contiguous()).to(dt)))

    X[:, 0], Fv[:, 0] = flat(x0), fx(flat(x0))
    X[:, 1], Fv[:, 1] = Fv[:, 0], fx(Fv[:, 0])
    lag = (CHECK_LAG if check_lag is None else int(check_lag)) if x0.is_cuda else 0
    flags = LaggedFlags(lag, max_iter) if lag > 0 else None
    res = float("inf")
    k, converged = 1, False
    for k in range(2, max_iter):
        n = min(k, m)
        last = (k - 1) % m
        # stored G = F - X: only the row(s) changed since the last Gram are recomputed; on the GPU
        # the residual and the (n+1)^2 solve are ONE launch after the Gram pass (AO.gram_solve)
        alpha, res_t = AO.gram_solve(X, Fv, n, last, Gs, (0, 1) if k == 2 else (last,), lam, k > 2)
        if k > 2:  # residual of the iterate produced by the previous iteration
            if flags is None:
                res = float(res_t)
                if res < tol:
                    k, converged = k - 1, True
                    break
            else:
                flags.push(k, res_t)
                hit = flags.pop_ready()
                if hit is not None and hit[1] < tol:
                    # iterate hit[0] - 1 converged; the newest one (iteration k - 1) is at least as good
                    res, k, converged = hit[1], k - 1, True
                    break
        z = AO.mix(X, Fv, alpha, k % m, beta, dt)
        Fv[:, k % m] = fx(z)
    if not converged:
        s = k % m
        res_t = (Fv[:, s] - X[:, s]).norm() / (1e-5 + Fv[:, s].norm())
        res = res_t if flags is not None else float(res_t)
    return unflat(X[:, k % m].contiguous()).to(dt), k, res


class DEQFixedPoint(nn.Module):
    def __init__(self, f: nn.Module, max_iter=30, tol=1e-4, bwd_iter=30, bwd_tol=1e-4, check_lag: int | None = None):
        super().__init__()
        self.f = f
        self.max_iter, self.tol, self.bwd_iter, self.bwd_tol = max_iter, tol, bwd_iter, bwd_tol
        self.check_lag = check_lag
        self.last_iters = 0
        self.last_bwd_iters = 0

    def forward(self, x):
        # the cell's GroupNorm parameters cast to fp32 once for the ~30 calls below
        with fp32_affine_cache(self.f):
            return self._forward(x)

    def _forward(self, x):
        # the solver's ~30 evaluations by direct kernel calls when the cell allows (no autograd
        # Function objects per call: the DEQ step is host-bound, profiles/rd3h_ab_deq.jsonl)
        raw = MANUAL_VJP and hasattr(self.f, "manual_ok") and self.f.manual_ok(x)
        fz = (lambda z: self.f.forward_raw(z, x)) if raw else (lambda z: self.f(z, x))
        with torch.no_grad():
            z, self.last_iters, _ = anderson(fz, torch.zeros_like(x), max_iter=self.max_iter,
                                             tol=self.tol, check_lag=self.check_lag)
        z = self.f(z, x)  # one differentiable step re-engages autograd at z*
        if not torch.is_grad_enabled():
            return z
        z0 = z.clone().detach().requires_grad_()
        manual = MANUAL_VJP and hasattr(self.f, "manual_ok") and self.f.manual_ok(z0)
        if manual:
            # the adjoint's VJPs by direct kernel calls on the saved forward state (no autograd
            # graph for f0, no engine overhead per iteration)
            _, state = self.f.forward_state(z0.detach(), x.detach())
            vjp = lambda u: self.f.vjp(state, u)  # noqa: E731
        else:
            f0 = self.f(z0, x)

            def vjp(u):
                with skip_param_grads():  # VJPs w.r.t. z only: no GroupNorm dw/db reductions
                    return torch.autograd.grad(f0, z0, u, retain_graph=True)[0]

        def backward_hook(grad):
            lag = (CHECK_LAG if self.check_lag is None else int(self.check_lag)) if grad.is_cuda else 0
            flags = LaggedFlags(lag, self.bwd_iter) if lag > 0 else None
            thresh = self.bwd_tol * (grad.norm() + 1e-9)  # device scalar, computed once
            thresh2 = thresh * thresh
            if z0.dim() == 4 and z0.is_contiguous(memory_format=torch.channels_last):
                # the incoming gradient (from the BatchNorm after the DEQ) may be NCHW: one layout
                # copy here instead of one per iteration in the cell's NHWC GroupNorm backward
                grad = grad.contiguous(memory_format=torch.channels_last)
            u = grad
            it = 0
            for it in range(self.bwd_iter):  # u = J^T u + grad
                v = vjp(u)
                # u_new = v + grad and |u_new - u|^2 in one pass (ops/anderson.adjoint_step)
                u_new, ss = AO.adjoint_step(v, grad, u)
                done = ss <= thresh2
                u = u_new
                if flags is None:
                    if bool(done):
                        break
                else:  # lagged test: a converged adjoint keeps contracting for <= lag more steps
                    flags.push(it, done)
                    hit = flags.pop_ready()
                    if hit is not None and hit[1] > 0.5:
                        break
            self.last_bwd_iters = it + 1
            return u

        if z.requires_grad:
            z.register_hook(backward_hook)
        return z


class ResidualCell(nn.Module):
    """f(z, x) = GN(relu(z + GN(conv2(GN(relu(conv1 z))) + x)))  (MDEQ-style cell)."""

    def __init__(self, ch=48, groups=8):
        super().__init__()
        self.conv1 = nn.Conv2d(ch, ch, 3, padding=1, bias=False)
        self.conv2 = nn.Conv2d(ch, ch, 3, padding=1, bias=False)
        # FusedGroupNorm: GN(relu(x + add)) in one NHWC pass on the GPU (ops/groupnorm.py)
        self.n1, self.n2, self.n3 = (FusedGroupNorm(groups, ch) for _ in range(3))
        for c in (self.conv1, self.conv2):
            nn.init.normal_(c.weight, 0, 0.01)

    def _conv(self, conv, t, link=None):
        # bf16 channels_last on the GPU: the implicit-GEMM MFMA kernels (ops/fused_block.conv3x3,
        # per-shape choice against MIOpen for the forward, input and weight gradients)
        if conv3x3_supported(t, conv):
            return conv3x3(t, conv.weight, gradlink=link)
        return conv(t)

    def manual_ok(self, z) -> bool:
        """The fused GPU path that :meth:`forward_state` / :meth:`vjp` drive directly."""
        return (conv3x3_supported(z, self.conv1) and conv3x3_supported(z, self.conv2)
                and gn_native_ok(z, self.n1.num_groups) and gn_native_ok(z, self.n3.num_groups)
                and gn_native_ok(z, self.n2.num_groups))

    @torch.no_grad()
    def forward_raw(self, z, x):
        """``f(z, x)`` by direct kernel calls (no autograd Functions): the solver iterations."""
        return self.forward_state(z, x, keep=False)

    @torch.no_grad()
    def forward_state(self, z, x, keep: bool = True):
        """``f(z, x)`` without autograd, keeping what :meth:`vjp` needs (GPU fused path)."""
        from ..ops.fused_block import conv3x3_fwd_raw
        from ..ops.groupnorm import gn_fwd_raw
        c1 = conv3x3_fwd_raw(z, self.conv1.weight)
        a1, h1, m1, r1, w1 = gn_fwd_raw(c1, None, self.n1.weight, self.n1.bias, self.n1.num_groups, self.n1.eps, True)
        c2 = conv3x3_fwd_raw(a1, self.conv2.weight)
        a2, h2, m2, r2, w2 = gn_fwd_raw(c2, x, self.n2.weight, self.n2.bias, self.n2.num_groups, self.n2.eps, False)
        out, h3, m3, r3, w3 = gn_fwd_raw(z, a2, self.n3.weight, self.n3.bias, self.n3.num_groups, self.n3.eps, True)
        if not keep:
            return out
        return out, (tuple(z.shape), (h1, m1, r1, w1), (h2, m2, r2, w2), (h3, m3, r3, w3))

    @torch.no_grad()
    def vjp(self, state, u):
        """``J_f(z)^T u`` from :meth:`forward_state`'s state by direct kernel calls — the adjoint
        solve's per-iteration VJP without the autograd engine (~6 launches per iteration)."""
        from ..ops.fused_block import conv3x3_dgrad_raw
        from ..ops.groupnorm import gn_bwd_raw
        zs, (h1, m1, r1, w1), (h2, m2, r2, w2), (h3, m3, r3, w3) = state
        d3, _ = gn_bwd_raw(u, h3, m3, r3, w3, self.n3.num_groups, True)    # d(z + a2), ReLU-masked
        d2, _ = gn_bwd_raw(d3, h2, m2, r2, w2, self.n2.num_groups, False)  # d conv2 output (x is constant)
        da1 = conv3x3_dgrad_raw(d2, self.conv2.weight, h1.shape)
        d1, _ = gn_bwd_raw(da1, h1, m1, r1, w1, self.n1.num_groups, True)  # d conv1 output
        return conv3x3_dgrad_raw(d1, self.conv1.weight, zs, residual=d3)   # + n3's direct path to z

    def forward(self, z, x):
        # z feeds conv1 and n3's add: n3's backward hands its gradient of z to conv1's dgrad
        # epilogue (GradLink) instead of autograd summing the two with an add kernel
        link = None
        if torch.is_grad_enabled() and z.requires_grad and conv3x3_supported(z, self.conv1) and \
                gn_native_ok(z, self.n3.num_groups):
            link = GradLink()
        y = self.n1(self._conv(self.conv1, z, link), relu=True)
        return self.n3(z, add=self.n2(self._conv(self.conv2, y), add=x), relu=True, link=link)


class DEQClassifier(nn.Module):
    def __init__(self, cin=1, ch=48, num_classes=10, **solver):
        super().__init__()
        self.inj = nn.Conv2d(cin, ch, 3, padding=1, bias=False)
        # our NHWC BatchNorm kernels (ops/batchnorm.py) instead of MIOpen's (nn.BatchNorm2d API,
        # same parameters / state dict)
        self.inj_norm = FusedBatchNorm2d(ch)
        self.deq = DEQFixedPoint(ResidualCell(ch), **solver)
        self.out_norm = FusedBatchNorm2d(ch)
        self.head = nn.Linear(ch * 4 * 4, num_classes)

    def forward(self, x):
        x = self.inj_norm(self.inj(x))
        z = self.out_norm(self.deq(x))
        z = F.adaptive_avg_pool2d(z, 4).flatten(1)
        return self.head(z)


def deq_mnist(num_classes=10, **kw) -> DEQClassifier:
    return DEQClassifier(1, 48, num_classes, **kw)
