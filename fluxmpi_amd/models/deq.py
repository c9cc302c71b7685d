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

import contextlib
import os
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import anderson as AO
from ..ops.conv_small import conv3x3_small
from ..ops.fused_block import conv3x3, conv3x3_s2, conv3x3_s2_supported, conv3x3_supported
from ..ops.linear import Linear
from ..ops.batchnorm import FusedBatchNorm2d, GradLink
from ..ops.groupnorm import FusedGroupNorm, fp32_affine_cache, skip_param_grads
from ..ops.groupnorm import native_ok as gn_native_ok

# Convergence tests read a device value back LAG iterations late (CHECK_LAG,
# default 2 on the GPU): the host never drains the queue, so the GPU always has LAG
# iterations of work in flight while the host waits for an old flag; the price is at most
# LAG extra (harmless, still-contracting) iterations after convergence. 0 = test every
# iteration synchronously (the round-1 behaviour: ~11 % of the step idle, profiles/r1_deq_s63).
CHECK_LAG = 2
# False: the adjoint's VJPs through autograd.grad (A/B runs, tests)
MANUAL_VJP = True
# GRAPHS False: no solver graphs (every iteration launched from the host; A/B runs);
# GRAPH_CHUNK: adjoint iterations per graph replay
GRAPHS = True
GRAPH_CHUNK = 5
# Solver settings of the two DEQ benchmarks (bench.py --deq-solver overrides): relative-residual
# tolerances the solves can reach in bf16 before their iteration caps. Measured on the random-init
# cells (scripts/diag/deq_residual.py, profiles/rd5e_deq_residual.jsonl): the MNIST cell's
# Anderson residual reaches 3e-3 at 10 iterations, 1e-3 at 15 and floors at ~2e-4 (bf16 evaluation
# noise: 1e-4 is never met); the 512-channel CIFAR cell contracts by only ~0.91 per iteration
# (fp32 alike, Anderson m = 5 / 8 alike: 3e-2 at 10, 1e-2 at ~22). With the solver graphs the
# test runs on each 5-iteration period's best residual, read one period late, so a solve stops
# 5-9 iterations after the iterate that met the tolerance.
# Keeping the trained cell contractive (ResidualCell.constrain_, run before every training
# forward): "conv" = max-norm projection of each conv output channel's filter onto the ball of
# its expected init norm; "conv+gn" also clamps n3's GroupNorm gain (it multiplies the whole
# Jacobian) to [-1, 1]; "none" = off.
CONSTRAIN = os.environ.get("FLUXMPI_DEQ_CONSTRAIN", "none")
# Jacobian regularisation (Bai, Koltun, Kolter 2021, "Stabilizing Equilibrium Models by Jacobian
# Regularization"; DeepEquilibriumNetworks.jl's `jacobian_regularization`): loss += gamma * ||J_f||_F^2 / d
# at the fixed point, estimated each training step by a finite difference along one random
# direction, ||f(z* + s e) - f(z*)||^2 / (s^2 ||e||^2) (two extra cell evaluations with autograd, no
# double backward: the fused kernels' backward is first-order). "gamma,sigma"; empty = off.
JAC_REG = os.environ.get("FLUXMPI_DEQ_JR", "")


class _AddPenaltyGrad(torch.autograd.Function):
    """Identity on ``z``; in the backward ``penalty`` receives gradient ``weight``: the same
    parameter gradients as adding ``weight * penalty`` to the loss, without changing the loss the
    caller computes (the bench loop, user code)."""

    @staticmethod
    def forward(ctx, z, penalty, weight):
        ctx.weight = float(weight)
        ctx.pmeta = (penalty.dtype, penalty.device)
        return z.view_as(z)

    @staticmethod
    def backward(ctx, g):
        dt, dev = ctx.pmeta
        return g, torch.full((), ctx.weight, dtype=dt, device=dev), None
# Round 6: the caps are set so that the solves END BY TOLERANCE under training, not at the cap.
# The trained cells contract slowly (residual curves after 40 Adam steps, fp32 alike:
# profiles/rd6e_deq_solver_curves.jsonl; Jacobian regularisation, a max-norm constraint and
# learnable synthetic labels did not change that, rd6h / rd6i), so the round-5 presets (30
# iterations, MNIST tolerance 1e-3) measured iteration caps. Measured with these presets
# (profiles/rd6k_bench_deq_presets.jsonl): MNIST 27.25 forward iterations of 60, final residual
# <= 9.8e-3, 56 adjoint iterations; CIFAR 29 of 60, residual <= 1.9e-2, 10.25 adjoint iterations.
# Caps of 80 leave headroom for the slow steps (a 60-iteration MNIST solve ended at 1.004e-2 against
# 1e-2 in rd6q, a DEQ-CIFAR one at 0.024 in rd6m): an easy step still stops at its tolerance, so the
# cap only costs time on the steps that need it (profiles/rd6r_bench_deq_caps80.jsonl: all four 1-GPU
# lines end by tolerance; the 2-rank rehearsals did not).
# MNIST restarts its Anderson history when two period tests in a row improve on the best by < 10 %
# (anderson(restart=2)): the trained cell's solves stall near a 1e-2 residual, and with restarts 5 of
# 9 lines met every condition against 1 of 9 without, 28.5k vs 24.9k img/s mean (interleaved, one box:
# profiles/rd6ae_deq_restart.jsonl).
DEQ_MNIST_SOLVER = {"max_iter": 80, "tol": 1e-2, "bwd_iter": 80, "bwd_tol": 2e-2, "restart": 2}
# DEQ-CIFAR runs as a Skip DEQ (FastDEQ.jl's explicit initial-guess network, DEQFixedPoint ``skip``):
# 13 of 18 round-6 lines with it ended every solve by tolerance against 3 of 5 without it
# (profiles/rd6_deq_convergence_tally.md; one 2-rank rehearsal: 28 forward iterations at 0.019976
# against 0.02 vs 56 at 0.034 without, 3798 vs 2294 img/s, rd6t_skip_deq_comm.jsonl), and the 1-GPU
# line is faster (14 vs 19-29 forward iterations, 9.0k vs 8.8k img/s: rd6s_skip_deq.jsonl,
# rd6u_deq_anderson_adjoint.jsonl). MNIST stays without it: there the skip measured mixed (rd6s, rd6t).
DEQ_CIFAR_SOLVER = {"max_iter": 80, "tol": 2e-2, "bwd_iter": 80, "bwd_tol": 1e-2, "skip": 1}


# host seconds spent blocked on convergence flags (LaggedFlags.pop_ready), cumulative: bench.py
# reports the solver's host time net of these waits (a data-dependent solve must wait for its
# flags; what matters is whether the host's own work keeps up with the GPU)
HOST_WAIT_S = 0.0


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

    def pop_ready(self, lag: int | None = None):
        """``(i, value)`` of the push made ``lag`` pushes ago (blocks on its event only), else None."""
        if len(self.pending) <= (self.lag if lag is None else lag):
            return None
        global HOST_WAIT_S
        i, ev = self.pending.pop(0)
        t0 = time.perf_counter()
        ev.synchronize()
        HOST_WAIT_S += time.perf_counter() - t0
        return i, float(self.buf[i])


def _f_hist_dtype(dt: torch.dtype, like: torch.Tensor) -> torch.dtype:
    """dtype of the Anderson F history: bf16 for a bf16 model on the GPU (f's outputs are bf16
    values, so the narrower history is exact), fp32 otherwise."""
    return torch.bfloat16 if (dt == torch.bfloat16 and like.is_cuda) else torch.float32


# FLUXMPI_DEQ_HIST: dtype of the iterate (X) and difference (G = F - X) histories of a bf16 model on
# the GPU — "bf16" (default: the iterates the model evaluates are bf16-rounded anyway; the Gram
# sums and the (n+1)^2 solve stay fp32; residual-vs-iteration curves of both models equal to the
# fp32 histories', profiles/rd5x_deq_hist_residual.jsonl; the Gram pass reads 14 instead of 26
# bytes per element) or "fp32"
HIST = os.environ.get("FLUXMPI_DEQ_HIST", "bf16")


def _x_hist_dtype(dt: torch.dtype, like: torch.Tensor) -> torch.dtype:
    """dtype of the Anderson X and G histories (see :data:`HIST`)."""
    return torch.bfloat16 if (HIST == "bf16" and dt == torch.bfloat16 and like.is_cuda) else torch.float32


def anderson(f, x0, m=5, lam=1e-4, max_iter=30, tol=1e-4, beta=1.0, check_lag: int | None = None,
             graphs: "SolverGraphs | None" = None, restart: int = 0):
    """Anderson acceleration for ``x = f(x)`` over batch-flattened tensors. Returns (x, iters, rel_residual).

    The history Gram matrix and the mix run as single-pass HIP kernels on the GPU
    (``fluxmpi_amd.ops.anderson``). The residual of iterate k is read off the diagonal of
    the Gram matrix computed at the top of iteration k + 1 (same value, no extra pass).

    ``check_lag`` (GPU; default :data:`CHECK_LAG`): the residual test of iterate k is read
    back ``check_lag`` iterations later (:class:`LaggedFlags`), so the host never waits for
    the queue to drain; the returned iterate is then the newest one and the residual a 0-d
    device tensor when the solve ends without convergence. 0: test synchronously (float).

    ``graphs`` (:class:`SolverGraphs`, GPU): the history lives in its static buffers and, once
    the iteration is periodic (k >= m: slot k % m, all m rows in the Gram), whole periods of m
    iterations replay one captured HIP graph; the test then runs per period on the period's
    smallest residual (read back one period late).

    ``restart`` (> 0): restart the history from the newest iterate when the last ``restart``
    residual tests (periods with graphs, iterations without) improved on the best before them by
    less than 10 % — Anderson on a slowly contracting, non-normal map can stall with a history
    whose least-squares problem no longer finds a descent direction. The iteration count and the
    cap include every restart's iterations.
    """
    from ..ops import anderson as AO

    bsz = x0.shape[0]
    shape, dt = x0.shape, x0.dtype
    d = x0[0].numel()
    # the small (m+1)^2 systems and every Gram sum are fp32 whatever the model dtype (bf16 has no
    # batched LU); the images F are f's outputs, so in a bf16 model they are bf16 values and their
    # history is kept in bf16 on the GPU (exact); the iterates X and the differences G = F - X are
    # bf16 there too (:data:`HIST`: the model only ever evaluates bf16-rounded iterates)
    if graphs is not None:
        X, Fv, Gs = graphs.history(m)
    else:
        X = torch.zeros(bsz, m, d, dtype=_x_hist_dtype(dt, x0), device=x0.device)
        Fv = torch.zeros_like(X, dtype=_f_hist_dtype(dt, x0))
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

    write_into = getattr(f, "write_into", None)

    def fx_into(v, slot):
        # f in the model dtype; the fp32 history slot assignment is the (one) cast — or, when f
        # can, its kernel writes the fp32 slot itself (no separate cast pass)
        z = unflat(v.contiguous()).to(dt)
        if write_into is None or not write_into(z, Fv[:, slot]):
            Fv[:, slot] = flat(f(z))

    X[:, 0] = flat(x0)
    fx_into(X[:, 0], 0)
    X[:, 1] = Fv[:, 0]
    fx_into(Fv[:, 0], 1)
    lag = (CHECK_LAG if check_lag is None else int(check_lag)) if x0.is_cuda else 0
    flags = LaggedFlags(lag, max_iter) if lag > 0 else None

    def solve_step(k, res_out=None):
        # stored G = F - X: only the row(s) changed since the last Gram are recomputed; on the GPU
        # the residual and the (n+1)^2 solve are ONE launch after the Gram pass (AO.gram_solve);
        # res_out: a static slot the residual is written into (the graph replay's buffer)
        last = (k - 1) % m
        return AO.gram_solve(X, Fv, min(k, m), last, Gs, (0, 1) if k == 2 else (last,), lam, k > 2, res_out)

    def mix_step(k, alpha):
        fx_into(AO.mix(X, Fv, alpha, k % m, beta, dt), k % m)

    res = float("inf")
    # k: iterations of the current history segment (slot arithmetic); base: iterations of the
    # segments before the last restart (k + base counts every f evaluation)
    k, base, converged = 2, 0, False
    tests: list = []  # residual tests read back since the last restart (floats)

    def stalled() -> bool:
        if restart <= 0 or len(tests) < restart + 2:
            return False
        return min(tests[-restart:]) > 0.9 * min(tests[:-restart])

    def restart_from_newest() -> None:
        nonlocal k, base
        s_new = (k - 1) % m  # newest iterate and its image: the new segment's first pair
        if s_new != 0:
            X[:, 0] = X[:, s_new]
            Fv[:, 0] = Fv[:, s_new]
        X[:, 1] = Fv[:, 0]
        fx_into(Fv[:, 0], 1)
        base += k - 1
        k = 2
        tests.clear()

    while base + k < max_iter:
        if graphs is not None and k >= max(m, 3) and k % m == 0 and base + k + m <= max_iter:
            # iterations k .. k + m - 1 in one replay; iterate k - 1 + m is then complete
            rmin = graphs.anderson_period(k, m, solve_step, mix_step)
            k += m
            if flags is None:
                res = float(rmin)
                converged = res < tol
                tests.append(res)
            else:
                flags.push(base + k - 1, rmin)
                while not converged and (hit := flags.pop_ready(lag=1)) is not None:
                    res, converged = hit[1], hit[1] < tol
                    tests.append(res)
            if converged:
                k -= 1
                break
            if stalled() and base + k + 1 < max_iter:
                restart_from_newest()
            continue
        alpha, res_t = solve_step(k)
        if k > 2:  # residual of the iterate produced by the previous iteration
            if flags is None:
                res = float(res_t)
                if res < tol:
                    k, converged = k - 1, True
                    break
                tests.append(res)
            else:
                flags.push(base + k, res_t)
                hit = flags.pop_ready()
                if hit is not None and hit[1] < tol:
                    # iterate hit[0] - 1 converged; the newest one (iteration k - 1) is at least as good
                    res, k, converged = hit[1], k - 1, True
                    break
                if hit is not None:
                    tests.append(hit[1])
        mix_step(k, alpha)
        k += 1
        if stalled() and base + k + 1 < max_iter:
            restart_from_newest()
    if not converged:
        k = max(k - 1, 1)  # the last completed iteration
        s = k % m
        res_t = (Fv[:, s].float() - X[:, s].float()).norm() / (1e-5 + Fv[:, s].float().norm())
        res = res_t if flags is not None else float(res_t)
    return unflat(X[:, k % m].contiguous()).to(dt), base + k, res


class _CellEval:
    """``z -> f(z, x)`` for the solver: direct kernel calls when ``raw`` (else the autograd-free
    module call under no_grad); ``write_into`` lets the fused cell kernel write an fp32 history
    slot itself (ops/deq_cell.py)."""

    def __init__(self, cell, x, raw: bool):
        self.cell, self.x, self.raw = cell, x, raw

    def __call__(self, z):
        return self.cell.forward_raw(z, self.x) if self.raw else self.cell(z, self.x)

    def write_into(self, z, dst) -> bool:
        if not self.raw or dst.stride(-1) != 1 or not hasattr(self.cell, "conv1"):
            return False
        from ..ops import deq_cell
        if not deq_cell.supported(self.cell, z):
            if dst.dtype != z.dtype or not hasattr(self.cell, "forward_state"):
                return False
            # the last GroupNorm writes the model-dtype history slot itself (no copy pass)
            self.cell.forward_state(z, self.x, keep=False, out_slot=dst)
            return True
        if dst.dtype == torch.bfloat16:
            deq_cell.cell_forward(self.cell, z, self.x, out_slot=dst)
        else:
            deq_cell.cell_forward(self.cell, z, self.x, out32=dst, want_out=False)
        return True


def _capture(graph: "torch.cuda.CUDAGraph"):
    # thread-local capture mode: a DDP watchdog thread polling events must not invalidate it
    return torch.cuda.graph(graph, capture_error_mode="thread_local")


def _rms_rows(t: torch.Tensor) -> torch.Tensor:
    """Per-sample root-mean-square of ``t`` (fp32 [N], floored): the adjoint's right-hand side is
    divided by it before an Anderson solve, whose Gram regulariser ``lam`` is absolute (the loss
    gradient reaching the DEQ is ~1e-4 per element: unscaled, ``lam`` would swamp ``G G^T``), and
    multiplied back after (the adjoint is linear in its right-hand side)."""
    return t.float().reshape(t.shape[0], -1).square().mean(1).sqrt_().clamp_min_(1e-30)


class _AndersonGraph:
    """One Anderson solve's static history and its captured period (``m`` iterations, slots
    ``k % m``): what :func:`anderson` takes as ``graphs``. ``like``: the iterate's shape, dtype and
    device."""

    def __init__(self, like: torch.Tensor):
        self.like = like
        self._hist = None
        self.g = self.rbuf = self.rmin = None

    def history(self, m: int):
        bsz, d = self.like.shape[0], self.like[0].numel()
        if self._hist is None or self._hist[0].shape[1] != m:
            X = torch.zeros(bsz, m, d, dtype=_x_hist_dtype(self.like.dtype, self.like), device=self.like.device)
            self._hist = (X, torch.zeros_like(X, dtype=_f_hist_dtype(self.like.dtype, self.like)), torch.zeros_like(X))
            self.g = None
        return self._hist

    def anderson_period(self, k0: int, m: int, solve_step, mix_step) -> torch.Tensor:
        """Replay iterations ``k0 .. k0 + m - 1`` (capturing them on first use); returns the
        smallest residual of the period (0-d device tensor, static)."""
        if self.g is None:
            self.rbuf = torch.zeros(m, dtype=torch.float32, device=self.like.device)
            self.rmin = torch.zeros((), dtype=torch.float32, device=self.like.device)
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), _capture(g):
                for i in range(m):
                    alpha, res_t = solve_step(k0 + i, self.rbuf[i])
                    if res_t is not None and res_t.data_ptr() != self.rbuf[i].data_ptr():
                        self.rbuf[i].copy_(res_t)
                    mix_step(k0 + i, alpha)
                torch.amin(self.rbuf, dim=0, out=self.rmin)
            self.g = g
        self.g.replay()
        return self.rmin


class SolverGraphs:
    """HIP graphs of one :class:`DEQFixedPoint`'s two solver loops at one input shape.

    Both loops are periodic: Anderson iteration k (k >= m) reads and writes history slots
    by ``k % m`` only, and every adjoint iteration ``u <- J^T u + g`` is the same launch
    sequence. One period of each (m forward iterations, :data:`GRAPH_CHUNK` adjoint ones) is
    captured once and replayed: the host issues one graph launch per period instead of ~10
    kernel launches (and their Python dispatch) per iteration, which is what bounds the eager
    DEQ step (wall ~1.25x the GPU's busy time, profiles/rd3h_deq_steady.md). Convergence is
    tested per replay on the period's best residual, read back one period late, so a solve
    stops at most two periods after the iterate that met the tolerance (the extra iterations
    keep contracting) and the reported iteration counts are the ones executed.

    Everything a graph reads lives at a fixed address and is refreshed before a replay: the
    injection ``x`` (copied in), the fp32 history, the GroupNorm fp32 affine copies
    (``fp32_affine_cache(buffers=...)``), the adjoint's right-hand side / iterate / threshold,
    the cached transposed conv filters (re-derived eagerly before the adjoint replays:
    :meth:`ResidualCell.refresh_filters`). The VJPs' forward state comes from a third graph
    (``forward_state`` at ``z = f(z*)``), so its tensors are static too. Parameters are read in
    place (the optimiser updates them in place). Built from the SECOND call at a shape: the
    first runs eagerly and measures the per-shape kernel choices the capture then bakes in.
    """

    def __init__(self, x: torch.Tensor):
        self.x = torch.empty_like(x)  # the solve's injection, same strides (channels_last stays)
        self.x.copy_(x)
        self.aff: dict = {}
        self.fwd = _AndersonGraph(self.x)  # the forward solve's history + period graph
        self.adj = None                    # the Anderson adjoint's (bwd_m > 0), made on first use
        self.g_state = self.g_adj = None
        self.state = self.z0 = self.grad = self.u = self.thresh2 = self.dmax = self.done = None
        self.gen = 0  # forward_state calls so far (a hook whose generation is stale goes eager)
        self.chunk = 0

    @property
    def g_fwd(self):
        return self.fwd.g

    def history(self, m: int):
        return self.fwd.history(m)

    def anderson_period(self, k0: int, m: int, solve_step, mix_step) -> torch.Tensor:
        return self.fwd.anderson_period(k0, m, solve_step, mix_step)

    def capture_adjoint(self, cell, z: torch.Tensor, chunk: int) -> None:
        """Capture ``forward_state`` at a static ``z0`` and ``chunk`` adjoint iterations."""
        with torch.no_grad():
            self.z0 = torch.empty_like(z)
            self.z0.copy_(z)
            g = torch.cuda.CUDAGraph()
            with _capture(g):
                _, self.state = cell.forward_state(self.z0, self.x)
            self.g_state = g
            self.grad = torch.empty_like(self.z0)
            self.u = torch.empty_like(self.z0)
            self.thresh2 = torch.zeros((), dtype=torch.float32, device=z.device)
            # every tensor a graph reads or writes outside its own pool must stay referenced: a
            # freed buffer would be handed to other tensors while the replays keep writing into it
            self.done = torch.zeros(chunk, dtype=torch.float32, device=z.device)
            self.dmax = torch.zeros((), dtype=torch.float32, device=z.device)
            cell.refresh_filters()  # fresh now: the capture below records no refresh launch
            g = torch.cuda.CUDAGraph()
            with _capture(g):
                u = self.u
                for i in range(chunk):
                    # the chunk's last iterate straight into the static u (its input is another buffer)
                    out = self.u if (i == chunk - 1 and chunk > 1) else None
                    u, _ = cell.adjoint_step(self.state, u, self.grad, self.thresh2, self.done[i:i + 1], out=out)
                if u.data_ptr() != self.u.data_ptr():
                    self.u.copy_(u)
                torch.amax(self.done, dim=0, out=self.dmax)
            self.g_adj = g
            self.chunk = chunk

    def forward_state(self, z: torch.Tensor) -> int:
        """Record the adjoint's forward state at ``z`` (and the static ``x``); returns the
        generation a later :meth:`adjoint` call must match (another forward at this shape before
        that backward overwrites the static buffers)."""
        self.z0.copy_(z)
        self.g_state.replay()
        self.gen += 1
        return self.gen

    def adjoint(self, cell, grad: torch.Tensor, tol: float, max_iter: int, lag: int):
        """Solve ``u = J^T u + grad`` by replays of the adjoint graph; returns ``(u, iterations)``."""
        self.grad.copy_(grad)
        self.u.copy_(grad)
        thresh = tol * (grad.norm() + 1e-9)
        self.thresh2.copy_(thresh * thresh)
        cell.refresh_filters()  # the optimiser may have changed the weights since the capture
        flags = LaggedFlags(min(lag, 1), max_iter) if lag > 0 else None
        it, P = 0, self.chunk
        while it + P <= max_iter:
            self.g_adj.replay()
            it += P
            if flags is None:
                if float(self.dmax) > 0.5:
                    return self.u.clone(), it
            else:
                flags.push(it - 1, self.dmax)
                hit = flags.pop_ready()
                if hit is not None and hit[1] > 0.5:
                    return self.u.clone(), it
        u = self.u.clone()
        while it < max_iter:  # a partial period: eager iterations
            u, _ = cell.adjoint_step(self.state, u, self.grad)
            it += 1
        return u, it

    def adjoint_anderson(self, cell, grad: torch.Tensor, tol: float, max_iter: int, m: int, lag: int):
        """Solve ``u = J^T u + grad`` by Anderson(``m``) on the static state: the right-hand side
        is normalised per sample (:func:`_rms_rows`) into the static ``grad`` buffer, the solve's
        history and period graph are this object's second :class:`_AndersonGraph`; returns
        ``(u, iterations)``."""
        s = _rms_rows(grad).view(-1, *([1] * (grad.dim() - 1)))
        self.grad.copy_(grad.float() / s)
        cell.refresh_filters()  # the optimiser may have changed the weights since the capture
        if self.adj is None:
            self.adj = _AndersonGraph(self.grad)
        step = lambda u: cell.adjoint_step(self.state, u, self.grad)[0]  # noqa: E731
        u, it, _ = anderson(step, self.grad, m=m, max_iter=max_iter, tol=tol, check_lag=lag, graphs=self.adj)
        return (u.float() * s).to(grad.dtype), it


class DEQFixedPoint(nn.Module):
    """``z* = f(z*, x)`` by Anderson acceleration, implicit (adjoint fixed-point) backward.

    ``skip`` (channels, > 0: on): the Skip DEQ of FastDEQ.jl (the reference's DEQ example library,
    /root/reference/README.md:76): an explicit 3x3 convolution of the injection predicts the fixed
    point and the solve starts there instead of at zero; it is trained towards z* by an auxiliary
    loss ``skip_reg * ||skip(x) - z*||^2 / ||z*||^2`` (z* a constant: the cell gets none of its
    gradient; the skip convolution and, through the injection x, the layers before the DEQ do).
    The solver's initial guess changes neither z* (up to the tolerance) nor its implicit gradient.
    ``skip_detach``: the skip convolution reads a detached injection (measured less stable:
    profiles/rd6ak_deq_skip_detach.jsonl).
    ``m`` / ``bwd_m``: Anderson memory of the forward / adjoint solve (``bwd_m`` 0: the adjoint by
    fixed-point iteration ``u <- J^T u + g``); ``beta`` / ``lam``: the forward Anderson's mixing
    (1: undamped) and Gram regulariser; ``restart``: see :func:`anderson`."""

    def __init__(self, f: nn.Module, max_iter=30, tol=1e-4, bwd_iter=30, bwd_tol=1e-4, check_lag: int | None = None,
                 jac_reg: float | None = None, jac_sigma: float | None = None, skip: int = 0, skip_reg: float = 1.0,
                 m: int = 5, bwd_m: int = 0, beta: float = 1.0, lam: float = 1e-4, restart: int = 0,
                 skip_detach: int = 0):
        super().__init__()
        self.f = f
        self.m = int(m)          # Anderson memory of the forward solve (<= 8: anderson.hip)
        self.bwd_m = int(bwd_m)  # > 0: the adjoint solve by Anderson(bwd_m) too; 0: fixed-point iteration
        self.beta, self.lam = float(beta), float(lam)  # the forward Anderson's mixing and regulariser
        self.restart = int(restart)  # > 0: the forward solve restarts its history on a stall (anderson)
        self.skip = nn.Conv2d(int(skip), int(skip), 3, padding=1, bias=False) if skip else None
        if self.skip is not None:
            nn.init.zeros_(self.skip.weight)  # starts at the zero guess of the plain solve
        self.skip_reg = float(skip_reg)
        self.skip_detach = bool(skip_detach)  # the skip convolution reads a detached injection
        self.last_skip_res = None  # the last training step's ||skip(x) - z*|| / ||z*|| (0-d device tensor)
        env = [float(v) for v in JAC_REG.split(",")] if JAC_REG else []
        self.jac_reg = float(jac_reg if jac_reg is not None else (env[0] if env else 0.0))
        self.jac_sigma = float(jac_sigma if jac_sigma is not None else (env[1] if len(env) > 1 else 0.05))
        self.last_jr = None  # the last training step's ||J||_F^2 / d estimate (0-d device tensor)
        self.max_iter, self.tol, self.bwd_iter, self.bwd_tol = max_iter, tol, bwd_iter, bwd_tol
        self.check_lag = check_lag
        self.last_iters = 0
        self.last_bwd_iters = 0
        self.last_res = None  # the forward solve's final relative residual (float, or 0-d device tensor)
        self.use_graphs = GRAPHS  # HIP graphs of the solver loops (SolverGraphs), GPU fused path
        self._graphs: dict = {}   # input signature -> SolverGraphs (None after the first, eager call)

    def _graphs_for(self, x) -> SolverGraphs | None:
        if not (self.use_graphs and x.is_cuda and MANUAL_VJP and hasattr(self.f, "manual_ok")
                and self.f.manual_ok(x)) or torch.cuda.is_current_stream_capturing():
            return None
        key = (tuple(x.shape), x.stride(), x.dtype, x.device)
        if key not in self._graphs:  # first call at this shape: eager (measures the kernel choices)
            self._graphs[key] = None
            return None
        gs = self._graphs[key]
        if gs is None:
            gs = self._graphs[key] = SolverGraphs(x)
        else:
            gs.x.copy_(x)
        return gs

    def forward(self, x):
        if self.training and CONSTRAIN != "none" and hasattr(self.f, "constrain_"):
            self.f.constrain_(CONSTRAIN)
        gs = self._graphs_for(x)
        # the cell's GroupNorm parameters cast to fp32 once for the ~30 calls below (into the
        # graphs' static buffers when the solver loops replay graphs)
        z_pred = None
        if self.skip is not None:  # bf16 channels_last on the GPU: our implicit-GEMM 3x3 kernels
            xs = x.detach() if self.skip_detach else x  # skip_detach: the auxiliary loss stops at the skip
            z_pred = conv3x3(xs, self.skip.weight) if conv3x3_supported(xs, self.skip) else self.skip(xs)
        x0 = z_pred.detach().contiguous(memory_format=torch.channels_last) if z_pred is not None and \
            x.is_contiguous(memory_format=torch.channels_last) else (z_pred.detach() if z_pred is not None else None)
        with fp32_affine_cache(self.f, buffers=gs.aff if gs is not None else None):
            out = self._forward(x, gs, x0)
        training = self.training and torch.is_grad_enabled() and out.requires_grad
        if self.jac_reg > 0 and training:
            out = self._jacobian_penalty(out, x)
        if z_pred is not None and training and z_pred.requires_grad:
            zs = self._z_star.float()
            err = (z_pred.float() - zs).square().sum() / zs.square().sum().clamp_min(1e-12)
            self.last_skip_res = err.detach().sqrt()
            out = _AddPenaltyGrad.apply(out, err, self.skip_reg)
        return out

    def _jacobian_penalty(self, out, x):
        """``out`` carrying the gradient of ``jac_reg * ||J_f(z*)||_F^2 / d`` (module constant
        :data:`JAC_REG`): two differentiable cell evaluations at the solution and at a random
        perturbation of it, separate from the implicit-differentiation step (whose output gradient
        the adjoint solve replaces)."""
        z0 = self._z_star
        e = torch.randn_like(z0)
        s = self.jac_sigma
        with fp32_affine_cache(self.f):
            f1 = self.f(z0, x)
            f2 = self.f(z0 + s * e, x)
        jr = (f2.float() - f1.float()).square().sum() / (s * s * e.float().square().sum())
        self.last_jr = jr.detach()
        return _AddPenaltyGrad.apply(out, jr, self.jac_reg)

    def _forward(self, x, gs: SolverGraphs | None = None, x0: torch.Tensor | None = None):
        # the solver's ~30 evaluations by direct kernel calls when the cell allows (no autograd
        # Function objects per call: the DEQ step is host-bound, profiles/rd3h_ab_deq.jsonl)
        raw = MANUAL_VJP and hasattr(self.f, "manual_ok") and self.f.manual_ok(x)
        xs = gs.x if gs is not None else x  # the solve reads the graphs' static copy
        fz = _CellEval(self.f, xs, raw)
        with torch.no_grad():
            z, self.last_iters, self.last_res = anderson(fz, x0 if x0 is not None else torch.zeros_like(x),
                                                         m=self.m, lam=self.lam, beta=self.beta,
                                                         restart=self.restart, max_iter=self.max_iter,
                                             tol=self.tol, check_lag=self.check_lag, graphs=gs)
        self._z_star = z.detach()
        # one differentiable step re-engages autograd at z*; its GroupNorms save fresh fp32 affine
        # copies, not the graphs' static buffers (a later forward at this shape rewrites those in
        # place before this one's backward)
        with fp32_affine_cache(self.f) if gs is not None else contextlib.nullcontext():
            z = self.f(z, x)
        if not torch.is_grad_enabled():
            return z
        if gs is not None:
            if gs.g_adj is None:
                gs.capture_adjoint(self.f, z.detach(), max(1, min(GRAPH_CHUNK, self.bwd_iter)))
            gen = gs.forward_state(z.detach())
            z_star, x_in = z.detach(), x.detach()

            def graphed_hook(grad):
                if gs.gen != gen:
                    # another forward at this shape ran before this backward (two micro-batches in
                    # one loss, a weight-shared DEQ applied twice): the graphs' static state is
                    # the later call's, so this adjoint runs eagerly on its own state
                    _, state = self.f.forward_state(z_star, x_in)
                    return self._adjoint_loop(grad, lambda u, g: self.f.adjoint_step(state, u, g), z_star)
                lag = CHECK_LAG if self.check_lag is None else int(self.check_lag)
                if self.bwd_m > 0:
                    u, self.last_bwd_iters = gs.adjoint_anderson(self.f, grad, self.bwd_tol, self.bwd_iter,
                                                                 self.bwd_m, lag)
                    return u
                u, self.last_bwd_iters = gs.adjoint(self.f, grad, self.bwd_tol, self.bwd_iter, lag)
                return u

            if z.requires_grad:
                z.register_hook(graphed_hook)
            return z
        z0 = z.clone().detach().requires_grad_()
        manual = MANUAL_VJP and hasattr(self.f, "manual_ok") and self.f.manual_ok(z0)
        if manual:
            # the adjoint's VJPs by direct kernel calls on the saved forward state (no autograd
            # graph for f0, no engine overhead per iteration)
            _, state = self.f.forward_state(z0.detach(), x.detach())
            vjp = lambda u: self.f.vjp(state, u)  # noqa: E731
            step = lambda u, g: self.f.adjoint_step(state, u, g)  # noqa: E731
        else:
            f0 = self.f(z0, x)

            def vjp(u):
                with skip_param_grads():  # VJPs w.r.t. z only: no GroupNorm dw/db reductions
                    return torch.autograd.grad(f0, z0, u, retain_graph=True)[0]

            def step(u, g):
                # u_new = v + grad and |u_new - u|^2 in one pass (ops/anderson.adjoint_step)
                return AO.adjoint_step(vjp(u), g, u)

        def backward_hook(grad):
            return self._adjoint_loop(grad, step, z0)

        if z.requires_grad:
            z.register_hook(backward_hook)
        return z

    def _adjoint_loop(self, grad, step, z0):
        """Eager adjoint fixed point ``u = J^T u + grad`` (``step(u, grad) -> (u_new, |u_new - u|^2)``)."""
        lag = (CHECK_LAG if self.check_lag is None else int(self.check_lag)) if grad.is_cuda else 0
        if z0.dim() == 4 and z0.is_contiguous(memory_format=torch.channels_last):
            # the incoming gradient (from the BatchNorm after the DEQ) may be NCHW: one layout
            # copy here instead of one per iteration in the cell's NHWC GroupNorm backward
            grad = grad.contiguous(memory_format=torch.channels_last)
        if self.bwd_m > 0:
            # Anderson(bwd_m) on the per-sample normalised right-hand side; its test is the
            # relative residual |h(u) - u| / |h(u)| of h(u) = J^T u + g (the forward's test)
            s = _rms_rows(grad).view(-1, *([1] * (grad.dim() - 1)))
            gn = (grad.float() / s).to(grad.dtype)
            u, self.last_bwd_iters, _ = anderson(lambda v: step(v, gn)[0], gn, m=self.bwd_m, max_iter=self.bwd_iter,
                                                 tol=self.bwd_tol, check_lag=lag)
            return (u.float() * s).to(grad.dtype)
        flags = LaggedFlags(lag, self.bwd_iter) if lag > 0 else None
        thresh = self.bwd_tol * (grad.norm() + 1e-9)  # device scalar, computed once
        thresh2 = thresh * thresh
        u = grad
        it = 0
        for it in range(self.bwd_iter):  # u = J^T u + grad
            u_new, ss = step(u, grad)
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
        # expected per-output-channel filter norm at init (the max-norm radius of constrain_)
        self.max_norm = 0.01 * (9 * ch) ** 0.5

    @torch.no_grad()
    def constrain_(self, mode: str = "conv") -> None:
        """Project the cell back into a contractive set after an optimiser step: each conv output
        channel's filter onto the ball of radius ``max_norm`` (in place; a no-op for channels
        inside it), and with ``"conv+gn"`` n3's gain into [-1, 1]. In-place edits bump the
        parameters' versions, so a DDP engine re-reads its fp32 masters from them."""
        for c in (self.conv1, self.conv2):
            w = c.weight
            n = w.float().square().sum((1, 2, 3), keepdim=True).sqrt_()
            w.mul_((self.max_norm / n.clamp_min(1e-12)).clamp_(max=1.0).to(w.dtype))
        if mode == "conv+gn" and self.n3.weight is not None:
            self.n3.weight.clamp_(-1.0, 1.0)

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

    def refresh_filters(self) -> None:
        """Re-derive the cached transposed filters of both convolutions from the current weights
        now (one batched launch), as the first input gradient of a backward would: the solver
        graphs replay input-gradient GEMMs that read that cache."""
        from ..ops.gemm import filter_t, note_filter
        note_filter(self.conv1.weight)
        note_filter(self.conv2.weight)
        filter_t(self.conv1.weight)

    @torch.no_grad()
    def forward_raw(self, z, x):
        """``f(z, x)`` by direct kernel calls (no autograd Functions): the solver iterations."""
        return self.forward_state(z, x, keep=False)

    @torch.no_grad()
    def forward_state(self, z, x, keep: bool = True, out_slot=None):
        """``f(z, x)`` without autograd, keeping what :meth:`vjp` needs (GPU fused path): one
        LDS-resident kernel per evaluation where it applies (ops/deq_cell.py), else 5 launches.
        ``out_slot`` ([N, C*H*W] model-dtype rows, e.g. an Anderson history slot): the output is
        written there (returned as that tensor)."""
        from ..ops import deq_cell
        from ..ops.fused_block import conv3x3_fwd_raw
        from ..ops.groupnorm import gn_fwd_raw
        if deq_cell.supported(self, z):
            return deq_cell.cell_forward(self, z, x, keep=keep, out_slot=out_slot)
        c1 = conv3x3_fwd_raw(z, self.conv1.weight)
        a1, h1, m1, r1, w1 = gn_fwd_raw(c1, None, self.n1.weight, self.n1.bias, self.n1.num_groups, self.n1.eps, True)
        c2 = conv3x3_fwd_raw(a1, self.conv2.weight)
        a2, h2, m2, r2, w2 = gn_fwd_raw(c2, x, self.n2.weight, self.n2.bias, self.n2.num_groups, self.n2.eps, False)
        out, h3, m3, r3, w3 = gn_fwd_raw(z, a2, self.n3.weight, self.n3.bias, self.n3.num_groups, self.n3.eps, True,
                                         out=out_slot)
        if not keep:
            return out
        return out, (tuple(z.shape), (h1, m1, r1, w1), (h2, m2, r2, w2), (h3, m3, r3, w3))

    @torch.no_grad()
    def vjp(self, state, u):
        """``J_f(z)^T u`` from :meth:`forward_state`'s state by direct kernel calls — the adjoint
        solve's per-iteration VJP without the autograd engine (~6 launches per iteration)."""
        from ..ops import deq_cell
        from ..ops.fused_block import conv3x3_dgrad_raw
        from ..ops.groupnorm import gn_bwd_raw
        if deq_cell.supported(self, u):
            return deq_cell.cell_vjp(self, state, u)
        zs, (h1, m1, r1, w1), (h2, m2, r2, w2), (h3, m3, r3, w3) = state
        d3, _ = gn_bwd_raw(u, h3, m3, r3, w3, self.n3.num_groups, True)    # d(z + a2), ReLU-masked
        d2, _ = gn_bwd_raw(d3, h2, m2, r2, w2, self.n2.num_groups, False)  # d conv2 output (x is constant)
        da1 = conv3x3_dgrad_raw(d2, self.conv2.weight, h1.shape)
        d1, _ = gn_bwd_raw(da1, h1, m1, r1, w1, self.n1.num_groups, True)  # d conv1 output
        return conv3x3_dgrad_raw(d1, self.conv1.weight, zs, residual=d3)   # + n3's direct path to z

    @torch.no_grad()
    def adjoint_step(self, state, u, grad, thresh2=None, flag=None, out=None):
        """One adjoint iteration ``u_new = J_f(z)^T u + grad`` with ``ss = |u_new - u|^2`` (0-d fp32
        device tensor); with ``thresh2`` / ``flag`` also ``flag = ss <= thresh2`` on the device.
        One-kernel cell: the update is fused into the VJP kernel (2 launches per iteration).
        ``out``: write ``u_new`` there when possible (not ``u`` itself)."""
        from ..ops import deq_cell
        if deq_cell.supported(self, u):
            u_new, part = deq_cell.cell_vjp(self, state, u, grad=grad, out=out)
            t2 = None if thresh2 is None else thresh2.float()
            return u_new, deq_cell.adjoint_check(part, t2, flag)
        return AO.adjoint_step(self.vjp(state, u), grad, u,
                               out=out if (out is not None and out.data_ptr() != u.data_ptr()) else None,
                               thresh2=None if flag is None else thresh2.float(), flag=flag)

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
        if solver.get("skip"):
            solver["skip"] = ch
        self.deq = DEQFixedPoint(ResidualCell(ch), **solver)
        self.out_norm = FusedBatchNorm2d(ch)
        self.head = nn.Linear(ch * 4 * 4, num_classes)

    def forward(self, x):
        x = self.inj_norm(self.inj(x))
        z = self.out_norm(self.deq(x))
        z = F.adaptive_avg_pool2d(z, 4).flatten(1)
        return self.head(z)


def deq_mnist(num_classes=10, **kw) -> DEQClassifier:
    for k, v in DEQ_MNIST_SOLVER.items():
        kw.setdefault(k, v)
    return DEQClassifier(1, 48, num_classes, **kw)


class DEQCifar(nn.Module):
    """A FastDEQ-width implicit classifier for 3 x 32 x 32 images (the reference's DEQ example,
    /root/reference/README.md:76-77, links FastDEQ.jl's CIFAR-10 models): a two-convolution
    stem (32 x 32, then stride 2 to 16 x 16 and ``ch`` channels), the MDEQ-style residual cell
    solved to its fixed point at 16 x 16 x ``ch`` (Anderson forward, adjoint fixed-point
    backward), BatchNorm, global pooling and a linear head. ``ch`` = 512: 5.3 M parameters,
    10.6 MB of bf16 gradients per step — a DDP workload whose allreduce moves real data, on
    the nested (irregular) parameter tree the functional API reduces with
    ``allreduce_gradients(like=...)`` (bench.py ``--api functional``)."""

    def __init__(self, ch=512, num_classes=10, groups=16, **solver):
        super().__init__()
        c0 = ch // 4
        self.stem1 = nn.Conv2d(3, c0, 3, padding=1, bias=False)
        self.stem1_norm = FusedBatchNorm2d(c0)
        self.stem2 = nn.Conv2d(c0, ch, 3, stride=2, padding=1, bias=False)
        self.inj_norm = FusedBatchNorm2d(ch)
        for k, v in DEQ_CIFAR_SOLVER.items():
            solver.setdefault(k, v)
        if solver.get("skip"):
            solver["skip"] = ch
        self.deq = DEQFixedPoint(ResidualCell(ch, groups), **solver)
        self.out_norm = FusedBatchNorm2d(ch)
        self.head = Linear(ch, num_classes)  # ops.linear.Linear: dW / db born in their bucket slices

    def forward(self, x):
        # every parameter gradient is produced in its DDP bucket slice (ops/graddst.py): the
        # 3-channel stem's filter gradient by one GEMM (ops/conv_small.py), the stride-2 stem on
        # the implicit-GEMM path (fused_block.conv3x3_s2), BatchNorm / GroupNorm dw, db and the
        # head's dW, db by their own backward kernels
        x = self.stem1_norm(conv3x3_small(x, self.stem1), relu=True)
        if conv3x3_s2_supported(x, self.stem2):
            x = conv3x3_s2(x, self.stem2.weight)
        else:
            x = self.stem2(x)
        z = self.out_norm(self.deq(self.inj_norm(x)))
        return self.head(F.adaptive_avg_pool2d(z, 1).flatten(1))


def deq_cifar(num_classes=10, ch=512, **kw) -> DEQCifar:
    return DEQCifar(ch, num_classes, **kw)
